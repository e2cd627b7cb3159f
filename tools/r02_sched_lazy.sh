#!/bin/bash
# GPU: scheduled-filter tests + the sched bench row (lazy wave-convergent apply).
#   gpurun -- bash tools/r02_sched_lazy.sh TAG
set -o pipefail
TAG=${1:-sched_lazy}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "sched or Sched" tests/test_gpu_ref15.py tests/test_gpu_compat.py > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python bench.py --config sched --no-cpu-baseline > gpurun_out/$TAG/bench_sched.json 2>&1 || { tail -20 gpurun_out/$TAG/bench_sched.json; exit 1; }
python -c "
import json
for l in open('gpurun_out/$TAG/bench_sched.json'):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); print('sched', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'])"
