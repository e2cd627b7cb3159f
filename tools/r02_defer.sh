#!/bin/bash
# GPU: the deferred-predict tests + the per-step call shape of configs 3, 4, 2, 5 (deferred vs eager).
#   gpurun -- bash tools/r02_defer.sh
set -o pipefail
mkdir -p gpurun_out/defer
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_deferred_predict.py tests/test_gpu_parity.py > gpurun_out/defer/pytest.log 2>&1 || { tail -40 gpurun_out/defer/pytest.log; exit 1; }
tail -3 gpurun_out/defer/pytest.log
for c in 3 4 2 5; do timeout -k 10 300 python bench.py --config $c --per-step --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/defer/perstep_$c.json 2>&1 || exit 1; done
python - <<'P'
import json
for c in '3425':
    for l in open(f'gpurun_out/defer/perstep_{c}.json'):
        if l.startswith('{"metric"'):
            d=json.loads(l)['per_step_api']; print(c, 'deferred %.3g %.4f ms' % (d['value'], d['ms_per_step']), '| eager %.3g %.4f ms' % (d['eager']['value'], d['eager']['ms_per_step']), ('| run_t1 %.3g %.4f ms' % (d['run_t1']['value'], d['run_t1']['ms_per_step'])) if 'run_t1' in d else '')
P
