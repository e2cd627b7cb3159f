"""kf_set_option / kf_get_option on a live handle (include/kf.h KF_OPT_*): every value the header
documents is accepted and read back, every other value and an unknown option id is KF_EINVAL and
leaves the option unchanged, and a new handle starts with every option 0 — needs an MI355X."""
import pytest

import kfmi
from kfmi import _lib
from kfmi.engine import OPTIONS

pytestmark = pytest.mark.gpu

# include/kf.h: the values each option takes besides 0
VALID = {
    'predict': [1], 'cv_kernel': [1, 2, 4, 8], 'blocks_per_cu': [2, 5, 8], 'events_kernel': [1, 2, 3, 4],
    'stream': [1], 'stream_chunks': [2, 8192, 1 << 24], 'stream_final': [1], 'start_threads': [1, 64, 256],
    'search_kernel': [1, 2], 'search_pm': [1], 'sched_kernel': [1, 2, 3, 4], 'sched_group': [1, 4],
    'sched_order': [1], 'sched_rec_time': [1], 'search_head': [1], 'axis_sym': [1], 'search_end': [1],
    'search_pair': [1, 2, 3, 1024, 1 << 22],
}
INVALID = {
    'predict': [2, -1], 'cv_kernel': [3, 16], 'blocks_per_cu': [1, 9], 'events_kernel': [5],
    'stream': [2], 'stream_chunks': [1, (1 << 24) + 1], 'stream_final': [2], 'start_threads': [257, -1],
    'search_kernel': [3], 'search_pm': [2], 'sched_kernel': [5, -1], 'sched_group': [2, 3], 'sched_order': [2],
    'sched_rec_time': [2, -1], 'search_head': [2], 'axis_sym': [2], 'search_end': [2, -1],
    'search_pair': [4, 1023, -1],
}


def test_every_option_documented_and_validated():
    assert set(VALID) == set(OPTIONS) == set(INVALID)
    kf = kfmi.BatchedKF('ref15', 64, 'f64')
    try:
        for name in OPTIONS:
            assert kf.get_option(name) == 0, name
        for name, values in VALID.items():
            for v in values:
                kf.set_option(name, v)
                assert kf.get_option(name) == v, (name, v)
            for v in INVALID[name]:
                with pytest.raises(_lib.KFError):
                    kf.set_option(name, v)
                assert kf.get_option(name) == values[-1], (name, v)  # unchanged
            kf.set_option(name, 0)
        L = _lib.lib()
        assert L.kf_set_option(kf.handle, _lib.KF_OPT_COUNT, 0) == _lib.KF_EINVAL
        assert L.kf_set_option(kf.handle, 0, 0) == _lib.KF_EINVAL
    finally:
        kf.close()
