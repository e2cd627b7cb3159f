"""ctypes binding of libkfmi.so (include/kf.h).

This is the only place the shared library is touched.  It fails loudly: a missing or
unloadable library raises ``KFError`` — there is no CPU fallback anywhere in ``kfmi``.
"""
from __future__ import annotations

import ctypes
import glob
import hashlib
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# KFMI_LIB selects an alternative build (e.g. an occupancy variant); relative to the cwd.
LIB_PATH = os.path.abspath(os.environ.get('KFMI_LIB') or os.path.join(HERE, 'libkfmi.so'))
HEADER = os.path.normpath(os.path.join(HERE, '..', '..', 'include', 'kf.h'))
CSRC = os.path.normpath(os.path.join(HERE, '..', 'csrc'))

KF_OK = 0
KF_EINVAL = -1
KF_EHIP = -2
KF_ENOTSPD = -3
KF_ENODEV = -4
KF_ENOMEM = -5
KF_F32 = 0
KF_F64 = 1
KF_MODEL_CV2 = 2
KF_MODEL_CV3 = 3
KF_MODEL_REF15 = 15
KF_MODEL_REF8 = 8
KF_EVENT_GPS = 0
KF_EVENT_IMU = 1
KF_EVENT_PREDICT = 2
KF_EVENT_NONE = 255
KF_INGEST_GPS_ALTITUDE = 1
KF_DT_FULL = 0
KF_DT_MONOTONE = 1
KF_DT_RAW = 2

KF_OPT_PREDICT = 1
KF_OPT_CV_KERNEL = 2
KF_OPT_BLOCKS_PER_CU = 3
KF_OPT_EVENTS_KERNEL = 4
KF_OPT_STREAM = 5
KF_OPT_STREAM_CHUNKS = 6
KF_OPT_STREAM_FINAL = 7
KF_OPT_START_THREADS = 8
KF_OPT_SEARCH_KERNEL = 9
KF_OPT_SEARCH_PM = 10
KF_OPT_SCHED_KERNEL = 11
KF_OPT_SCHED_GROUP = 12
KF_OPT_SCHED_ORDER = 13
KF_OPT_SCHED_REC_TIME = 14
KF_OPT_SEARCH_HEAD = 15
KF_OPT_AXIS_SYM = 16
KF_OPT_SEARCH_END = 17
KF_OPT_SEARCH_PAIR = 18
KF_OPT_COUNT = 19

_ERRNAMES = {KF_EINVAL: 'KF_EINVAL', KF_EHIP: 'KF_EHIP', KF_ENOTSPD: 'KF_ENOTSPD',
             KF_ENODEV: 'KF_ENODEV', KF_ENOMEM: 'KF_ENOMEM'}


class KFError(RuntimeError):
    """Non-zero return from libkfmi (or the library itself is unavailable)."""

    def __init__(self, code, msg):
        self.code = code
        super().__init__(f'{_ERRNAMES.get(code, code)}: {msg}')


class kf_params(ctypes.Structure):
    _fields_ = [('q_pos', ctypes.c_double), ('q_vel', ctypes.c_double),
                ('r', ctypes.c_double * 9), ('p0_pos', ctypes.c_double), ('p0_vel', ctypes.c_double),
                ('ref_q', ctypes.c_double * 15), ('ref_r_imu', ctypes.c_double * 15),
                ('ref_r_gps', ctypes.c_double * 3), ('ref_p0', ctypes.c_double * 15)]


class kf_ingest_info(ctypes.Structure):
    _fields_ = [('n_events', ctypes.c_int64), ('n_fixes', ctypes.c_int64), ('n_imu', ctypes.c_int64),
                ('first_valid_index', ctypes.c_int64), ('origin_row', ctypes.c_int64),
                ('gyro_bias', ctypes.c_double * 3), ('accel_bias', ctypes.c_double * 3),
                ('utm_origin', ctypes.c_double * 2)]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_d = ctypes.c_double

# name -> (restype, argtypes); must match include/kf.h exactly (tests/test_capi.py checks).
SIGNATURES = {
    'kf_version': (ctypes.c_char_p, []),
    'kf_set_option': (_i, [_vp, _i, _i64]),
    'kf_get_option': (_i, [_vp, _i, ctypes.POINTER(_i64)]),
    'kf_last_error': (ctypes.c_char_p, []),
    'kf_default_params': (_i, [_i, ctypes.POINTER(kf_params)]),
    'kf_device_count': (_i, [ctypes.POINTER(_i)]),
    'kf_init': (_i, [_i]),
    'kf_alloc': (_i, [ctypes.POINTER(_vp), _i, _i64, _i, ctypes.POINTER(kf_params)]),
    'kf_free': (_i, [_vp]),
    'kf_release_retired': (_i, [_vp, ctypes.POINTER(_i64)]),
    'kf_dims': (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i),
                     ctypes.POINTER(_i64), ctypes.POINTER(_i)]),
    'kf_reset': (_i, [_vp, _vp, _vp]),
    'kf_set_state': (_i, [_vp, _vp, _vp, _i, _vp]),
    'kf_get_state': (_i, [_vp, _vp, _vp, _i, _vp]),
    'kf_get_status': (_i, [_vp, _vp, _i, _vp]),
    'kf_predict': (_i, [_vp, _d, _vp, _vp, _vp, _vp]),
    'kf_update': (_i, [_vp, _vp, _vp, _vp, _vp]),
    'kf_run': (_i, [_vp, _i, _d, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp]),
    'kf_synth': (_i, [_vp, ctypes.c_uint64, _i64, _i, _d, _i, _vp, _vp, _vp, _vp]),
    'kf_run_events': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _d, _vp]),
    'kf_run_events_seq': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _d, _vp]),
    'kf_run_stream': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    'kf_stream_check': (_i, [_vp, _vp, _vp]),
    'kf_eval_combos': (_i, [_vp, _i, _vp, _vp, _d, _d, _i, ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    'kf_search_combos': (_i, [_vp, _i, _vp, _vp, _d, _d, _d, _i, _i, _i, ctypes.c_uint64,
                              ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_i), _vp, _vp, _vp]),
    'kf_search_plan': (_i, [_vp, _i, _vp, _i, ctypes.c_uint64, _i, _vp]),
    'kf_search_info': (_i, [_vp, _vp]),
    'kf_score_candidates': (_i, [_vp, _i, _vp, _i, _vp, _vp, _vp]),
    'kf_score_rows': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp]),
    'kf_run_scheduled': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _vp, _d, _vp, _vp, _vp, _vp, _vp]),
    'kf_run_scheduled_rec': (_i, [_vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _d, _vp, _vp, _vp, _vp, _vp]),
    'kf_run_scheduled_random': (_i, [_vp, _i, _vp, _vp, _vp, _i, _vp, _vp, _d, _vp, _i, _vp, _vp, _vp, _vp, _vp,
                                     _vp]),
    'kf_sched_random_picks': (_i, [_vp, _i, _vp, _vp, _vp, _vp, _d, _vp, _i, _vp, _vp, _vp, _vp, _vp]),
    'kf_csv_shape': (_i, [ctypes.c_char_p, _i, ctypes.POINTER(_i64), ctypes.POINTER(_i)]),
    'kf_csv_read': (_i, [ctypes.c_char_p, _i, _i, _vp, _i64, _i64]),
    'kf_ingest': (_i, [_vp, _i64, _i64, _vp, _i64, _i64, _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                       ctypes.POINTER(kf_ingest_info), _vp]),
    'kf_quat_to_euler': (_i, [_i64, _vp, _i64, _vp, _vp]),
    'kf_events_dt': (_i, [_i64, _vp, _vp, _d, _i, _vp, _vp, _vp]),
    'kf_events_select': (_i, [_i64, _vp, _vp, _vp, _i, _vp, _vp, _vp, ctypes.POINTER(_i64), _vp]),
}

_lib = None


def header_functions(path=HEADER):
    """Names of every function include/kf.h declares."""
    text = open(path).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(kf_\w+)\s*\(', text)))


def source_hash():
    """SHA-256 (16 hex) of the sources in this tree that libkfmi.so is built from, in the
    Makefile's order (HASHED): csrc/*.cpp, *.h, *.hip sorted by name, then include/kf.h.  None
    when the sources are not here (an installed package): the library's origin is then unknown."""
    files = sorted(p for ext in ('cpp', 'h', 'hip') for p in glob.glob(os.path.join(CSRC, '*.' + ext)))
    if not files or not os.path.exists(HEADER):
        return None
    h = hashlib.sha256()
    try:
        for p in files + [HEADER]:
            with open(p, 'rb') as f:
                h.update(f.read())
    except OSError:
        return None
    return h.hexdigest()[:16]


def library_hash(handle):
    v = handle.kf_version().decode()
    return v.rsplit('src:', 1)[1] if 'src:' in v else None


def lib():
    """Load libkfmi.so once and bind every entry point; raise KFError if it is missing or was
    built from other sources than this tree's (a stale build would test and time old code)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KFError(KF_ENODEV, f'{LIB_PATH} not built: run `make -C sensorfusion-kalmanfilter_amd` '
                                 f'or __graft_entry__.build() (no CPU fallback exists)')
    try:
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the host
        raise KFError(KF_ENODEV, f'cannot load {LIB_PATH}: {e}') from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if os.environ.get('KFMI_ALLOW_FOREIGN_LIB') != '1':
        built, tree = library_hash(handle), source_hash()
        if tree is None:
            raise KFError(KF_ENODEV, f'{LIB_PATH}: the sources it must match (csrc/, include/kf.h) are not in '
                                     f'this tree; KFMI_ALLOW_FOREIGN_LIB=1 loads it unchecked')
        if built != tree:
            raise KFError(KF_ENODEV, f'{LIB_PATH} was built from sources {built}, this tree is {tree}: rebuild '
                                     f'(make -C sensorfusion-kalmanfilter_amd); KFMI_ALLOW_FOREIGN_LIB=1 loads it '
                                     f'anyway (A/B of another revision only)')
    _lib = handle
    return _lib


def build_info():
    """Provenance of the loaded library, for the bench line."""
    L = lib()
    built, tree = library_hash(L), source_hash()
    return {'lib': os.path.relpath(LIB_PATH, os.path.join(HERE, '..', '..')), 'version': L.kf_version().decode(),
            'src_hash': built, 'tree_hash': tree, 'match': built == tree}


def last_error():
    return lib().kf_last_error().decode()


def check(rc):
    if rc != KF_OK:
        raise KFError(rc, last_error())
    return rc
