"""The C ABI library loads and exports what include/kf.h declares (no GPU needed).

Only non-compute entry points are called here; on a host without a GPU they must fail
cleanly (KF_ENODEV), never fall back to a CPU path.
"""
import ctypes
import os

import pytest

import kfmi
from kfmi import _lib


def test_library_present_and_loads():
    assert os.path.exists(_lib.LIB_PATH), 'libkfmi.so not built (run __graft_entry__.build())'
    L = _lib.lib()
    assert L.kf_version().decode().startswith('kfmi')


def test_every_header_function_is_exported_and_bound():
    names = _lib.header_functions()
    assert len(names) >= 15
    L = _lib.lib()
    for n in names:
        assert hasattr(L, n), f'{n} declared in include/kf.h but not exported'
    # the ctypes signature table covers exactly the header
    assert sorted(_lib.SIGNATURES) == names


def test_binding_arity_matches_header_prototypes():
    """Each ctypes argtypes list has as many entries as the C prototype has parameters."""
    import re
    text = re.sub(r'/\*.*?\*/', '', open(_lib.HEADER).read(), flags=re.S)
    protos = dict(re.findall(r'\b(kf_\w+)\s*\(([^;{]*?)\)\s*;', text))
    assert sorted(protos) == sorted(_lib.SIGNATURES)
    for name, params in protos.items():
        params = ' '.join(params.split())
        n = 0 if params in ('', 'void') else params.count(',') + 1
        assert len(_lib.SIGNATURES[name][1]) == n, (name, params)


def test_integration_guide_binds_every_header_function():
    """INTEGRATION.md's reference-side ctypes stubs cover every entry point include/kf.h
    declares (the maintainer's binding stays in step with the header)."""
    import re
    guide = open(os.path.join(os.path.dirname(_lib.HEADER), '..', 'INTEGRATION.md')).read()
    documented = set(re.findall(r'lib\.(kf_\w+)\.(?:argtypes|restype)', guide))
    missing = sorted(set(_lib.header_functions()) - documented)
    assert not missing, f'INTEGRATION.md has no ctypes stub for {missing}'


def test_header_constants_match_binding():
    text = open(_lib.HEADER).read()
    for name in ('KF_OK', 'KF_EINVAL', 'KF_EHIP', 'KF_ENOTSPD', 'KF_ENODEV', 'KF_ENOMEM',
                 'KF_F32', 'KF_F64', 'KF_MODEL_CV2', 'KF_MODEL_CV3', 'KF_MODEL_REF15', 'KF_MODEL_REF8',
                 'KF_EVENT_GPS', 'KF_EVENT_IMU', 'KF_EVENT_PREDICT', 'KF_EVENT_NONE'):
        import re
        m = re.search(rf'#define {name}\s+\(?(-?\d+)\)?', text)
        assert m, name
        assert int(m.group(1)) == getattr(_lib, name), name


def test_default_params_are_reference_constants():
    p = kfmi.default_params('cv3')
    assert (p.q_pos, p.q_vel) == (5.0, 1.0)             # kf_workers.py:521,523
    assert list(p.r) == [3, 0, 0, 0, 3, 0, 0, 0, 3]     # kf_workers.py:583
    assert (p.p0_pos, p.p0_vel) == (1e4, 1e3)           # kf_workers.py:651
    p2 = kfmi.default_params('cv2')
    assert list(p2.r)[:4] == [3, 0, 0, 3]
    assert (p2.p0_pos, p2.p0_vel) == (1000.0, 100.0)    # hw5_2.py:317-326
    L = _lib.lib()
    assert L.kf_default_params(99, ctypes.byref(_lib.kf_params())) == _lib.KF_EINVAL
    assert 'unknown model' in _lib.last_error()


def test_null_handle_is_einval():
    L = _lib.lib()
    assert L.kf_run(None, 4, 0.1, None, None, None, None, 1, None, None, None) == _lib.KF_EINVAL
    assert 'null' in _lib.last_error()
    assert L.kf_free(None) == _lib.KF_OK


def test_no_gpu_fails_loudly():
    if kfmi.device_count() > 0:
        pytest.skip('a GPU is visible; covered by the gpu tests')
    L = _lib.lib()
    assert L.kf_init(0) == _lib.KF_ENODEV
    with pytest.raises(kfmi.KFError) as e:
        kfmi.BatchedKF('cv3', 8, 'f64')
    assert e.value.code == _lib.KF_ENODEV


def test_bad_model_and_dtype_rejected_before_device():
    with pytest.raises(ValueError):
        kfmi.BatchedKF('cv9', 8, 'f64')
    with pytest.raises(ValueError):
        kfmi.BatchedKF('cv3', 8, 'bf16')


def test_options_constants_and_null_handle():
    """kf_set_option / kf_get_option: the header's KF_OPT_* match the binding and the Python
    option table; a null handle is KF_EINVAL (option values are checked on the GPU box)."""
    import re
    from kfmi import engine
    text = open(_lib.HEADER).read()
    ids = {m.group(1): int(m.group(2)) for m in re.finditer(r'#define (KF_OPT_\w+)\s+(\d+)', text)}
    for name, v in ids.items():
        assert getattr(_lib, name) == v, name
    assert sorted(o for o, _ in engine.OPTIONS.values()) == sorted(v for k, v in ids.items() if k != 'KF_OPT_COUNT')
    L = _lib.lib()
    assert L.kf_set_option(None, _lib.KF_OPT_PREDICT, 1) == _lib.KF_EINVAL
    out = ctypes.c_int64(7)
    assert L.kf_get_option(None, _lib.KF_OPT_PREDICT, ctypes.byref(out)) == _lib.KF_EINVAL


def test_library_source_hash_matches_tree():
    """kf_version() carries the hash of the sources it was built from; the loader refuses a
    library built from other sources (a stale .so would test and time old code)."""
    info = _lib.build_info()
    assert info['match'] and info['src_hash'] == _lib.source_hash() and len(info['src_hash']) == 16


def test_library_does_not_read_the_environment():
    """The variant switches are handle options (kf_set_option), not environment variables."""
    import glob
    for p in glob.glob(os.path.join(os.path.dirname(_lib.HEADER), '..', 'sensorfusion-kalmanfilter_amd', 'csrc', '*')):
        assert 'getenv' not in open(p).read(), p


def test_loader_without_sources_raises_kferror(monkeypatch, tmp_path):
    """Loaded from a tree without its sources (an installed package), the hash gate reports the
    origin unknown as KFError, not a raw FileNotFoundError; KFMI_ALLOW_FOREIGN_LIB=1 skips it
    before any source file is read."""
    monkeypatch.setattr(_lib, 'CSRC', str(tmp_path / 'no_csrc'))
    monkeypatch.setattr(_lib, 'HEADER', str(tmp_path / 'no_kf.h'))
    monkeypatch.setattr(_lib, '_lib', None)
    assert _lib.source_hash() is None
    monkeypatch.delenv('KFMI_ALLOW_FOREIGN_LIB', raising=False)
    with pytest.raises(_lib.KFError):
        _lib.lib()
    monkeypatch.setattr(_lib, '_lib', None)
    monkeypatch.setenv('KFMI_ALLOW_FOREIGN_LIB', '1')
    assert _lib.lib() is not None
