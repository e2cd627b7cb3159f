"""Host sanitizer run (CPU): the CSV reader (kf_csv.cpp) built with AddressSanitizer + UBSan and
driven through its edge cases and a multi-threaded 24 MB parse checked value by value against
strtod (tools/sanitize/csv_asan.cpp).  GPU sanitizers are not available on the MI355X pool, so
only host code is instrumented."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, 'tools', 'sanitize')


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++ with ASan')
def test_csv_reader_under_asan_ubsan(tmp_path):
    subprocess.run(['make', '-s', '-C', SAN], check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload a library of its own ahead of ASan's
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=0:verify_asan_link_order=0',
               UBSAN_OPTIONS='print_stacktrace=1')
    r = subprocess.run([os.path.join(SAN, 'csv_asan'), str(tmp_path)], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '0 failure(s)' in r.stdout
