"""Host-code AddressSanitizer check of the C-ABI (SURVEY §5 aux subsystems;
VERDICT round 3 "an ASan build of the C-ABI host code"): `make -C art-sbir_amd
asan` compiles the library's host code with -Xarch_host -fsanitize=address
(device code as usual) and links tests/asan/capi_asan.cpp against it.  The
driver runs without a GPU: the autotune table parser and writer, the error
buffer with over-long arguments, and the entry points' argument checks, under
ASan (any invalid access aborts it).  __graft_entry__.build() builds it."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "art-sbir_amd", "build_asan", "capi_asan")
# written by __graft_entry__.build() when `make asan` fails (removed when it succeeds)
FAILED = os.path.join(ROOT, "art-sbir_amd", "build_asan", "BUILD_FAILED")


def test_asan_build_did_not_fail():
    """a failed sanitizer build must not pass as a skip"""
    if os.path.exists(FAILED):
        with open(FAILED) as f:
            pytest.fail("the AddressSanitizer build failed:\n" + f.read()[-3000:])


@pytest.mark.skipif(not os.path.exists(EXE), reason="ASan build absent: make -C art-sbir_amd asan")
def test_capi_host_code_under_asan(tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asan capi ok" in r.stdout
