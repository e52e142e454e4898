"""CPU: the host-only parts of libsgx.so -- exchange planning (sgx_plan.cpp), the
IndexShuffleBlockResolver index/data commit (sgx_index.cpp), the RCCL-id bootstrap
(sgx_bootstrap.cpp) and the error channel (sgx_errors.cpp) -- built with
-fsanitize=address,undefined and driven by tests/native/host_sanitize.cpp (an
ASan/UBSan build of the C-ABI CPU code).  Any sanitizer report aborts the driver."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "sparkucx_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_sanitize")
    srcs = [os.path.join(ROOT, "tests", "native", "host_sanitize.cpp")] + [
        os.path.join(SRC, f) for f in ("sgx_index.cpp", "sgx_plan.cpp", "sgx_errors.cpp", "sgx_bootstrap.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-pthread", "-o", exe] + srcs, check=True)
    # verify_asan_link_order=0: the environment may preload its own library ahead of ASan's
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, str(tmp_path)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
