"""The C-ABI's host-side argument validation under AddressSanitizer + UBSan
(SURVEY §5): tests/asan/capi_args.cpp against an ASan build of
libpolarldpc.so's host code (tests/asan/Makefile), run on CPU.  Bad arguments
must be refused with PL_EINVAL / PL_EUNSUPPORTED, plans on a machine without a
device must fail cleanly, and no path may leak or touch memory it does not own."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "asan")


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_capi_argument_validation_under_asan():
    subprocess.run(["make", "-s", "-j8", "-C", HERE], check=True, timeout=900,
                   stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               LSAN_OPTIONS="suppressions=" + os.path.join(HERE, "lsan.supp"),
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", HIP_VISIBLE_DEVICES="")
    p = subprocess.run([os.path.join(HERE, "_build", "capi_args")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "all checks passed" in p.stdout
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
