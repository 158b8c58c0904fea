"""rtc_test on be=hip (boda_hip_rtc_test): Boda's minimal backend conformance test
(src/rtc_compute.cc:135-194; known-good verdict test/good_tr/test_rtc_nvrtc/rtc_test.txt,
"All is Well."), run through hip_compute_t's hiprtc JIT path with a CUCL program: compile,
vars, a 1-D launch with a by-value scalar (my_dot) and a by-value struct (my_dot_struct),
copy back, compare."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_rtc_test")
PROG = os.path.join(ROOT, "tests", "rtc", "vec_add.cucl")


@pytest.mark.parametrize("func", ["my_dot", "my_dot_struct"])
@pytest.mark.parametrize("n", [10000, 1, 1000003])
def test_rtc_test_all_is_well(func, n, tmp_path):
    out = tmp_path / "rtc_test.txt"
    r = subprocess.run([BIN, "--prog-fn=" + PROG, "--func-name=" + func, "--data-sz=%d" % n, "--out-fn=" + str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert out.read_text() == "All is Well.\n"


def test_rtc_test_missing_function_is_an_error(tmp_path):
    r = subprocess.run([BIN, "--prog-fn=" + PROG, "--func-name=no_such_func"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 3 and "no_such_func" in r.stderr
