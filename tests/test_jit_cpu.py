"""The hiprtc JIT path of the backend (bh_jit_build / bh_jit_compile; Boda's nvrtc_compute_t
compiles every non-intercepted CUCL function this way, src/nvrtc_util.cc:216-260) without a GPU:
hiprtc builds gfx950 code objects on the host, so the CUCL dialect and the error path are
checked here; running the code is test_gpu_rtc.py's job."""
import os

import pytest

import boda_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRELUDE = """
typedef unsigned uint32_t;
#define CUCL_GLOBAL_KERNEL extern "C" __global__
#define GASQ
#define GLOB_ID_1D (blockDim.x * blockIdx.x + threadIdx.x)
"""


def test_jit_builds_the_rtc_test_program():
    src = PRELUDE + open(os.path.join(ROOT, "tests", "rtc", "vec_add.cucl")).read()
    n, log = boda_hip.jit_build(src, "-ffast-math")
    assert n > 1000, log


def test_jit_reports_compile_errors():
    with pytest.raises(boda_hip.BodaHipError) as e:
        boda_hip.jit_build(PRELUDE + "CUCL_GLOBAL_KERNEL void f( GASQ float * x ) { undeclared_thing = 1; }")
    assert "undeclared_thing" in str(e.value)
