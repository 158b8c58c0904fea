"""CPU-only checks of the product's host side and the C-ABI library (no GPU).

* libboda_hip.so loads and exports every symbol include/boda_hip.h declares;
* without a usable GPU the product fails loudly (no CPU fallback);
* the C++ host side (boda_hip_ops_prof) parses every reference op list exactly
  as the Python glue does, and round-trips every known-good digest of the
  reference's wisdom files byte-identically;
* the flop/byte totals match BASELINE.md's figures for the headline sets.
"""
import ctypes
import os
import re
import subprocess

import pytest

import boda_hip
from boda_hip import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "boda_hip.h")
OPS = os.path.join(ROOT, "tests", "golden", "ops")
WIS = os.path.join(ROOT, "tests", "golden", "wis")
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_ops_prof")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bh_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_symbols() == sorted(boda_hip.EXPORTS)


def test_library_exports_every_symbol():
    lib = ctypes.CDLL(boda_hip.LIB_PATH)
    for s in header_symbols():
        assert hasattr(lib, s), s
    assert boda_hip.lib().bh_abi_version() == 3


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", boda_hip.LIB_PATH], capture_output=True,
                         text=True).stdout
    out += subprocess.run(["strings", boda_hip.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_no_cpu_fallback_without_gpu():
    if boda_hip.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(boda_hip.BodaHipError):
        boda_hip.Device(0)
    r = subprocess.run([BIN, "--ops-fn=" + os.path.join(OPS, "sgemm-ops-tiny.txt")], capture_output=True, text=True)
    assert r.returncode != 0 and "no HIP device" in r.stderr


@pytest.mark.parametrize("fn", sorted(os.listdir(WIS)))
def test_cpp_wisdom_roundtrip(fn):
    r = subprocess.run([BIN, "--selftest-wisdom=" + os.path.join(WIS, fn)], capture_output=True, text=True)
    assert r.returncode == 0 and "selftest ok" in r.stdout, r.stderr


@pytest.mark.parametrize("fn", ["conv-ops-1-5-20-nin-alex-gn.txt", "sgemm-ops-full.txt", "op_sigs_full.txt",
                                "conv-ops-debug.txt", "sgemm-ops-small.txt", "conv-ops-tiny.txt"])
def test_cpp_and_python_parse_agree(fn):
    r = subprocess.run([BIN, "--dump-ops=" + os.path.join(OPS, fn)], capture_output=True, text=True, check=True)
    lines = r.stdout.strip().split("\n")
    py, skipped = ops.read_ops(os.path.join(OPS, fn))
    assert lines[-1] == "skipped %d" % skipped
    assert len(lines) - 1 == len(py)
    for l, op in zip(lines, py):
        f = l.split()
        s = ops.shape_of(op)
        if op.type == "Convolution":
            assert f[0] == "Convolution" and [int(x) for x in f[1:12]] == s.as_dims()
        else:
            assert f[0] == "sgemm" and [int(x) for x in f[1:4]] == [s.M, s.N, s.K]
        assert float(f[-2]) == s.flops() and float(f[-1]) == s.bytes()


def test_baseline_totals():
    conv, _ = ops.read_ops(os.path.join(OPS, "conv-ops-1-5-20-nin-alex-gn.txt"))
    sg, _ = ops.read_ops(os.path.join(OPS, "sgemm-ops-full.txt"))
    assert len(conv) == 204 and len(sg) == 17
    assert round(sum(ops.shape_of(o).flops() for o in conv) / 1e9, 2) == 158.47
    assert round(sum(ops.shape_of(o).bytes() for o in conv) / 1e6, 1) == 1937.7
    assert round(sum(ops.shape_of(o).flops() for o in sg) / 1e9) == 8650
    sigs, skipped = ops.read_ops(os.path.join(OPS, "op_sigs_full.txt"))
    assert len(sigs) == 178 and skipped == 408


def test_lexp_dialects_equivalent():
    cur = ("(str_vals=(type=Convolution),nda_vals=(biases=(dims=(out_chan=16)),filts=(dims=(out_chan=16,in_chan=96,"
           "y=1,x=1)),in=(dims=(img=3,chan=96,y=55,x=55)),in_pad=(tn=none,dims=(y=0,x=0)),kern_sz=(tn=none,dims=(y=1,"
           "x=1)),out=(dims=(img=3,chan=16,y=55,x=55)),out_chans=(tn=uint32_t,v=16),stride=(tn=none,dims=(y=1,x=1))))")
    leg = ("(type=Convolution,dims_vals=(biases=(out_chan=16),filts=(out_chan=16,in_chan=96,y=1,x=1),in=(img=3,chan=96,"
           "y=55,x=55),in_pad=(y=0,x=0),kern_sz=(y=1,x=1),out=(img=3,chan=16,y=55,x=55),stride=(y=1,x=1)),"
           "str_vals=(out_chans=16))")
    assert ops.conv_shape(ops.parse_op(cur)) == ops.conv_shape(ops.parse_op(leg))
    with pytest.raises(ops.LexpError):
        ops.parse_lexp("(a=1,a=2)")
    with pytest.raises(ops.LexpError):
        ops.parse_lexp("(a=(b=1)")
    assert ops.parse_lexp(r"(a=x\,y)")["a"] == "x,y"


def test_inconsistent_ops_rejected():
    bad = ("(type=Convolution,dims_vals=(biases=(out_chan=16),filts=(out_chan=16,in_chan=96,y=1,x=1),in=(img=3,chan=96,"
           "y=55,x=55),in_pad=(y=0,x=0),kern_sz=(y=1,x=1),out=(img=3,chan=16,y=54,x=55),stride=(y=1,x=1)))")
    with pytest.raises(ValueError):
        ops.conv_shape(ops.parse_op(bad))


def test_vendor_library_exports_every_symbol():
    """The comparator library (include/boda_hip_vendor.h) loads and exports its C-ABI; the product
    library does not link rocBLAS/MIOpen."""
    from boda_hip import vendor
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "boda_hip_vendor.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(bhv_[a-z0-9_]+)\s*\(", txt)))
    assert syms == sorted(vendor.EXPORTS)
    lib = ctypes.CDLL(vendor.LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s
    deps = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-d", boda_hip.LIB_PATH], capture_output=True,
                          text=True).stdout
    assert "rocblas" not in deps.lower() and "miopen" not in deps.lower()
