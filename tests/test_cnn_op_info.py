"""cnn_op_info (boda_hip_cnn_op_info: Boda's cnn_op_info_t::main, src/cnn-prof.cc:59-130): one tune
against the rocBLAS / MIOpen comparator per op, the comp_vars verdict and the latex info / eff rows
(conv_op_info_to_latex_t, src/latex-util.H:22-139).

CPU (no GPU):
* pp_val's engineering-suffix printing (src/str_util.cc:230-256) reproduces numbers the reference's
  own recorded eff tables hold (doc/sgemm-notes.txt: 64.2us, 65.3GF/s, 990m, 1.48TF/s ...);
* raw eff rows (--print-format=1 --inc-op-info-in-eff=1) have the 12 '&' fields the reference's
  consumer pysrc/op-eff-plot.py:81-90 asserts, with the variant name where it slices it, and the
  bytes / flops / F/B columns equal to the latex-util model (boda_hip.ops) for every op of the set;
* info rows carry KSZ & stride & OC & B & dims(in) & dims(out) & MKN.
GPU: the reference's test_cnn_op_info_{1,conv_cudnn_1} runs (test/test_cmds.xml:103,108: gen_data
modes 600 / 5 on sgemm-ops-debug / conv-ops-debug) print "vars_to_compare: c|out" and
***ALL IS WELL*** (good_tr/test_cnn_op_info_*/cnn_op_info.txt); the eff rows carry finite runtimes
for both sides. Tolerance: the reference loosens its own vendor comparison (ops-prof
--func-mrd-toler='(cudnn_conv=4e-4)', test/test_cmds.xml:110). Ours against rocBLAS / MIOpen
measured max min_sig_mag_rel_diff up to 7.2e-4 (SGEMM 2048^3, mode 5; 1.1e-3 at 1536^3) and 1.56e-3
(direct / GEMM conv routes over the 204 conv-set ops; MIOpen itself is 1.17e-3 from float64 on
20x384x13^2->384): two fp32 accumulation orders apart, with cancellation on near-zero outputs that
min_sig_mag_rel_diff measures absolutely. The comparator runs here at 2e-3 (SGEMM) / 3e-3 (conv);
Winograd routes at the driver's --wino-mrd-toler (2e-3: the reference's own widening for cuDNN's
Winograd, src/rtc_prof.cc:314-319; the 6x6 forms' points 0, +-2/3, +-3/2 and their IC caps keep the
routed ops inside it). The eff rows time both sides in the reference's per-call
convention (the event pair of the last of run_iter calls, src/rtc_prof.cc:104-124), so their speedup
columns compare like with like; the graph-amortized per-call time (--graph-reps) is printed to the
log only. Normalized
(max|d| / max|ref|) the same outputs are within 8.6e-6 of float64 (tools/vendor_acc.py,
profiles/r04/cnn_op_info/vendor_acc.txt). Our kernels are held to the float64 oracle
at the suite's normalized tolerances elsewhere (test_gpu_sgemm / test_gpu_conv / test_gpu_wgx).
"""
import math
import os
import re
import subprocess

import pytest

from boda_hip import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_cnn_op_info")
OPS = os.path.join(ROOT, "tests", "golden", "ops")

needs_bin = pytest.mark.skipif(not os.path.exists(BIN), reason="boda_hip_cnn_op_info not built (make vendor)")


@needs_bin
def test_pp_val_matches_reference_tables():
    # value -> string as printed in the reference's recorded eff tables (doc/sgemm-notes.txt:9-32)
    cases = {64.2e-6: "64.2u", 65.3e9: "65.3G", 0.99: "990m", 1.48e12: "1.48T", 8.14: "8.14", 1.37e-3: "1.37m",
             537e9: "537G", 22.4: "22.4", 121e-6: "121u", 3.56e-3: "3.56m", 0: "0"}
    ks = list(cases)
    r = subprocess.run([BIN, "--pp-vals=" + ",".join(repr(k) for k in ks)], capture_output=True, text=True,
                       check=True)
    assert r.stdout.split() == [cases[k] for k in ks]


@needs_bin
@pytest.mark.parametrize("fn", ["conv-ops-1-5-20-nin-alex-gn.txt", "conv-ops-small.txt"])
def test_raw_eff_rows_parse_as_op_eff_plot(fn, tmp_path):
    eff, info = tmp_path / "eff.raw", tmp_path / "info.tex"
    subprocess.run([BIN, "--cnn-func-sigs-fn=" + os.path.join(OPS, fn), "--no-run=1", "--print-format=1",
                    "--inc-op-info-in-eff=1", "--op-eff-tab-fn=" + str(eff), "--op-info-tab-fn=" + str(info)],
                   capture_output=True, text=True, check=True)
    o, _ = ops.read_ops(os.path.join(OPS, fn))
    shapes = [s for s in (ops.shape_of(x) for x in o) if isinstance(s, ops.ConvShape)]
    rows = open(eff).read().splitlines()
    assert len(rows) == len(shapes) > 0
    for s, row in zip(shapes, rows):
        f = [x.strip() for x in row.split("&")]
        assert len(f) == 12  # read_eff_file's assert
        assert f[0:3] == [str(s.KY), str(s.sy), str(s.OC)]
        assert f[3] == "$ %d \\dx %d \\dx %d \\dx %d $" % (s.B, s.H, s.W, s.IC)
        assert f[4][6:-1] == "Convolution"  # EffPt.varname
        assert math.isclose(float(f[6]), s.bytes(), rel_tol=1e-5)
        assert math.isclose(float(f[7]), s.flops(), rel_tol=1e-5)
        assert math.isclose(float(f[8]), s.flops() / s.bytes(), rel_tol=1e-5)
        assert math.isnan(float(f[9]))  # no run: runtime NAN
    irows = open(info).read().splitlines()
    assert len(irows) == len(shapes)
    s, f = shapes[0], [x.strip() for x in irows[0].split("&")]
    assert f[3] == str(s.B) and f[5] == "$  %d \\dx %d \\dx %d $" % (s.OH, s.OW, s.OC)
    assert f[6] == "$ %d \\dx %d \\dx %d $" % (s.B * s.OH * s.OW, s.IC * s.KY * s.KX, s.OC)


@pytest.mark.gpu
@pytest.mark.parametrize("fn,mode,var", [("sgemm-ops-debug.txt", 600, "c"), ("sgemm-ops-debug.txt", 5, "c"),
                                         ("conv-ops-debug.txt", 5, "out"), ("conv-ops-small.txt", 5, "out")])
def test_cnn_op_info_all_is_well_vs_vendor(fn, mode, var, tmp_path):
    toler = "2e-3" if var == "c" else "3e-3"
    assert os.path.exists(BIN), "boda_hip_cnn_op_info not built"
    eff = tmp_path / "eff.tex"
    r = subprocess.run([BIN, "--cnn-func-sigs-fn=" + os.path.join(OPS, fn), "--gen-data-mode=%d" % mode,
                        "--op-eff-tab-fn=" + str(eff), "--max-err=10", "--mrd-toler=" + toler, "--show-mrd=1"],
                       capture_output=True, text=True, timeout=110)
    print(r.stdout[-3000:], r.stderr[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr
    assert r.stdout.strip().endswith("***ALL IS WELL***")
    n = len(ops.read_ops(os.path.join(OPS, fn))[0])
    assert r.stdout.count("vars_to_compare: %s\n" % var) == n
    mrds = re.findall(r"max_rel_diff=(\S+) toler=(\S+) variant=(\S+)", r.stdout)
    assert len(mrds) == n and all(float(m) < float(t) for m, t, _ in mrds), mrds
    rows = open(eff).read().splitlines()
    assert len(rows) == n
    for row in rows:
        assert "NAN" not in row and "nan" not in row
        if var == "out":  # ... & \verb|variant| & runtime & GF/s & %peak
            f = [x.strip() for x in row.split("&")]
            assert f[4].startswith("\\verb|") and re.match(r"[\d.]+[munp]?s$", f[5]), row
        else:  # ... & comparator runtime & GF/s & runtime & GF/s & speedup
            assert re.search(r"& [\d.]+x \\\\", row), row
