"""boda_hip_wis_ana (Boda's wis-ana, src/op-tuner.cc:204-330) on the
reference's own merged wisdom (tests/golden/wis/wisdom-merged.wis, copied from the reference's
test/ directory): the per-op-best sums per platform it reports are the reference's published
per-op figures (Titan X OpenCL 1.13 TF/s ~ 140 ms, Fiji 0.40 TF/s ~ 393 ms
over the 204 conv-ops-1-5-20 ops). No GPU."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_wis_ana")
WIS = os.path.join(ROOT, "tests", "golden", "wis", "wisdom-merged.wis")


def run(*args):
    r = subprocess.run([BIN, "--wisdom-in-fn=" + WIS] + list(args), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = {}
    for l in r.stdout.splitlines():
        m = re.match(r"(\S.*?)\s+(\d+)\s+([\d.]+)\s+([\d.]+)$", l)
        if m and not l.startswith("platform"):
            rows[m.group(1)] = (int(m.group(2)), float(m.group(3)), float(m.group(4)))
    return rows, r.stdout


def test_reference_platform_sums():
    rows, out = run()
    assert rows["ocl:GeForce GTX TITAN X"][0] == 204
    assert abs(rows["ocl:GeForce GTX TITAN X"][2] - 1108.3) < 1.0  # GFLOP/s: BASELINE.md's ~1.1 TF/s
    assert abs(rows["ocl:Fiji"][1] - 392.8) < 0.5                   # ms: BASELINE.md's 393 ms
    assert rows["nvrtc:GeForce GTX TITAN X"][1] < rows["ocl:GeForce GTX TITAN X"][1]
    assert "geomean speedup" in out


def test_filters_and_csv(tmp_path):
    csv = tmp_path / "w.csv"
    rows, _ = run("--s-plat=Fiji", "--s-img=20", "--csv-out-fn=" + str(csv))
    assert list(rows) == ["ocl:Fiji"] and rows["ocl:Fiji"][0] == 68
    lines = csv.read_text().splitlines()
    assert lines[0].startswith("OP FLOPS") and len(lines) == 1 + 68
