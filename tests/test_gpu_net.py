"""Full-net forward on the GPU (BASELINE config C4): the net
executor driven through Boda's net-level plugin surface (boda_hip_rtc_fwd: prototxt reader +
has_conv_fwd_t mode "rtc" = conv_pipe_fwd_t over be=hip, every layer a hand-written kernel behind
the C-ABI) against oracle/net.py, the CPU restatement running the same plan with the per-layer
oracles, on the reference's own nets.

Bar: rel-L2 <= 1e-4 and max|d| / max(1, max|ref|) <= 1e-3 on the net output and, as the
reference's test_compute compares every var (src/test_compute.cc:170-200, mrd_toler with
per-layer overrides), on EVERY blob of the forward (fp32 rounding of up to ~70 stacked layers vs
a double-accumulating CPU conv; the per-op bar is 1e-5 / 1e-4).
"""
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import net as onet
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_rtc_fwd")
NETS = os.path.join(ROOT, "tests", "golden", "nets")


def run_net(net, img, tmp, extra=()):
    pt = os.path.join(NETS, net + ".prototxt")
    r = subprocess.run([BIN, "--net", pt, "--img", str(img), "--plan-json"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout)
    r = subprocess.run([BIN, "--net", pt, "--img", str(img), "--iters", "2", "--save", str(tmp)] + list(extra),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    print(r.stdout)
    x = np.fromfile(os.path.join(tmp, "in.f32"), dtype=np.float32)
    got = np.fromfile(os.path.join(tmp, "out.f32"), dtype=np.float32)
    return plan, x, got, r.stdout


NETS5 = ["alexnet_ng_conv", "nin_imagenet", "googlenet_conv", "resnet-50", "vgg_19"]
# per-blob bars (src/test_compute.cc's var_mrd_toler: one default, per-var overrides where needed)
BLOB_RL2, BLOB_NM = 1e-4, 1e-3


def plan_of(net, img, extra=()):
    r = subprocess.run([BIN, "--net", os.path.join(NETS, net + ".prototxt"), "--img", str(img), "--plan-json"] +
                       list(extra), capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def run_blobs(net, img, tmp, sample=0, extra=()):
    """Every blob of the forward (--save-blobs, rewrites that hide blobs off), sampled with a
    stride of ceil(elems / sample) when sample > 0: {name: (values, stride)}."""
    pt = os.path.join(NETS, net + ".prototxt")
    cmd = [BIN, "--net", pt, "--img", str(img), "--iters", "1", "--save", str(tmp), "--save-blobs", str(tmp),
           "--no-inplace-concat", "--no-resadd"] + (["--blob-sample", str(sample)] if sample else []) + list(extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    idx = json.load(open(os.path.join(tmp, "blobs.json")))
    x = np.fromfile(os.path.join(tmp, "in.f32"), dtype=np.float32)
    return x, {b["name"]: (np.fromfile(os.path.join(tmp, b["file"]), dtype=np.float32), b["stride"])
               for b in idx["blobs"]}, r.stdout


def check_blobs(net, plan, ref_blobs, got):
    tops = {t for op in plan["ops"] for t in op["tops"]}
    assert set(got) == tops, (net, sorted(tops ^ set(got)))
    worst = (0.0, 0.0, "")
    for name, (v, stride) in got.items():
        ref = ref_blobs[name].reshape(-1)[::stride]
        assert ref.shape == v.shape, (net, name, ref.shape, v.shape)
        nm, rl2, _ = orc.normalized_errors(ref, v)
        assert rl2 <= BLOB_RL2 and nm <= BLOB_NM, (net, name, nm, rl2)
        worst = max(worst, (rl2, nm, name))
    print(net, "%d blobs, worst rl2 %.2e nm %.2e (%s)" % (len(got), worst[0], worst[1], worst[2]))


@pytest.mark.parametrize("net", NETS5)
def test_net_every_blob(net, tmp_path):
    """Per-layer parity at batch 1: every blob the net produces against the net oracle's."""
    plan = plan_of(net, 1)
    x, got, _ = run_blobs(net, 1, tmp_path)
    d0 = plan["inputs"][0]["dims"]
    np.testing.assert_array_equal(x, onet.det_hash_rand_vec(int(np.prod(d0)), onet.IN_SEED))
    check_blobs(net, plan, onet.forward(plan, x.reshape(d0)), got)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("net", ["resnet-50", "vgg_19"])
def test_net_every_blob_batch20(net, tmp_path):
    """Per-layer parity at batch 20 (BASELINE config C4): every blob, sampled (~4096 elements
    each, a fixed stride), against the net oracle's."""
    plan = plan_of(net, 20)
    x, got, _ = run_blobs(net, 20, tmp_path, sample=4096)
    check_blobs(net, plan, onet.forward(plan, x.reshape(plan["inputs"][0]["dims"])), got)


def test_det_dropout_seeded(tmp_path):
    """set_det_drop_seed: the rtc mode's deterministic dropout (in place, --det-dropout SEED) against
    the net oracle's mask for that seed, on every blob; another seed gives another output."""
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    plan = plan_of("alexnet_ng_conv", 2, ["--det-dropout", "7"])
    assert [o["tag"] for o in plan["ops"] if o["type"] == "Dropout"] == ["drop6", "drop7"]
    x, got, _ = run_blobs("alexnet_ng_conv", 2, a, extra=["--det-dropout", "7"])
    ref = onet.forward(plan, x.reshape(plan["inputs"][0]["dims"]), drop_seed=7)
    check_blobs("alexnet_ng_conv", plan, ref, got)
    _, got8, _ = run_blobs("alexnet_ng_conv", 2, b, extra=["--det-dropout", "8"])
    out = plan["out_node"]
    assert not np.array_equal(got8[out][0], got[out][0])


def test_mode_options_stats_and_per_call_file(tmp_path):
    """Mode options through init(cp, nia): enable_stats puts min / max / sum / cnt of each fetched
    blob in get_info_log, per_call_fn writes run_fwd's per-layer time file."""
    pcf = tmp_path / "per_call.py"
    pt = os.path.join(NETS, "nin_imagenet.prototxt")
    r = subprocess.run([BIN, "--net", pt, "--img", "1", "--iters", "1", "--save", str(tmp_path), "--mode-args",
                        "(enable_stats=1,per_call_fn=%s)" % pcf], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    out = np.fromfile(os.path.join(tmp_path, "out.f32"), dtype=np.float32)
    plan = plan_of("nin_imagenet", 1)
    stats = dict(l.split("=") for l in r.stdout.splitlines() if l.startswith(plan["out_node"] + "_"))
    assert float(stats[plan["out_node"] + "_cnt"]) == out.size
    assert float(stats[plan["out_node"] + "_max"]) == out.max()
    np.testing.assert_allclose(float(stats[plan["out_node"] + "_sum"]), out.astype(np.float64).sum(), rtol=1e-6)
    lines = pcf.read_text().splitlines()
    assert lines[0].startswith("net.args.runtime=") and float(lines[0].split("=")[1]) > 0
    assert sum(l.startswith("per_layer_time['") for l in lines) == len(
        [o for o in plan["ops"]]), lines


@pytest.mark.parametrize("net", NETS5)
def test_net_forward(net, tmp_path):
    plan, x, got, _ = run_net(net, 1, tmp_path)
    d0 = plan["inputs"][0]["dims"]
    np.testing.assert_array_equal(x, onet.det_hash_rand_vec(int(np.prod(d0)), onet.IN_SEED))
    blobs = onet.forward(plan, x.reshape(d0))
    ref = blobs[plan["out_node"]].reshape(-1)
    assert ref.shape == got.shape
    nm, rl2, _ = orc.normalized_errors(ref, got)
    print(net, "out", plan["out_node"], "nm %.2e rl2 %.2e" % (nm, rl2))
    assert rl2 <= 1e-4 and nm <= 1e-3, (net, nm, rl2)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("net", ["resnet-50", "vgg_19"])
def test_net_forward_batch20(net, tmp_path):
    """BASELINE config C4 at its batch: ResNet-50 / VGG-19 forward at batch 20 (BatchNorm / Scale
    folding, residual epilogues and every b20 tuning-table route on) against the CPU net oracle --
    the role of the reference's test_compute net comparison (src/test_compute.cc:216-276)."""
    plan, x, got, _ = run_net(net, 20, tmp_path)
    d0 = plan["inputs"][0]["dims"]
    assert d0[0] == 20
    np.testing.assert_array_equal(x, onet.det_hash_rand_vec(int(np.prod(d0)), onet.IN_SEED))
    ref = onet.forward(plan, x.reshape(d0))[plan["out_node"]].reshape(-1)
    nm, rl2, _ = orc.normalized_errors(ref, got)
    print(net, "b20 out", plan["out_node"], "nm %.2e rl2 %.2e" % (nm, rl2))
    assert rl2 <= 1e-4 and nm <= 1e-3, (net, nm, rl2)


def test_net_unpacked_bank_same_bits(tmp_path):
    """--no-pack (filter banks transformed inside every conv call) gives the same output bits."""
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    _, _, g1, _ = run_net("alexnet_ng_conv", 2, a)
    _, _, g2, _ = run_net("alexnet_ng_conv", 2, b, ["--no-pack"])
    np.testing.assert_array_equal(g1, g2)


def test_resnet_bn_scale_folded(tmp_path):
    """BatchNorm / Scale folded into the producing conv (conv_pipe_fwd_t::plan_folds): no
    affine kernel runs, and the output matches the unfolded executor to fp32 rounding."""
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    _, _, g1, log1 = run_net("resnet-50", 1, a)
    _, _, g2, log2 = run_net("resnet-50", 1, b, ["--no-fold"])
    assert "hip_affine__" not in log1 and log2.count("hip_affine__") == 106
    nm, rl2, _ = orc.normalized_errors(g2, g1)
    assert rl2 <= 1e-5 and nm <= 1e-4, (nm, rl2)


def test_googlenet_concat_in_place_same_bits(tmp_path):
    """Convs writing their Concat slab in place (plan_slabs) give the copying executor's bits."""
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    _, _, g1, log1 = run_net("googlenet_conv", 2, a)
    _, _, g2, log2 = run_net("googlenet_conv", 2, b, ["--no-inplace-concat"])
    np.testing.assert_array_equal(g1, g2)
    assert log1.count("hip_copy__") < log2.count("hip_copy__")


@pytest.mark.parametrize("net", ["googlenet_conv", "resnet-50"])
def test_forward_graph_replay(net, tmp_path):
    """The whole forward captured as one hipGraph and replayed (--graph): it runs, reports a
    time, and leaves the eager forward's output bits."""
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    _, _, g1, _ = run_net(net, 2, a)
    _, _, g2, log = run_net(net, 2, b, ["--graph", "3"])
    np.testing.assert_array_equal(g1, g2)
    line = [l for l in log.splitlines() if l.startswith("forward as one hipGraph")]
    assert len(line) == 1 and float(line[0].split(")")[1].split()[0]) > 0, log


def test_resnet_residual_in_conv_epilogue_same_bits(tmp_path):
    """Shortcut Eltwise SUM (+ ReLU) in the producing conv's epilogue (plan_resadds): no eltwise
    kernel runs, and the output bits equal the executor running Eltwise as its own layer."""
    a = tmp_path / "a"
    b = tmp_path / "b"
    a.mkdir()
    b.mkdir()
    _, _, g1, log1 = run_net("resnet-50", 2, a)
    _, _, g2, log2 = run_net("resnet-50", 2, b, ["--no-resadd"])
    assert "hip_eltwise__" not in log1 and log2.count("hip_eltwise__") == 16
    np.testing.assert_array_equal(g1, g2)
