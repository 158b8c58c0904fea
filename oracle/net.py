"""CPU restatement of a full-net forward pass, executing the plan the product's prototxt reader
(boda-1_amd/host/conv_pipe.cc, `boda_hip_rtc_fwd --plan-json`) produced.

*** TEST INFRASTRUCTURE ONLY *** -- used by tests/ as the checker of the net executor; never by
the product path. It re-derives every blob's dims from the op parameters by the reference's
size rules (src/conv_util.cc:167-220; conv floor, Caffe pooling ceil, InnerProduct / global
pooling to 1x1, Concat summing channels) and checks them against the plan, regenerates the
synthetic parameters by the formulas conv_pipe.H documents (the reference ships no
.caffemodel), and runs each layer with the per-layer oracles: oracle.conv_ref
(double accumulation) and oracle/layers.py.

Parity pinning: the per-layer arithmetic is pinned where the layer oracles are (conv: the
reference's known-good digests; other layers: hand-computed known answers, "parity unpinned"
beyond them). The net-level composition -- layer order, blob routing, ReLU fusion, Dropout /
Data / Softmax handling -- follows src/caffepb.cc:166-330 and src/rtc_fwd.cc:263-405.
"""
import numpy as np

from oracle import layers as L
from oracle import oracle as orc

F32 = np.float32
IN_SEED = 234234567  # gen_data_Convolution_in seed (test/rtc/gen_data_Convolution_in.cucl)


def det_hash_rand_vec(n, seed):
    """test/rtc/gen-util.h:1-9 over i = 0..n-1 (+seed), with the final multiply-add fused (as
    the reference JIT and the product's host code compute it): exact in float64, one rounding."""
    h = (np.arange(n, dtype=np.uint64) + np.uint64(seed)).astype(np.uint32)
    h ^= h >> np.uint32(16)
    h = (h.astype(np.uint64) * 0x85EBCA6B).astype(np.uint32)
    h ^= h >> np.uint32(13)
    h = (h.astype(np.uint64) * 0xC2B2AE35).astype(np.uint32)
    h ^= h >> np.uint32(16)
    c = np.float64(F32(10.0) / F32(4294967295.0))
    return (h.astype(F32).astype(np.float64) * c - 5.0).astype(F32)


def param_seed(layer, which):
    """FNV-1a (32-bit) of "layer/which" (conv_pipe.cc param_seed)."""
    h = 2166136261
    for ch in (layer + "/" + which).encode():
        h ^= ch
        h = (h * 16777619) & 0xFFFFFFFF
    return h


def synth(n, layer, which, scale):
    return det_hash_rand_vec(n, param_seed(layer, which)) * F32(scale)


def conv_scale(fan_in):
    return np.sqrt(F32(3.0) / F32(fan_in)) / F32(5.0)


def pool_out_sz(n, k, s, p):
    return L.pool_out_sz(n, k, s, p)


def check_dims(plan):
    """Recompute every op's output dims from its inputs and parameters; return {blob: dims}."""
    dims = {i["name"]: tuple(i["dims"]) for i in plan["inputs"]}
    for op in plan["ops"]:
        B, C, H, W = dims[op["bots"][0]]
        t = op["type"]
        ky, kx = op["k"]
        sy, sx = op["s"]
        py, px = op["p"]
        if t == "Convolution":
            out = (B, op["out_chans"], L.conv_out_sz(H, ky, sy, py), L.conv_out_sz(W, kx, sx, px))
        elif t == "InnerProduct":
            out = (B, op["out_chans"], 1, 1)
        elif t == "Pooling":
            if op["global"]:
                out = (B, C, 1, 1)
            else:
                out = (B, C, pool_out_sz(H, ky, sy, py), pool_out_sz(W, kx, sx, px))
        elif t == "Concat":
            out = (B, sum(dims[b][1] for b in op["bots"]), H, W)
        else:
            out = (B, C, H, W)
        assert tuple(op["out_dims"]) == out, (op["tag"], op["out_dims"], out)
        for tp in op["tops"]:
            dims[tp] = out
    return dims


class _S:  # conv shape for oracle.conv_ref
    def __init__(self, **kw):
        self.__dict__.update(kw)


def forward(plan, x, drop_seed=0):
    """Run the plan on input x (B x C x H x W float32); returns {blob: array}. Dropout ops
    (plans read with --det-dropout) use the rtc mode's deterministic mask seeded by drop_seed."""
    check_dims(plan)
    blobs = {plan["inputs"][0]["name"]: x.astype(F32)}
    for op in plan["ops"]:
        t, tag = op["type"], op["tag"]
        a = blobs[op["bots"][0]]
        B, C, H, W = a.shape
        if t in ("Convolution", "InnerProduct"):
            ip = t == "InnerProduct"
            KY, KX = (H, W) if ip else op["k"]
            (sy, sx), (py, px) = ((1, 1), (0, 0)) if ip else (op["s"], op["p"])
            OC = op["out_chans"]
            s = _S(B=B, IC=C, H=H, W=W, OC=OC, KY=KY, KX=KX, sy=sy, sx=sx, py=py, px=px,
                   OH=L.conv_out_sz(H, KY, sy, py), OW=L.conv_out_sz(W, KX, sx, px))
            f = synth(OC * C * KY * KX, tag, "filts", conv_scale(C * KY * KX))
            b = synth(OC, tag, "biases", 0.1 / 5.0) if op["bias"] else None
            out = orc.conv_ref(np.ascontiguousarray(a).reshape(-1), f, b, s, op["relu"]).reshape(B, OC, s.OH, s.OW)
        elif t == "ReLU":
            out = L.relu(a)
        elif t == "Dropout":  # in place (src/rtc_fwd.cc:348-358)
            out = L.dropout(a, op["ratio"], drop_seed)
        elif t == "Pooling":
            ky, kx = (H, W) if op["global"] else op["k"]
            sy, sx = (1, 1) if op["global"] else op["s"]
            py, px = (0, 0) if op["global"] else op["p"]
            out, _ = L.pool(a, ky, kx, sy, sx, py, px, op["avg"])
        elif t == "LRN":
            out, _ = L.lrn(a, op["local_size"], F32(op["alpha"]), F32(op["beta"]), F32(op["kk"]))
        elif t in ("Concat", "Copy"):
            out = L.concat([blobs[b] for b in op["bots"]])
        elif t in ("BatchNorm", "Scale"):
            if t == "BatchNorm":
                mean = synth(C, tag, "mean", 0.1 / 5.0)
                var = F32(1.0) + synth(C, tag, "var", 0.5 / 5.0)
                sc = F32(1.0) / np.sqrt(var + F32(op["kk"]))
                sh = -mean * sc
            else:
                sc = F32(1.0) + synth(C, tag, "gamma", 0.1 / 5.0)
                sh = synth(C, tag, "beta", 0.1 / 5.0) if op["bias"] else np.zeros(C, F32)
            out = (a * sc[None, :, None, None] + sh[None, :, None, None]).astype(F32)
            if op["relu"]:
                out = L.relu(out)
        elif t == "Eltwise":
            b2 = blobs[op["bots"][1]]
            e = op["eltwise"]
            out = (a + b2) if e == "SUM" else (a * b2 if e == "PROD" else np.maximum(a, b2))
            out = out.astype(F32)
            if op["relu"]:
                out = L.relu(out)
        else:
            raise ValueError("net oracle: no restatement for layer type " + t)
        if op["relu"] and t in ("Convolution", "InnerProduct"):
            pass  # conv_ref applied it
        for tp in op["tops"]:
            blobs[tp] = out
    return blobs
