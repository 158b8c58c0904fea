"""ctypes wrapper of oracle/liboracle.so.

*** TEST INFRASTRUCTURE ONLY *** -- imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, as the checker / CPU baseline, never by the
product path (boda-1_amd/). See oracle.c for the reference file:line each
function restates and for how the oracle is pinned to the reference's own
known-good digests (tests/golden/).
"""
import ctypes
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_L = None
u32, u64, f32p = ctypes.c_uint32, ctypes.c_uint64, ctypes.POINTER(ctypes.c_float)


def _lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        vp = ctypes.c_void_p
        L.orc_det_hash_rand.argtypes = [u32]
        L.orc_det_hash_rand.restype = ctypes.c_float
        L.orc_gen_sgemm_a.argtypes = [vp, u32, u32, u32, ctypes.c_float]
        L.orc_gen_sgemm_b.argtypes = [vp, u32, u32, u32, ctypes.c_float]
        L.orc_gen_conv4.argtypes = [vp, u32, u32, u32, u32, ctypes.c_int, u32, ctypes.c_float]
        L.orc_gen_conv_biases.argtypes = [vp, u32, u32, ctypes.c_float]
        L.orc_conv_out_sz.argtypes = [u32, u32, u32, u32]
        L.orc_conv_out_sz.restype = u32
        L.orc_sgemm_ref.argtypes = [vp, vp, vp, u32, u32, u32]
        L.orc_sgemm_fast.argtypes = [vp, vp, vp, u32, u32, u32]
        L.orc_conv_ref.argtypes = [vp, vp, vp, vp] + [u32] * 11 + [ctypes.c_int]
        L.orc_conv_fast.argtypes = [vp, vp, vp, vp] + [u32] * 11 + [ctypes.c_int]
        L.orc_conv_ref_at.argtypes = [vp, vp, vp, vp, u64, vp] + [u32] * 11 + [ctypes.c_int]
        L.orc_digest_plan.argtypes = [u64, vp, ctypes.c_int, u64, vp, ctypes.c_int]
        L.orc_digest_plan.restype = ctypes.c_int
        L.orc_digest.argtypes = [vp, u64, vp, ctypes.c_int, u64, f32p, f32p, vp, ctypes.c_int]
        L.orc_digest.restype = ctypes.c_int
        L.orc_min_sig_mag_rel_diff.argtypes = [ctypes.c_double] * 3
        L.orc_min_sig_mag_rel_diff.restype = ctypes.c_double
        L.orc_digest_compare.argtypes = [vp, ctypes.c_float, ctypes.c_float, vp, ctypes.c_float, ctypes.c_float,
                                         vp, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
        L.orc_digest_compare.restype = ctypes.c_int
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_num_threads.argtypes = [ctypes.c_int]
        _L = L
    return _L


def _p(a):
    return a.ctypes.data


def det_hash_rand(i):
    return _lib().orc_det_hash_rand(i)


def gen_sgemm(M, N, K, mode, vi=0.0):
    a = np.empty(K * M, np.float32)
    b = np.empty(K * N, np.float32)
    _lib().orc_gen_sgemm_a(_p(a), K, M, mode, vi)
    _lib().orc_gen_sgemm_b(_p(b), K, N, mode, vi)
    return a, b


def gen_conv(s, mode, vi=0.0):
    inp = np.empty(s.B * s.IC * s.H * s.W, np.float32)
    filts = np.empty(s.OC * s.IC * s.KY * s.KX, np.float32)
    biases = np.empty(s.OC, np.float32)
    _lib().orc_gen_conv4(_p(inp), s.B, s.IC, s.H, s.W, 0, mode, vi)
    _lib().orc_gen_conv4(_p(filts), s.OC, s.IC, s.KY, s.KX, 1, mode, vi)
    _lib().orc_gen_conv_biases(_p(biases), s.OC, mode, vi)
    return inp, filts, biases


def sgemm_ref(a, b, M, N, K, fast=False):
    c = np.empty(M * N, np.float32)
    (_lib().orc_sgemm_fast if fast else _lib().orc_sgemm_ref)(_p(a), _p(b), _p(c), M, N, K)
    return c


def conv_ref(inp, filts, biases, s, relu=1, fast=False):
    out = np.empty(s.B * s.OC * s.OH * s.OW, np.float32)
    f = _lib().orc_conv_fast if fast else _lib().orc_conv_ref
    f(_p(inp), _p(filts), _p(biases) if biases is not None else None, _p(out),
      s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px, int(relu))
    return out


def conv_ref_at(inp, filts, biases, s, idx, relu=1):
    """Double-accumulated outputs at the flat NCHW output indices idx (sampled checks of big shapes)."""
    idx = np.ascontiguousarray(idx, np.uint64)
    vals = np.empty(idx.size, np.float32)
    _lib().orc_conv_ref_at(_p(inp), _p(filts), _p(biases) if biases is not None else None, _p(idx), idx.size,
                           _p(vals), s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px, int(relu))
    return vals


def set_threads(n):
    _lib().orc_set_num_threads(int(n))


def num_threads():
    return _lib().orc_num_threads()


def conv_out_sz(i, pad, k, stride):
    return _lib().orc_conv_out_sz(i, pad, k, stride)


# ---------------------------------------------------------------- digests

def f32_from_hex(w):
    return struct.unpack("<f", struct.pack("<I", w))[0]


class Digest:
    """nda_digest_T<float> (src/boda_base.cc:214-276)."""

    def __init__(self, dims, seed, mn, mx, samps, sis):
        self.dims, self.seed, self.min, self.max, self.samps, self.sis = dims, seed, mn, mx, samps, sis

    @staticmethod
    def dim_strides(dims):
        st, acc = [], 1
        for _, sz in reversed(dims):
            st.append(acc)
            acc *= sz
        return list(reversed(st)), acc

    @classmethod
    def of(cls, arr, dims, seed):
        """dims: [(name, size), ...] outermost first."""
        arr = np.ascontiguousarray(arr, np.float32)
        strides, n = cls.dim_strides(dims)
        assert arr.size == n
        st = np.array(strides, np.uint64)
        cap = 4096
        sis = np.zeros(3 * cap, np.uint64)
        cnt = _lib().orc_digest_plan(n, _p(st), len(strides), seed, _p(sis), cap)
        assert cnt <= cap
        samps = np.zeros(cnt, np.float32)
        mn, mx = ctypes.c_float(), ctypes.c_float()
        _lib().orc_digest(_p(arr), n, _p(st), len(strides), seed, ctypes.byref(mn), ctypes.byref(mx), _p(samps), cnt)
        return cls(dims, seed, mn.value, mx.value, samps, sis[:3 * cnt].copy())

    @classmethod
    def from_golden(cls, kg):
        """A decoded known-good digest from tests/golden/*.json."""
        dims = [(d[0], d[1]) for d in kg["dims"]]
        strides, n = cls.dim_strides(dims)
        assert [d[2] for d in kg["dims"]] == strides and kg["strides_sz"] == n
        st = np.array(strides, np.uint64)
        cap = 4096
        sis = np.zeros(3 * cap, np.uint64)
        cnt = _lib().orc_digest_plan(n, _p(st), len(strides), kg["seed"], _p(sis), cap)
        samps = np.array([f32_from_hex(w) for w in kg["samps"]], np.float32)
        if cnt != len(samps):
            raise ValueError("digest plan has %d samples, fixture %d" % (cnt, len(samps)))
        return cls(dims, kg["seed"], f32_from_hex(kg["min"]), f32_from_hex(kg["max"]), samps, sis[:3 * cnt].copy())

    def compare(self, other, mrd=2e-4):
        """mrd_comp (src/boda_base.cc:284-310) with self as the known-good side.
        Returns (n_failures, worst rd / allowed ratio)."""
        assert self.dims == other.dims and self.seed == other.seed
        w = ctypes.c_double(0)
        fails = _lib().orc_digest_compare(_p(self.samps), self.min, self.max, _p(other.samps), other.min, other.max,
                                          _p(self.sis), len(self.samps), mrd, ctypes.byref(w))
        return fails, w.value


def normalized_errors(ref, got):
    """F11 parity metrics against the double-accumulated oracle:
    max|d| / max(1, max|ref|), rel-L2, and the raw elementwise hybrid max
    (min_sig_mag_rel_diff, src/boda_base.cc:140-153)."""
    r = ref.astype(np.float64)
    g = got.astype(np.float64)
    d = np.abs(g - r)
    scale = max(1.0, float(np.max(np.abs(r))) if r.size else 1.0)
    norm_max = float(d.max()) / scale if d.size else 0.0
    rl2 = float(np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)) if r.size else 0.0
    hyb = float(np.max(d / np.maximum(1.0, np.maximum(np.abs(r), np.abs(g))))) if r.size else 0.0
    return norm_max, rl2, hyb
