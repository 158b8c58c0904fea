"""ctypes binding of libboda_hip.so (include/boda_hip.h) for tests and bench.py.

The binding is thin on purpose: every call goes straight through the C-ABI a
Boda maintainer would bind from hip_compute_t. There is no CPU
fallback: without a gfx950 device Device() raises BodaHipError.
"""
import ctypes
import os

import numpy as np

from . import ops  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# BH_LIB_NAME selects an alternative in-tree build (e.g. libboda_hip_ktrace.so, tools/ktrace.py)
LIB_PATH = os.path.join(PKG, "lib", os.environ.get("BH_LIB_NAME", "libboda_hip.so"))

BH_OK, BH_ERR, BH_UNSUP = 0, 1, 2
GEN_SGEMM_A, GEN_SGEMM_B, GEN_CONV_IN, GEN_CONV_FILTS, GEN_CONV_BIASES = range(5)

# every symbol include/boda_hip.h declares (checked by tests/test_abi.py)
EXPORTS = ["bh_abi_version", "bh_last_error", "bh_device_count", "bh_init", "bh_destroy", "bh_plat_tag",
           "bh_get_stream", "bh_alloc", "bh_free", "bh_memset0", "bh_h2d", "bh_d2h", "bh_sync",
           "bh_event_record", "bh_elapsed_ms", "bh_events_reset", "bh_gen_data", "bh_sgemm_kmajor",
           "bh_conv2d_fwd_nchw", "bh_variant_name", "bh_variant_name_ctx", "bh_tune_set", "bh_tune_set_policy", "bh_tune_cfg_name",
           "bh_capture_begin", "bh_capture_end", "bh_graph_launch", "bh_graph_destroy",
           "bh_stamp", "bh_stamps_read", "bh_time_next_call", "bh_spin", "bh_conv2d_fwd_nchw_pk",
           "bh_conv_filts_packed_floats", "bh_conv_filts_pack", "bh_pool_out_size", "bh_pool_fwd_nchw",
           "bh_lrn_fwd_nchw", "bh_relu_inplace", "bh_dropout_inplace", "bh_softmax_chans", "bh_chan_copy", "bh_chan_affine",
           "bh_eltwise", "bh_conv2d_fwd_nchw_slab", "bh_conv2d_fwd_nchw_res", "bh_jit_build", "bh_jit_compile",
           "bh_jit_launch", "bh_jit_release", "bh_conv_filts_packed_floats_banks", "bh_conv_filts_pack_banks",
           "bh_conv_route_banks", "bh_conv2d_fwd_nchw_pkb"]
BANK_W23, BANK_W43, BANK_W25, BANKS_ALL = 1, 2, 4, 0xffffffff


class BodaHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


class UnsupportedError(BodaHipError):
    pass


_lib = None
c_u32 = ctypes.c_uint32
c_vp = ctypes.c_void_p


def lib():
    """Load libboda_hip.so (built in-tree by __graft_entry__.build / make)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BodaHipError(BH_ERR, "libboda_hip.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        L.bh_last_error.restype = ctypes.c_char_p
        L.bh_abi_version.restype = ctypes.c_int
        L.bh_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.bh_init.argtypes = [ctypes.c_int, ctypes.POINTER(c_vp)]
        L.bh_destroy.argtypes = [c_vp]
        L.bh_plat_tag.argtypes = [c_vp, ctypes.c_char_p, ctypes.c_size_t]
        L.bh_get_stream.argtypes = [c_vp, ctypes.POINTER(c_vp)]
        L.bh_alloc.argtypes = [c_vp, ctypes.c_size_t, ctypes.POINTER(c_vp)]
        L.bh_free.argtypes = [c_vp, c_vp]
        L.bh_memset0.argtypes = [c_vp, c_vp, ctypes.c_size_t]
        L.bh_h2d.argtypes = [c_vp, c_vp, c_vp, ctypes.c_size_t]
        L.bh_d2h.argtypes = [c_vp, c_vp, c_vp, ctypes.c_size_t]
        L.bh_sync.argtypes = [c_vp]
        L.bh_event_record.argtypes = [c_vp, ctypes.POINTER(ctypes.c_int)]
        L.bh_elapsed_ms.argtypes = [c_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.bh_events_reset.argtypes = [c_vp]
        L.bh_gen_data.argtypes = [c_vp, ctypes.c_int, c_vp, ctypes.POINTER(c_u32), c_u32, ctypes.c_float]
        L.bh_sgemm_kmajor.argtypes = [c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32]
        L.bh_conv2d_fwd_nchw.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp] + [c_u32] * 11 + [ctypes.c_int]
        L.bh_conv2d_fwd_nchw_pk.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp] + [c_u32] * 11 + [ctypes.c_int]
        L.bh_conv2d_fwd_nchw_res.argtypes = [c_vp] * 7 + [c_u32] * 11 + [ctypes.c_int]
        L.bh_conv2d_fwd_nchw_slab.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp] + [c_u32] * 13 + [ctypes.c_int]
        L.bh_conv_filts_packed_floats.argtypes = [c_u32] * 4
        L.bh_conv_filts_packed_floats.restype = ctypes.c_size_t
        L.bh_conv_filts_pack.argtypes = [c_vp, c_vp, c_vp] + [c_u32] * 4
        L.bh_conv_filts_packed_floats_banks.argtypes = [c_u32] * 5
        L.bh_conv_filts_packed_floats_banks.restype = ctypes.c_size_t
        L.bh_conv_filts_pack_banks.argtypes = [c_vp, c_vp, c_vp] + [c_u32] * 5
        L.bh_conv_route_banks.argtypes = [c_vp, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32)]
        L.bh_conv2d_fwd_nchw_pkb.argtypes = [c_vp, c_vp, c_vp, c_vp, c_u32, c_vp, c_vp, c_vp] + [c_u32] * 13 + [ctypes.c_int]
        L.bh_pool_out_size.argtypes = [c_u32] * 4
        L.bh_pool_fwd_nchw.argtypes = [c_vp, c_vp, c_vp, c_vp] + [c_u32] * 10 + [ctypes.c_int]
        L.bh_lrn_fwd_nchw.argtypes = [c_vp, c_vp, c_vp, c_vp] + [c_u32] * 5 + [ctypes.c_float] * 3
        L.bh_relu_inplace.argtypes = [c_vp, c_vp, ctypes.c_uint64]
        L.bh_dropout_inplace.argtypes = [c_vp, c_vp, ctypes.c_uint64, ctypes.c_float, c_u32]
        L.bh_softmax_chans.argtypes = [c_vp, c_vp, c_vp] + [c_u32] * 4
        L.bh_chan_copy.argtypes = [c_vp, c_vp, c_vp] + [c_u32] * 7
        L.bh_chan_affine.argtypes = [c_vp, c_vp, c_vp, c_vp, c_vp] + [c_u32] * 3 + [ctypes.c_int]
        L.bh_eltwise.argtypes = [c_vp, c_vp, c_vp, c_vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.bh_variant_name.argtypes = [ctypes.c_int, ctypes.POINTER(c_u32), ctypes.c_char_p, ctypes.c_size_t]
        L.bh_variant_name_ctx.argtypes = [c_vp, ctypes.c_int, ctypes.POINTER(c_u32), ctypes.c_char_p, ctypes.c_size_t]
        L.bh_stamp.argtypes = [c_vp, ctypes.c_int]
        L.bh_spin.argtypes = [c_vp, ctypes.c_int]
        L.bh_time_next_call.argtypes = [c_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.bh_stamps_read.argtypes = [c_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.bh_capture_begin.argtypes = [c_vp]
        L.bh_capture_end.argtypes = [c_vp, ctypes.POINTER(ctypes.c_int)]
        L.bh_graph_launch.argtypes = [c_vp, ctypes.c_int]
        L.bh_graph_destroy.argtypes = [c_vp, ctypes.c_int]
        L.bh_tune_set.argtypes = [c_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.bh_tune_set_policy.argtypes = [c_vp, ctypes.c_int, ctypes.c_int]
        L.bh_tune_cfg_name.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
        L.bh_jit_build.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                   ctypes.POINTER(ctypes.c_size_t)]
        _lib = L
    return _lib


def _check(rc):
    if rc != BH_OK:
        msg = lib().bh_last_error().decode(errors="replace")
        raise (UnsupportedError if rc == BH_UNSUP else BodaHipError)(rc, msg)


def device_count():
    n = ctypes.c_int(0)
    _check(lib().bh_device_count(ctypes.byref(n)))
    return n.value


def variant_name(op_kind, dims):
    arr = (c_u32 * 16)(*dims)
    buf = ctypes.create_string_buffer(256)
    _check(lib().bh_variant_name(op_kind, arr, buf, 256))
    return buf.value.decode()


def conv_filts_packed_floats(s, banks=None):
    """Floats of the transformed filter bank for conv shape s: the full pack (bh_conv_filts_pack), or
    with banks (a BANK_* mask) the k-major bank + those Winograd banks (bh_conv_filts_pack_banks)."""
    if banks is None:
        return lib().bh_conv_filts_packed_floats(s.OC, s.IC, s.KY, s.KX)
    return lib().bh_conv_filts_packed_floats_banks(s.OC, s.IC, s.KY, s.KX, banks)


def pool_out_size(n, k, stride, pad):
    return lib().bh_pool_out_size(n, k, stride, pad)


def jit_build(src, opts=""):
    """Compile a device program with hiprtc for gfx950 (no device needed); returns (code bytes, log)."""
    log = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t(0)
    rc = lib().bh_jit_build(src.encode(), opts.encode(), log, len(log), ctypes.byref(n))
    _check(rc)
    return n.value, log.value.decode(errors="replace")


def tune_cfg_names(op_kind):
    """Names of the tile configurations the library instantiates for op_kind (0 sgemm, 1 conv)."""
    out, i = [], 0
    buf = ctypes.create_string_buffer(64)
    while lib().bh_tune_cfg_name(op_kind, i, buf, 64) == BH_OK:
        out.append(buf.value.decode())
        i += 1
    return out


class DevBuf:
    """A device allocation owned by a Device (freed explicitly or with the Device)."""

    def __init__(self, dev, ptr, nbytes):
        self.dev, self.ptr, self.nbytes = dev, ptr, nbytes

    @property
    def nfloats(self):
        return self.nbytes // 4

    def upload(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.float32)
        assert a.nbytes <= self.nbytes
        _check(lib().bh_h2d(self.dev.ctx, self.ptr, a.ctypes.data, a.nbytes))

    def download(self, n=None, out=None):
        n = self.nfloats if n is None else n
        o = np.empty(n, np.float32) if out is None else out
        _check(lib().bh_d2h(self.dev.ctx, o.ctypes.data, self.ptr, n * 4))
        return o

    def zero(self):
        _check(lib().bh_memset0(self.dev.ctx, self.ptr, self.nbytes))

    def free(self):
        if self.ptr:
            _check(lib().bh_free(self.dev.ctx, self.ptr))
            self.dev._bufs.discard(self)
            self.ptr = None


class Device:
    """One bh_ctx: a gfx950 device and its stream."""

    def __init__(self, device=0):
        self.ctx = c_vp()
        _check(lib().bh_init(device, ctypes.byref(self.ctx)))
        self.index = device
        self._bufs = set()

    def close(self):
        if self.ctx:
            for b in list(self._bufs):
                b.free()
            _check(lib().bh_destroy(self.ctx))
            self.ctx = c_vp()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def plat_tag(self):
        buf = ctypes.create_string_buffer(256)
        _check(lib().bh_plat_tag(self.ctx, buf, 256))
        return buf.value.decode()

    def alloc(self, nbytes):
        p = c_vp()
        _check(lib().bh_alloc(self.ctx, nbytes, ctypes.byref(p)))
        b = DevBuf(self, p.value, nbytes)
        self._bufs.add(b)
        return b

    def alloc_floats(self, n):
        return self.alloc(4 * int(n))

    def sync(self):
        _check(lib().bh_sync(self.ctx))

    def event(self):
        i = ctypes.c_int(0)
        _check(lib().bh_event_record(self.ctx, ctypes.byref(i)))
        return i.value

    def elapsed_ms(self, b, e):
        ms = ctypes.c_float(0)
        _check(lib().bh_elapsed_ms(self.ctx, b, e, ctypes.byref(ms)))
        return ms.value

    def events_reset(self):
        _check(lib().bh_events_reset(self.ctx))

    def gen_data(self, kind, buf, dims, mode, vi=0.0):
        d = list(dims) + [1] * (4 - len(dims))
        arr = (c_u32 * 4)(*d)
        _check(lib().bh_gen_data(self.ctx, kind, buf.ptr, arr, mode, vi))

    def time_next_call(self):
        """Arm kernel-dispatch events for the next call; returns (begin id, end id)."""
        b, e = ctypes.c_int(-1), ctypes.c_int(-1)
        _check(lib().bh_time_next_call(self.ctx, ctypes.byref(b), ctypes.byref(e)))
        return b.value, e.value

    def stamp(self, slot):
        _check(lib().bh_stamp(self.ctx, slot))

    def spin(self, us):
        """Enqueue a bounded GPU busy-wait (queue pre-fill before timed batches)."""
        _check(lib().bh_spin(self.ctx, int(us)))

    def stamps_read(self, first, n):
        """Slots first..first+n-1 in microseconds relative to slot first (syncs)."""
        out = (ctypes.c_double * n)()
        _check(lib().bh_stamps_read(self.ctx, first, n, out))
        return list(out)

    def capture_begin(self):
        _check(lib().bh_capture_begin(self.ctx))

    def capture_end(self):
        g = ctypes.c_int(-1)
        _check(lib().bh_capture_end(self.ctx, ctypes.byref(g)))
        return g.value

    def graph_launch(self, g):
        _check(lib().bh_graph_launch(self.ctx, g))

    def graph_destroy(self, g):
        _check(lib().bh_graph_destroy(self.ctx, g))

    def tune_set(self, op_kind, cfg_index=-1, splits=0):
        _check(lib().bh_tune_set(self.ctx, op_kind, cfg_index, splits))

    def variant(self, op_kind, dims):
        """The kernel variant a call on this context runs now (with its tune overrides)."""
        arr = (c_u32 * 16)(*dims)
        buf = ctypes.create_string_buffer(256)
        _check(lib().bh_variant_name_ctx(self.ctx, op_kind, arr, buf, 256))
        return buf.value.decode()

    def tune_set_policy(self, op_kind, wt=-1):
        """Output store policy override: 1 write-through, 0 write-back, -1 the table's choice."""
        _check(lib().bh_tune_set_policy(self.ctx, op_kind, wt))

    def sgemm(self, a, b, c, M, N, K):
        _check(lib().bh_sgemm_kmajor(self.ctx, a.ptr, b.ptr, c.ptr, M, N, K))

    def conv(self, inp, filts, biases, out, s, relu=1, packed=None):
        """bh_conv2d_fwd_nchw; with packed (a bank made by conv_filts_pack) bh_conv2d_fwd_nchw_pk."""
        bp = biases.ptr if biases is not None else None
        if packed is None:
            _check(lib().bh_conv2d_fwd_nchw(self.ctx, inp.ptr, filts.ptr, bp, out.ptr, s.B, s.IC, s.H, s.W, s.OC,
                                            s.KY, s.KX, s.sy, s.sx, s.py, s.px, int(relu)))
        else:
            _check(lib().bh_conv2d_fwd_nchw_pk(self.ctx, inp.ptr, filts.ptr, packed.ptr, bp, out.ptr, s.B, s.IC, s.H,
                                               s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px, int(relu)))

    def conv_res(self, inp, filts, biases, res, out, s, relu=1, packed=None):
        """bh_conv2d_fwd_nchw_res: out = relu(conv + bias + res)."""
        _check(lib().bh_conv2d_fwd_nchw_res(self.ctx, inp.ptr, filts.ptr, packed.ptr if packed is not None else None,
                                            biases.ptr if biases is not None else None, res.ptr, out.ptr, s.B, s.IC,
                                            s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px, int(relu)))

    def conv_slab(self, inp, filts, biases, out, out_chans_total, out_chan_ofs, s, relu=1, packed=None):
        """bh_conv2d_fwd_nchw_slab: channels out_chan_ofs .. +OC of a B x out_chans_total x OH x OW output."""
        _check(lib().bh_conv2d_fwd_nchw_slab(self.ctx, inp.ptr, filts.ptr, packed.ptr if packed is not None else None,
                                             biases.ptr if biases is not None else None, out.ptr, out_chans_total,
                                             out_chan_ofs, s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py,
                                             s.px, int(relu)))

    # ---- the other forward layers (bh_fwdops.hip)
    def pool(self, inp, out, B, C, H, W, KY, KX, sy, sx, py, px, avg, out_in_yx=None):
        _check(lib().bh_pool_fwd_nchw(self.ctx, inp.ptr, out.ptr, out_in_yx.ptr if out_in_yx is not None else None,
                                      B, C, H, W, KY, KX, sy, sx, py, px, int(avg)))

    def lrn(self, inp, out, B, C, H, W, local_size, alpha, beta, k, out_scale_base=None):
        _check(lib().bh_lrn_fwd_nchw(self.ctx, inp.ptr, out.ptr,
                                     out_scale_base.ptr if out_scale_base is not None else None,
                                     B, C, H, W, local_size, alpha, beta, k))

    def relu(self, x, n):
        _check(lib().bh_relu_inplace(self.ctx, x.ptr, n))

    def dropout(self, x, n, ratio, seed):
        _check(lib().bh_dropout_inplace(self.ctx, x.ptr, n, ratio, seed))

    def softmax(self, inp, prob, B, C, H, W):
        _check(lib().bh_softmax_chans(self.ctx, inp.ptr, prob.ptr, B, C, H, W))

    def chan_copy(self, inp, out, B, HW, in_c, ic0, out_c, oc0, nc):
        _check(lib().bh_chan_copy(self.ctx, inp.ptr, out.ptr, B, HW, in_c, ic0, out_c, oc0, nc))

    def chan_affine(self, inp, out, scale, shift, B, C, HW, relu=0):
        _check(lib().bh_chan_affine(self.ctx, inp.ptr, out.ptr, scale.ptr, shift.ptr, B, C, HW, int(relu)))

    def eltwise(self, a, b, out, n, op=1, relu=0):
        _check(lib().bh_eltwise(self.ctx, a.ptr, b.ptr, out.ptr, n, op, int(relu)))

    def conv_filts_pack(self, filts, packed, s, banks=None):
        """Boda's xpose_filts counterpart: write the k-major bank of filts (+ the Winograd banks: all of
        the kernel size's, or those of the mask banks) into packed."""
        if banks is None:
            _check(lib().bh_conv_filts_pack(self.ctx, filts.ptr, packed.ptr, s.OC, s.IC, s.KY, s.KX))
        else:
            _check(lib().bh_conv_filts_pack_banks(self.ctx, filts.ptr, packed.ptr, s.OC, s.IC, s.KY, s.KX, banks))

    def route_banks(self, s):
        """The Winograd bank mask the route of conv shape s on this context reads (0: k-major only)."""
        arr = (c_u32 * 11)(*s.as_dims())
        b = c_u32(0)
        _check(lib().bh_conv_route_banks(self.ctx, arr, ctypes.byref(b)))
        return b.value

    def conv_pkb(self, inp, filts, packed, banks, biases, out, s, relu=1, res=None, out_chans_total=0,
                 out_chan_ofs=0):
        """bh_conv2d_fwd_nchw_pkb: packed (may be None) holds the k-major bank + the banks of mask banks."""
        _check(lib().bh_conv2d_fwd_nchw_pkb(self.ctx, inp.ptr, filts.ptr, packed.ptr if packed is not None else None,
                                            banks, biases.ptr if biases is not None else None,
                                            res.ptr if res is not None else None, out.ptr, out_chans_total,
                                            out_chan_ofs, s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py,
                                            s.px, int(relu)))
