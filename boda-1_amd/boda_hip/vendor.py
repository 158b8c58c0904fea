"""Same-node comparator: rocBLAS SGEMM and MIOpen conv forward through libboda_hip_vendor.so
(include/boda_hip_vendor.h) -- the role of the reference's culibs-wrap intercepts
(src/culibs-wrap.cc:94-242) as cnn_op_info's use_culibs comparator runs them
(src/cnn-prof.cc:40,90-91). Context only: the product path never imports this module.
"""
import ctypes
import os

from . import ops

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                        "libboda_hip_vendor.so")
EXPORTS = ["bhv_last_error", "bhv_init", "bhv_destroy", "bhv_sync", "bhv_sgemm_kmajor", "bhv_conv2d_fwd_nchw",
           "bhv_time_sgemm", "bhv_time_conv"]

_lib = None
c_vp = ctypes.c_void_p
u32 = ctypes.c_uint32


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("%s is not built (make -C boda-1_amd vendor)" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        L.bhv_last_error.restype = ctypes.c_char_p
        L.bhv_init.argtypes = [ctypes.c_int, ctypes.POINTER(c_vp)]
        L.bhv_destroy.argtypes = [c_vp]
        L.bhv_sync.argtypes = [c_vp]
        L.bhv_sgemm_kmajor.argtypes = [c_vp, c_vp, c_vp, c_vp, u32, u32, u32]
        L.bhv_conv2d_fwd_nchw.argtypes = [c_vp] + [c_vp] * 4 + [u32] * 11 + [ctypes.c_int]
        L.bhv_time_sgemm.argtypes = [c_vp, u32, u32, u32, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.bhv_time_conv.argtypes = ([c_vp] + [u32] * 11 + [ctypes.c_int, ctypes.c_int] +
                                    [ctypes.POINTER(ctypes.c_float)] * 3 + [ctypes.c_char_p, ctypes.c_size_t])
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("boda_hip_vendor: " + lib().bhv_last_error().decode())


class Vendor:
    """One bhv_ctx (rocBLAS + MIOpen handles on their own stream of `device`)."""

    def __init__(self, device=0):
        self.ctx = c_vp()
        _check(lib().bhv_init(device, ctypes.byref(self.ctx)))

    def close(self):
        if self.ctx:
            _check(lib().bhv_destroy(self.ctx))
            self.ctx = c_vp()

    def sync(self):
        _check(lib().bhv_sync(self.ctx))

    def sgemm(self, a, b, c, M, N, K):
        _check(lib().bhv_sgemm_kmajor(self.ctx, a, b, c, M, N, K))

    def conv(self, inp, filts, biases, out, s, relu=1):
        _check(lib().bhv_conv2d_fwd_nchw(self.ctx, inp, filts, biases, out, *s.as_dims(), relu))

    def time(self, shape, reps):
        """{"ms": per-call ms, ...} for one op shape (amortized over reps back-to-back calls)."""
        ms = ctypes.c_float(0)
        if isinstance(shape, ops.SgemmShape):
            _check(lib().bhv_time_sgemm(self.ctx, shape.M, shape.N, shape.K, reps, ctypes.byref(ms)))
            return {"ms": ms.value, "lib": "rocblas_sgemm"}
        conv_only, find = ctypes.c_float(0), ctypes.c_float(0)
        algo = ctypes.create_string_buffer(32)
        _check(lib().bhv_time_conv(self.ctx, *shape.as_dims(), 1, reps, ctypes.byref(ms), ctypes.byref(conv_only),
                                   ctypes.byref(find), algo, 32))
        return {"ms": ms.value, "conv_only_ms": conv_only.value, "find_ms": find.value,
                "lib": "miopen:" + algo.value.decode()}
