#!/usr/bin/env python3
"""Which side of a cnn_op_info MAD miss is off: ours (libboda_hip) and the comparator (rocBLAS /
MIOpen) against float64 on the same gen_data inputs, max min_sig_mag_rel_diff(1, ., .) each.
  python3 tools/vendor_acc.py   (GPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "boda-1_amd"))
sys.path.insert(0, ROOT)
import boda_hip  # noqa: E402
from boda_hip import GEN_CONV_BIASES, GEN_CONV_FILTS, GEN_CONV_IN, GEN_SGEMM_A, GEN_SGEMM_B, ops, vendor  # noqa: E402


def msr(ref, x):
    return float(np.max(np.abs(x - ref) / np.maximum(1.0, np.maximum(np.abs(ref), np.abs(x)))))


dev = boda_hip.Device(0)
vd = vendor.Vendor(0)
for n, mode in [(512, 5), (1536, 5), (2048, 5), (2048, 600)]:
    M = N = K = n
    a, b, c1, c2 = dev.alloc_floats(K * M), dev.alloc_floats(K * N), dev.alloc_floats(M * N), dev.alloc_floats(M * N)
    dev.gen_data(GEN_SGEMM_A, a, [K, M], mode)
    dev.gen_data(GEN_SGEMM_B, b, [K, N], mode)
    dev.sgemm(a, b, c1, M, N, K)
    dev.sync()
    vd.sgemm(a.ptr, b.ptr, c2.ptr, M, N, K)
    vd.sync()
    A = a.download().reshape(K, M).astype(np.float64)
    B = b.download().reshape(K, N).astype(np.float64)
    ref = A.T @ B
    o, v = c1.download().reshape(M, N), c2.download().reshape(M, N)
    print("sgemm %d mode %d: ours %.3g  vendor %.3g  ours-vs-vendor %.3g" % (n, mode, msr(ref, o), msr(ref, v),
                                                                           msr(o.astype(np.float64), v)), flush=True)
    for x in (a, b, c1, c2):
        x.free()


def conv64(x, f, b, s):  # float64 conv + bias + ReLU, NCHW
    xp = np.pad(x, ((0, 0), (0, 0), (s.py, s.py), (s.px, s.px)))
    out = np.zeros((s.B, s.OC, s.OH, s.OW))
    for ky in range(s.KY):
        for kx in range(s.KX):
            win = xp[:, :, ky:ky + s.sy * (s.OH - 1) + 1:s.sy, kx:kx + s.sx * (s.OW - 1) + 1:s.sx]
            out += np.einsum("bchw,oc->bohw", win, f[:, :, ky, kx])
    return np.maximum(out + b[None, :, None, None], 0)


for dims in [(5, 64, 14, 14, 64, 3, 3, 1, 1, 1, 1), (20, 3, 227, 227, 96, 11, 11, 4, 4, 0, 0),
             (5, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2), (20, 96, 27, 27, 256, 5, 5, 1, 1, 2, 2),
             (20, 64, 56, 56, 192, 3, 3, 1, 1, 1, 1), (20, 32, 28, 28, 96, 5, 5, 1, 1, 2, 2),
             (20, 384, 13, 13, 384, 3, 3, 1, 1, 1, 1)]:
    s = ops.ConvShape(*dims)
    i, f, b = dev.alloc_floats(s.B * s.IC * s.H * s.W), dev.alloc_floats(s.OC * s.IC * s.KY * s.KX), \
        dev.alloc_floats(s.OC)
    o1, o2 = dev.alloc_floats(s.B * s.OC * s.OH * s.OW), dev.alloc_floats(s.B * s.OC * s.OH * s.OW)
    dev.gen_data(GEN_CONV_IN, i, [s.B, s.IC, s.H, s.W], 5)
    dev.gen_data(GEN_CONV_FILTS, f, [s.OC, s.IC, s.KY, s.KX], 5)
    dev.gen_data(GEN_CONV_BIASES, b, [s.OC, 1, 1, 1], 5)
    dev.conv(i, f, b, o1, s, relu=1)
    dev.sync()
    vd.conv(i.ptr, f.ptr, b.ptr, o2.ptr, s, relu=1)
    vd.sync()
    ref = conv64(i.download().reshape(s.B, s.IC, s.H, s.W).astype(np.float64),
                 f.download().reshape(s.OC, s.IC, s.KY, s.KX).astype(np.float64), b.download().astype(np.float64), s)
    o, v = o1.download().reshape(ref.shape), o2.download().reshape(ref.shape)
    nm = lambda x: float(np.max(np.abs(x - ref)) / np.max(np.abs(ref)))  # noqa: E731  (the tests' normalized max)
    print("conv %s [%s]: ours %.3g (norm-max %.2g)  vendor %.3g (norm-max %.2g)  ours-vs-vendor %.3g"
          % (list(dims), boda_hip.variant_name(1, s.as_dims()), msr(ref, o), nm(o),
             msr(ref, v), nm(v), msr(o.astype(np.float64), v)), flush=True)
    for x in (i, f, b, o1, o2):
        x.free()
vd.close()
dev.close()
