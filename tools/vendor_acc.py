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
from boda_hip import GEN_SGEMM_A, GEN_SGEMM_B, vendor  # noqa: E402


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
vd.close()
dev.close()
