"""CPU restatements (numpy, fp32 in the reference's operation order) of the non-conv forward
layers of Boda's net executor, plus the net-level size rules.

*** TEST INFRASTRUCTURE ONLY *** -- imported by tests/ as the checker of the HIP kernels in
boda-1_amd/csrc/bh_fwdops.hip and of the net executor (boda-1_amd/host/conv_pipe.*), never
by the product path. Each function cites the reference file:line it restates.

Parity pinning: the reference ships no digests for these layers (its known-good digests,
test/good_tr/, cover conv and sgemm only) and the reference cannot be built here (SURVEY
F2), so these restatements are "parity unpinned" in the sense of the task: they follow the
reference kernel source line by line and are checked by hand-computed known answers in
tests/test_layers_cpu.py.
"""
import numpy as np

F32 = np.float32
FLT_MAX = np.finfo(np.float32).max


def pool_out_sz(n, k, s, p):
    """Caffe pooling output size: a partial last window adds an output
    (src/conv_util.cc:198-204: ceil_div(in + 2p - k, s) + 1; 1 when the padded input is
    smaller than the window)."""
    pin = n + 2 * p
    if pin < k:
        return 1
    return -(-(pin - k) // s) + 1


def conv_out_sz(n, k, s, p):
    """src/conv_util.cc:167-173 (floor)."""
    return (n + 2 * p - k) // s + 1


def pool(x, KY, KX, sy, sx, py, px, avg):
    """test/rtc/pool.cucl:12-39: only in-image taps count (max and average); loop order kx
    outer, ky inner decides the summation order and max ties. Returns (out, out_in_yx)."""
    B, C, H, W = x.shape
    OH, OW = pool_out_sz(H, KY, sy, py), pool_out_sz(W, KX, sx, px)
    out = np.full((B, C, OH, OW), F32(0) if avg else F32(-FLT_MAX), dtype=F32)
    cnt = np.zeros((OH, OW), dtype=F32)
    arg = np.full((B, C, OH, OW), -1.0, dtype=F32)
    oy = np.arange(OH)[:, None]
    ox = np.arange(OW)[None, :]
    for kx in range(KX):
        for ky in range(KY):
            iy = oy * sy + ky - py
            ix = ox * sx + kx - px
            ok = (iy >= 0) & (ix >= 0) & (iy < H) & (ix < W)
            iyc, ixc = np.clip(iy, 0, H - 1), np.clip(ix, 0, W - 1)
            v = x[:, :, iyc, ixc]  # B, C, OH, OW
            if avg:
                out = np.where(ok, out + v, out).astype(F32)
                cnt = cnt + ok.astype(F32)
            else:
                better = ok & (v > out)
                out = np.where(better, v, out)
                arg = np.where(better, (iyc * W + ixc).astype(F32), arg)
    if avg:
        out = (out / cnt).astype(F32)
    return out, arg


def lrn(x, local_size, alpha, beta, k):
    """test/rtc/lrn.cucl:30-48 (LRN_MATCH_CAFFE): running sum of squares over a window of
    local_size channels, + new^2 then - old^2, scale_base = k + sum * (alpha/ls),
    out = x * scale_base^-beta. Returns (out, scale_base)."""
    B, C, H, W = x.shape
    hls = local_size >> 1
    a = F32(F32(alpha) / F32(local_size))
    ring = np.zeros((local_size, B, H, W), dtype=F32)
    s = np.zeros((B, H, W), dtype=F32)
    out = np.empty_like(x)
    sb_all = np.empty_like(x)
    for c in range(C + hls):
        j = c % local_size
        old = ring[j].copy()
        ring[j] = x[:, c] if c < C else 0.0
        s = (s + ring[j] * ring[j]).astype(F32)
        s = (s - old * old).astype(F32)
        if c >= hls:
            oc = c - hls
            sb = (F32(k) + s * a).astype(F32)
            sb_all[:, oc] = sb
            out[:, oc] = ring[(j + local_size - hls) % local_size] * np.power(sb, F32(-beta), dtype=F32)
    return out, sb_all


def relu(x):
    """test/rtc/relu.cucl:4: x <= 0 -> 0."""
    return np.where(x <= 0, F32(0), x).astype(F32)


def dropout(x, ratio, seed):
    """test/rtc/dropout.cucl:7-19: element i (flat index) kept and scaled by 1 / (1 - ratio) iff the
    murmur3 finalizer of (i + det_drop_seed) exceeds U32_MAX * ratio (the ratio is substituted
    into the kernel text, so both products are double), else 0."""
    m = 0xffffffff
    h = (np.arange(x.size, dtype=np.uint64) + np.uint64(seed)) & m
    h ^= h >> 16
    h = (h * 0x85ebca6b) & m
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & m
    h ^= h >> 16
    r = float(F32(ratio))
    thresh = int(4294967295.0 * r)
    scale = F32(1.0 / (1.0 - r))
    flat = x.reshape(-1).astype(F32)
    return np.where(h > thresh, flat * scale, F32(0)).astype(F32).reshape(x.shape)


def softmax(x):
    """test/rtc/softmax.cucl:8-22: max starts at 0, exp(x - max), divide by the sum (channel
    order)."""
    mx = np.maximum(F32(0), x.max(axis=1, keepdims=True))
    e = np.exp((x - mx).astype(F32)).astype(F32)
    ssum = np.zeros(x.shape[:1] + x.shape[2:], dtype=F32)
    for c in range(x.shape[1]):
        ssum = (ssum + e[:, c]).astype(F32)
    return (e / ssum[:, None]).astype(F32)


def concat(xs):
    """Concat along channels (src/rtc_fwd.cc:267-281 + test/rtc/copy.cucl)."""
    return np.concatenate(xs, axis=1)
