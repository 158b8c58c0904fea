"""Known answers for the CPU restatements of the non-conv forward layers (oracle/layers.py),
worked by hand from the reference kernels (test/rtc/{pool,lrn,softmax,relu}.cucl) and the
size rules (src/conv_util.cc:167-204). These pin the checker the GPU layer tests use."""
import numpy as np

from oracle import layers as L


def test_pool_out_size_caffe_ceil():
    # AlexNet pool1: 55 -> 27 (k3 s2); GoogLeNet pool1: 112 -> 56 (k3 s2), ceil rule
    assert L.pool_out_sz(55, 3, 2, 0) == 27
    assert L.pool_out_sz(112, 3, 2, 0) == 56
    assert L.pool_out_sz(13, 3, 2, 0) == 6
    assert L.pool_out_sz(14, 3, 2, 0) == 7   # conv rule would give 6
    assert L.conv_out_sz(14, 3, 2, 0) == 6
    assert L.pool_out_sz(2, 3, 1, 0) == 1    # padded input smaller than the window


def test_max_pool_known_answer():
    x = np.arange(16, dtype=np.float32).reshape(1, 1, 4, 4)
    out, arg = L.pool(x, 3, 3, 2, 2, 0, 0, avg=False)
    # windows rows/cols {0-2},{2-3(partial)}
    assert out.shape == (1, 1, 2, 2)
    np.testing.assert_array_equal(out[0, 0], [[10, 11], [14, 15]])
    np.testing.assert_array_equal(arg[0, 0], [[10, 11], [14, 15]])


def test_avg_pool_counts_only_in_image_taps():
    x = np.ones((1, 1, 3, 3), dtype=np.float32)
    x[0, 0, 0, 0] = 4.0
    out, _ = L.pool(x, 2, 2, 1, 1, 1, 1, avg=True)
    # top-left window covers only (0,0): mean 4; next covers (0,0),(0,1): (4+1)/2
    assert out[0, 0, 0, 0] == 4.0 and out[0, 0, 0, 1] == 2.5
    assert out.shape == (1, 1, 4, 4)


def test_lrn_known_answer():
    x = np.array([1, 2, 3], dtype=np.float32).reshape(1, 3, 1, 1)
    out, sb = L.lrn(x, 3, 3.0, 1.0, 1.0)
    # sums of squares over windows {0,1},{0,1,2},{1,2}: 5, 14, 13; base = 1 + sum * (3/3)
    np.testing.assert_allclose(sb[0, :, 0, 0], [6, 15, 14])
    np.testing.assert_allclose(out[0, :, 0, 0], [1 / 6, 2 / 15, 3 / 14], rtol=1e-6)


def test_softmax_and_relu():
    x = np.array([-1, 0, 2], dtype=np.float32).reshape(1, 3, 1, 1)
    p = L.softmax(x)[0, :, 0, 0]
    e = np.exp([-3.0, -2.0, 0.0])
    np.testing.assert_allclose(p, e / e.sum(), rtol=1e-6)
    np.testing.assert_array_equal(L.relu(x)[0, :, 0, 0], [0, 0, 2])


def _murmur_fmix32(h):
    """Reference scalar form (test/rtc/dropout.cucl:12-17), for the known answers below."""
    h &= 0xffffffff
    h ^= h >> 16
    h = (h * 0x85ebca6b) & 0xffffffff
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & 0xffffffff
    h ^= h >> 16
    return h


def test_dropout_known_answer():
    x = np.arange(1, 65, dtype=np.float32).reshape(1, 4, 4, 4)
    for seed in (0, 7, 0xfffffff0):
        got = L.dropout(x, 0.5, seed).reshape(-1)
        for i, v in enumerate(x.reshape(-1)):
            keep = _murmur_fmix32(i + seed) > 2147483647  # (uint32)(U32_MAX * 0.5)
            assert got[i] == (v * np.float32(2.0) if keep else 0.0), (seed, i)
        kept = (got != 0).mean()
        assert 0.3 < kept < 0.7
    # murmur3's finalizer maps 0 to 0: element 0 at seed 0 is always dropped
    assert L.dropout(x, 0.25, 0).reshape(-1)[0] == 0
    # ratio 0.25: survivors scaled by 4/3 in fp32
    y = L.dropout(x, 0.25, 3).reshape(-1)
    nz = y != 0
    np.testing.assert_array_equal(y[nz], x.reshape(-1)[nz] * np.float32(1.0 / 0.75))
