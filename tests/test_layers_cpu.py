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
