"""CPU: properties of the post-processing oracle (oracle/post.py), the checker of dxrpt_post_process."""
import numpy as np

from oracle import post as P


def test_weights_are_the_reference_gaussian():
    w = P.weights(2.5)
    assert w.shape == (14,)
    assert np.argmax(w) == 7  # tap i = 0
    np.testing.assert_allclose(w[7 - 3], w[7 + 3], rtol=1e-7)  # symmetric where both taps exist
    assert 0.99 < float(w.sum()) < 1.0  # 14 taps of a unit-area Gaussian, tap +7 missing


def test_bloom_down_averages_each_2x2_block():
    rng = np.random.default_rng(1)
    img = rng.uniform(0, 4, size=(8, 10, 4)).astype(np.float32)
    b = P.bloom_down(img).astype(np.float32)
    assert b.shape == (4, 5, 4)
    ref = img[..., :3].reshape(4, 2, 5, 2, 3).mean(axis=(1, 3))
    np.testing.assert_allclose(b[..., :3], ref, rtol=2e-3)
    assert (b[..., 3] == 1.0).all()


def test_blur_of_constant_is_constant_times_weight_sum():
    w = P.weights(2.5)
    img = np.full((6, 20, 4), 0.5, dtype=np.float16)
    for horizontal in (True, False):
        out = P.blur(img, horizontal, w).astype(np.float32)
        np.testing.assert_allclose(out, 0.5 * float(w.sum()), rtol=1e-3)


def test_tonemap_curve():
    assert P.filmic(np.float32(0.0)) == 0.0
    x = np.linspace(0, 10, 101, dtype=np.float32)
    y = P.filmic(x)
    assert (np.diff(y) >= 0).all() and y[-1] < 1.0
    # black stays black through the whole stage
    out = P.post_process(np.zeros((4, 4, 4), dtype=np.float32))
    assert (out[..., :3] == 0).all() and (out[..., 3] == 1).all()
    q = P.post_process(np.zeros((4, 4, 4), dtype=np.float32), rgba8=True)
    assert q.dtype == np.uint8 and (q[..., :3] == 0).all() and (q[..., 3] == 255).all()
