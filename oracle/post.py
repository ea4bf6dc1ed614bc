"""CPU oracle of the post-processing stage (TEST INFRASTRUCTURE ONLY: imported by tests/ as the
checker, never by the product).  numpy float32 restatement of PostProcessor::Render
(DXRPathTracer/PostProcessor.cpp:43-92) and DXRPathTracer/PostProcessing.hlsl:

  bloom_down   Bloom (:83-99): GatherRed/Green/Blue(LinearSampler) at the half-res texel centre,
               (((0 + c0) + c1) + c2) + c3, / 4, stored RGBA16F (PostProcessor.cpp:62)
  blur         Blur (:29-54) with BlurH / BlurV (:110-118), taps i = -7..6, not normalised; H, V, H, V
               (PostProcessor.cpp:74-85), each pass stored RGBA16F
  tonemap      ToneMap (:121-137) + ToneMapFilmicALU (:57-62)

Sampler semantics are those defined in dxrpathtracer_amd/csrc/post_kernels.hip (D3D leaves filter
precision to the hardware, so they are parity-unpinned against the reference's GPU): clamp addressing,
point texel = floor(coord * size), bilinear at coord * size - 0.5 with float weights, Gather order
(x0,y1), (x1,y1), (x1,y0), (x0,y0).  Weights and exposure factors are computed in double and rounded to
float, as dxrpt_post_process does on the host.
"""
import math

import numpy as np

f32 = np.float32


def weights(sigma):
    g = 1.0 / math.sqrt(2.0 * 3.14159 * float(sigma) * float(sigma))
    return np.array([g * math.exp(-float(d * d) / (2.0 * float(sigma) * float(sigma))) for d in range(-7, 7)],
                    dtype=np.float32)


def _centres(n):
    return (np.arange(n, dtype=np.float32) + f32(0.5)) / f32(n)


def bloom_down(img):
    """img: (H, W, 4) float32 -> (H//2, W//2, 4) float16."""
    H, W = img.shape[:2]
    bh, bw = H // 2, W // 2
    u, v = _centres(bw), _centres(bh)
    x0 = np.floor(u * f32(W) - f32(0.5)).astype(np.int64)
    y0 = np.floor(v * f32(H) - f32(0.5)).astype(np.int64)
    xa, xb = np.clip(x0, 0, W - 1), np.clip(x0 + 1, 0, W - 1)
    ya, yb = np.clip(y0, 0, H - 1), np.clip(y0 + 1, 0, H - 1)
    c0 = img[yb][:, xa, :3]
    c1 = img[yb][:, xb, :3]
    c2 = img[ya][:, xb, :3]
    c3 = img[ya][:, xa, :3]
    r = np.zeros_like(c0)
    r = (((r + c0) + c1) + c2) + c3
    out = np.ones((bh, bw, 4), dtype=np.float32)
    out[..., :3] = r / f32(4.0)
    return out.astype(np.float16)


def blur(img16, horizontal, w):
    """One Blur pass of an (h, w, 4) float16 image along x or y; returns float16."""
    h, wd = img16.shape[:2]
    src = img16.astype(np.float32)
    u, v = _centres(wd), _centres(h)
    c = np.zeros((h, wd, 4), dtype=np.float32)
    for k in range(14):
        t = k - 7
        if horizontal:
            tu = u + (f32(t) / f32(wd)) * f32(1.0)
            sx = np.clip(np.floor(tu * f32(wd)).astype(np.int64), 0, wd - 1)
            s = src[:, sx, :]
        else:
            tv = v + (f32(t) / f32(h)) * f32(1.0)
            sy = np.clip(np.floor(tv * f32(h)).astype(np.int64), 0, h - 1)
            s = src[sy, :, :]
        c = c + s * w[k]
    return c.astype(np.float16)


def filmic(c):
    c = np.maximum(f32(0.0), c - f32(0.004))
    return (c * (f32(6.2) * c + f32(0.5))) / (c * (f32(6.2) * c + f32(1.7)) + f32(0.06))


def post_process(img, exposure=-14.0, bloom_exposure=-4.0, bloom_magnitude=1.0, bloom_sigma=2.5, rgba8=False):
    """img: (H, W, 4) float32 accumulation buffer -> (H, W, 4) float32 (or uint8 when rgba8)."""
    img = np.asarray(img, dtype=np.float32)
    H, W = img.shape[:2]
    w = weights(bloom_sigma)
    b = bloom_down(img)
    for _ in range(2):
        b = blur(b, True, w)
        b = blur(b, False, w)
    bh, bw = b.shape[:2]
    bf = b.astype(np.float32)
    u, v = _centres(W), _centres(H)
    tx, ty = u * f32(bw) - f32(0.5), v * f32(bh) - f32(0.5)
    fx0, fy0 = np.floor(tx), np.floor(ty)
    fx, fy = (tx - fx0)[None, :, None], (ty - fy0)[:, None, None]
    xa, xb = np.clip(fx0.astype(np.int64), 0, bw - 1), np.clip(fx0.astype(np.int64) + 1, 0, bw - 1)
    ya, yb = np.clip(fy0.astype(np.int64), 0, bh - 1), np.clip(fy0.astype(np.int64) + 1, 0, bh - 1)
    t00, t10 = bf[ya][:, xa], bf[ya][:, xb]
    t01, t11 = bf[yb][:, xa], bf[yb][:, xb]

    def lerp(a, c, t):
        return a + t * (c - a)

    bl = lerp(lerp(t00, t10, fx), lerp(t01, t11, fx), fy)[..., :3]
    mag = f32(bloom_magnitude)
    e2 = f32(np.exp2(np.float64(bloom_exposure)))
    scale = f32(np.exp2(np.float64(exposure)) / 0.0009765625)
    col = img[..., :3] + (bl * mag) * e2
    col = filmic(col * scale)
    if rgba8:
        q = np.rint(np.clip(col, 0.0, 1.0) * f32(255.0)).astype(np.uint8)
        out = np.full((H, W, 4), 255, dtype=np.uint8)
        out[..., :3] = q
        return out
    out = np.ones((H, W, 4), dtype=np.float32)
    out[..., :3] = col
    return out
