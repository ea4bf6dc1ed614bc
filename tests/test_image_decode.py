"""Texture-file decoding for scene ingest (LoadTexture, Graphics/Textures.cpp:38-172; WIC in the reference):
PNG of every colour type and bit depth, Adam7, palettes with tRNS -- lossless, so checked texel for
texel -- and sequential JPEG against libjpeg (PIL's decoder) within +-4 per channel (the IDCT rounding
differs; WIC's own decoder is unspecified, so JPEG texels are parity-unpinned against the reference).
The reference's own PNG/JPEG assets (theInn, Stronghold) are decoded when the checkout is present.
"""
import glob
import io
import os

import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from tests import image_util as I

REF = "/root/reference/Content/Models"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
PIL = pytest.importorskip("PIL.Image")


def _rng(seed=1):
    return np.random.default_rng(seed)


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("ctype,depth", [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16), (2, 8), (2, 16), (3, 1), (3, 2),
                                         (3, 4), (3, 8), (4, 8), (4, 16), (6, 8), (6, 16)])
def test_png_all_formats_exact(tmp_path, ctype, depth, interlace):
    rng = _rng(ctype * 100 + depth)
    h, w = 13, 21  # odd sizes: partial Adam7 passes, partial bytes at low depths
    nc = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    top = (1 << depth) - 1
    samples = rng.integers(0, top + 1, size=(h, w, nc))
    palette = trns = None
    if ctype == 3:
        n = 1 << depth
        palette = rng.integers(0, 256, size=(n, 3))
        trns = bytes(rng.integers(0, 256, size=n // 2 + 1).astype(np.uint8))
    path = tmp_path / f"t{ctype}_{depth}_{int(interlace)}.png"
    I.write_png(path, samples, ctype, depth, palette=palette, trns=trns, interlace=interlace, seed=ctype + depth)
    got, fmt = I.decode(path)
    assert fmt == A.TEX_RGBA8_UNORM and got.shape == (h, w, 4)
    to8 = (lambda v: v >> 8) if depth == 16 else ((lambda v: v) if depth == 8 else (lambda v: v * 255 // top))
    want = np.zeros((h, w, 4), np.int64)
    want[..., 3] = 255
    if ctype == 3:
        idx = samples[..., 0]
        want[..., :3] = palette[idx]
        alpha = np.full(1 << depth, 255)
        alpha[:len(trns)] = list(trns)
        want[..., 3] = alpha[idx]
    elif ctype in (0, 4):
        want[..., 0] = want[..., 1] = want[..., 2] = to8(samples[..., 0])
        if ctype == 4:
            want[..., 3] = to8(samples[..., 1])
    else:
        want[..., :3] = to8(samples[..., :3])
        if ctype == 6:
            want[..., 3] = to8(samples[..., 3])
    np.testing.assert_array_equal(got, want)


def test_png_matches_pil_and_srgb_flag(tmp_path):
    img = (_rng(3).random((40, 56, 4)) * 255).astype(np.uint8)
    path = tmp_path / "rgba.png"
    PIL.fromarray(img, "RGBA").save(path)
    got, fmt = I.decode(path, srgb=True)
    assert fmt == A.TEX_RGBA8_SRGB
    np.testing.assert_array_equal(got, img)


def _smooth_image(h, w, seed):
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    r = 128 + 100 * np.sin(x / 7.0 + seed) * np.cos(y / 11.0)
    g = 128 + 90 * np.cos((x + y) / 9.0)
    b = 128 + 80 * np.sin(y / 5.0 - seed)
    noise = _rng(seed).normal(0, 6, size=(h, w, 3))
    return np.clip(np.stack([r, g, b], -1) + noise, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("mode,subsampling", [("RGB", 0), ("RGB", 1), ("RGB", 2), ("L", 0)])
def test_jpeg_matches_libjpeg(tmp_path, mode, subsampling):
    img = _smooth_image(77, 130, subsampling + 1)  # not a multiple of the MCU: edge blocks
    pil = PIL.fromarray(img if mode == "RGB" else img[..., 0], mode)
    buf = io.BytesIO()
    pil.save(buf, "JPEG", quality=90, subsampling=subsampling)
    path = tmp_path / f"t_{mode}_{subsampling}.jpg"
    path.write_bytes(buf.getvalue())
    got, fmt = I.decode(path)
    ref = np.asarray(PIL.open(path).convert("RGBA")).astype(int)
    d = np.abs(got.astype(int) - ref)
    assert got.shape == ref.shape and fmt == A.TEX_RGBA8_UNORM
    assert d.max() <= 4 and d.mean() < 0.2, (d.max(), d.mean())
    assert (got[..., 3] == 255).all()


def test_jpeg_restart_intervals(tmp_path):
    # DRI + RSTn markers (PIL has no restart option: insert them by re-encoding through the decoder's
    # inverse is not available, so use libjpeg's own encoder via PIL's `restart_marker_blocks`)
    img = _smooth_image(64, 96, 9)
    buf = io.BytesIO()
    try:
        PIL.fromarray(img, "RGB").save(buf, "JPEG", quality=85, restart_marker_blocks=3)
    except TypeError:
        pytest.skip("PIL without restart-marker support")
    data = buf.getvalue()
    if b"\xff\xdd" not in data:
        pytest.skip("encoder wrote no restart markers")
    path = tmp_path / "rst.jpg"
    path.write_bytes(data)
    got, _ = I.decode(path)
    ref = np.asarray(PIL.open(path).convert("RGBA")).astype(int)
    assert np.abs(got.astype(int) - ref).max() <= 4


def test_unsupported_images_fail_loudly(tmp_path):
    buf = io.BytesIO()
    PIL.fromarray(_smooth_image(32, 32, 2), "RGB").save(buf, "JPEG", progressive=True)
    (tmp_path / "p.jpg").write_bytes(buf.getvalue())
    with pytest.raises(RuntimeError, match="progressive"):
        I.decode(tmp_path / "p.jpg")
    (tmp_path / "x.tga").write_bytes(b"\x00\x00\x02" + bytes(40))
    with pytest.raises(RuntimeError, match="unsupported image format"):
        I.decode(tmp_path / "x.tga")
    (tmp_path / "trunc.png").write_bytes(b"\x89PNG\r\n\x1a\n" + bytes(30))
    with pytest.raises(RuntimeError):
        I.decode(tmp_path / "trunc.png")
    with pytest.raises(RuntimeError, match="cannot open"):
        I.decode(tmp_path / "missing.png")


def _jpeg_segments(data):
    """(marker, offset of the 0xFF, segment length) of every header segment before the entropy data."""
    out, p = [], 2
    while p + 4 <= len(data):
        m = data[p + 1]
        n = (data[p + 2] << 8) | data[p + 3]
        out.append((m, p, n))
        if m == 0xDA:
            break
        p += 2 + n
    return out


def _patched(data, at, value):
    b = bytearray(data)
    b[at] = value
    return bytes(b)


def test_malformed_jpeg_fails_loudly(tmp_path):
    # table ids out of range and segments too short for their fixed fields must be rejected before
    # any read past the segment (Huffman / quantisation tables are indexed 0..3)
    buf = io.BytesIO()
    PIL.fromarray(_smooth_image(24, 24, 3), "RGB").save(buf, "JPEG", quality=80)
    good = buf.getvalue()
    seg = {m: (p, n) for m, p, n in _jpeg_segments(good)}
    sos_p, sos_n = seg[0xDA]
    sof_p, sof_n = seg[0xC0]
    dqt_p, _ = seg[0xDB]
    dht_p, _ = seg[0xC4]
    cases = {
        "scan DC table id 15": _patched(good, sos_p + 4 + 2, 0xF0 | (good[sos_p + 4 + 2] & 0x0F)),
        "scan AC table id 7": _patched(good, sos_p + 4 + 2, (good[sos_p + 4 + 2] & 0xF0) | 0x07),
        "quant table id 9": _patched(good, dqt_p + 4, 0x09),
        "quant precision 3": _patched(good, dqt_p + 4, 0x30),
        "huffman class 2": _patched(good, dht_p + 4, 0x20 | (good[dht_p + 4] & 0x0F)),
        "frame component quant id 5": _patched(good, sof_p + 4 + 8, 5),
        # SOF claiming 3 components in a 5-byte segment, then end of file
        "short frame header": good[:sof_p] + bytes([0xFF, 0xC0, 0x00, 0x07, 8, 0, 24, 0, 24]),
        "short scan header": good[:sos_p] + bytes([0xFF, 0xDA, 0x00, 0x03, 3]),
        "short restart interval": good[:sos_p] + bytes([0xFF, 0xDD, 0x00, 0x02]) + good[sos_p:],
        "quant table past the segment": good[:dqt_p] + bytes([0xFF, 0xDB, 0x00, 0x06, 0x00, 1, 2, 3]) + good[dqt_p:],
    }
    for what, data in cases.items():
        f = tmp_path / "bad.jpg"
        f.write_bytes(data)
        with pytest.raises(RuntimeError):
            I.decode(f)
        assert what


@needs_ref
def test_reference_png_assets_exact():
    # theInn's textures (Content/Models/theInn/textures): RGBA and RGB, 512..2048 px
    files = sorted(glob.glob(os.path.join(REF, "theInn", "textures", "*.png")))
    assert len(files) == 3
    for f in files:
        got, _ = I.decode(f)
        np.testing.assert_array_equal(got, np.asarray(PIL.open(f).convert("RGBA")), err_msg=f)


@needs_ref
def test_reference_jpeg_assets_match_libjpeg():
    # Stronghold's textures (Content/Models/Stronghold/textures): baseline 4:4:4, 128..2048 px
    files = sorted(glob.glob(os.path.join(REF, "Stronghold", "textures", "*.jp*g")))
    assert len(files) == 11
    for f in files:
        got, _ = I.decode(f)
        d = np.abs(got.astype(int) - np.asarray(PIL.open(f).convert("RGBA")).astype(int))
        assert d.max() <= 4 and d.mean() < 0.1, (f, d.max(), d.mean())


@needs_ref
def test_theinn_fbx_names_no_texture_files():
    # Scenes::Stronghold = theInn.fbx (DXRPathTracer.cpp:90): its material's texture map carries an empty
    # file name, so the reference's Model::CreateWithAssimp falls back to the default textures
    # (Graphics/Model.cpp:113) and never opens the PNGs next to it; the loader here does the same
    data = open(os.path.join(REF, "theInn", "source", "theInn.fbx"), "rb").read()
    for ext in (b".png", b".jpg", b".jpeg", b".dds", b".tga"):
        assert ext not in data.lower()
    sc = D.Scene.from_reference("stronghold")
    assert len(sc.textures) == 4
