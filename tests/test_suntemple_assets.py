"""The SunTemple proxy (BASELINE config C4) alpha-tests its foliage with the reference's own BC4 opacity
maps, packaged as dxrpathtracer_amd/data/suntemple/*.r8z by
scripts/make_suntemple_opacity.py.  Checked against the reference's DDS files when the checkout is
present, and by content digest everywhere (the GPU box has no checkout)."""
import hashlib
import os

import numpy as np
import pytest

import dxrpathtracer_amd as D
from tests import image_util as I

REF_TEX = "/root/reference/Content/Models/SunTemple/Textures"
# sha256 of the decoded R8 texels (mip 0), recorded when the files were generated
DIGESTS = {
    (1024, 1024): "9f5a02817e443ccebb0f0b2023dcc9a49a42b8eb9359ee2bda2f9bf55eb32b0c",
    (2048, 2048): "16911cbcfcb2d7bc3cde4861dff6e95c211eecddf6e1b88587d945426293bbba",
}


def _opacity_textures():
    sc = D.Scene("suntemple")
    ops = [int(m[4]) for m in sc.materials if m[4] != 0xFFFFFFFF]
    return sc, ops


def test_suntemple_foliage_uses_packaged_opacity_maps():
    sc, ops = _opacity_textures()
    sizes = sorted((sc.textures[o][0], sc.textures[o][1]) for o in ops)
    assert sizes == [(1024, 1024), (2048, 2048)]
    for o in ops:
        w, h, fmt, data = sc.textures[o]
        assert fmt == D._abi.TEX_R8_UNORM
        frac = float((data >= 90).mean())  # texels the any-hit shader keeps (opacity >= 0.35)
        assert 0.2 < frac < 0.4
        assert hashlib.sha256(data.tobytes()).hexdigest() == DIGESTS[(w, h)]


@pytest.mark.skipif(not os.path.isdir(REF_TEX), reason="reference checkout not present")
def test_packaged_maps_equal_reference_dds():
    sc, ops = _opacity_textures()
    by_size = {(sc.textures[o][0], sc.textures[o][1]): sc.textures[o][3] for o in ops}
    for name, size in (("T_M_Tree_Branches_0_A.dds", (1024, 1024)), ("T_Soul_Tree011M_Inst_0_A.dds", (2048, 2048))):
        img, _ = I.decode(os.path.join(REF_TEX, name))
        np.testing.assert_array_equal(by_size[size].reshape(size[1], size[0]), img)
