"""The BVH build options change the tree, never the image (include/dxrpt.h DXRPT_OPT_TREELET_PASSES,
DXRPT_OPT_LEAF_COST, DXRPT_OPT_SPATIAL_SPLITS).

The closest hit is the minimum (t, triangle) over every triangle the ray meets and an any-hit ray's
visibility is a boolean over them, so any correct acceleration structure gives the same frame bit for bit
(RayTrace.hlsl's TraceRay contract; the oracle builds its own tree).  Each variant context renders the
frame the shipped context renders (1 treelet pass, 150 % spatial-split budget, leaf cost 1.5) and must
match it exactly, while its BVH differs (node count or SAH), so the option did take effect.  SunTemple
carries the alpha-tested foliage (any-hit shader on both ray kinds), whose subtrees the treelet pass
leaves as built.
"""
import numpy as np
import pytest

import dxrpathtracer_amd as D
import dxrpathtracer_amd._abi as A
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import scene_bundle

pytestmark = pytest.mark.gpu

W, H = 640, 360
VARIANTS = {
    "no_treelets": {A.OPT_TREELET_PASSES: 0},
    "two_treelet_passes": {A.OPT_TREELET_PASSES: 2},
    "leaf_cost_1": {A.OPT_LEAF_COST: 100},
    "no_spatial_splits": {A.OPT_SPATIAL_SPLITS: 0},
}
_CTX = {}


def context(name, variant):
    key = (name, variant)
    if key not in _CTX:
        sc, sky = scene_bundle(name)
        t = DXRPathTracer(0)
        for o, v in VARIANTS.get(variant, {}).items():
            t.set_option(o, v)
        t.initialize_scene(sc, sky)
        info = t.build_rt_acceleration_structure()
        _CTX[key] = (t, (info.num_nodes, round(info.sah_cost, 6)))
    return _CTX[key]


def frame(torch, name, variant, L, sample):
    sc, sky = scene_bundle(name)
    st = sc.settings(MaxPathLength=L)
    t, _ = context(name, variant)
    acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    t.render_raw(D.make_constants(sc, st, sky, W, H, sample), st, acc.data_ptr(), W, H,
                 stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
    torch.cuda.synchronize()
    return acc.cpu().numpy()


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("name", ["sponza", "suntemple"])
def test_build_options_give_identical_frames(torch_cuda, name, variant):
    assert context(name, variant)[1] != context(name, "shipped")[1], f"{variant}: the BVH did not change"
    for L, sample in ((3, 0), (5, 3)):
        ref = frame(torch_cuda, name, "shipped", L, sample)
        got = frame(torch_cuda, name, variant, L, sample)
        assert np.isfinite(ref).all()
        np.testing.assert_array_equal(got, ref, err_msg=f"{name} {variant} L{L} s{sample}")


def test_treelet_option_range(torch_cuda):
    t = DXRPathTracer(0)
    with pytest.raises(RuntimeError, match="treelet passes"):
        t.set_option(A.OPT_TREELET_PASSES, 9)
    t.close()


def test_parallel_treelet_build_is_deterministic(torch_cuda):
    """The treelet pass restructures disjoint subtrees on host threads: two builds of the same scene give
    the same tree (node count, SAH) and the same frame."""
    sc, sky = scene_bundle("sponza")
    t = DXRPathTracer(0)
    t.initialize_scene(sc, sky)
    info = t.build_rt_acceleration_structure()
    assert (info.num_nodes, round(info.sah_cost, 6)) == context("sponza", "shipped")[1]
    st = sc.settings(MaxPathLength=3)
    acc = torch_cuda.zeros((W * H, 4), dtype=torch_cuda.float32, device="cuda")
    t.render_raw(D.make_constants(sc, st, sky, W, H, 0), st, acc.data_ptr(), W, H,
                 stream=torch_cuda.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
    torch_cuda.cuda.synchronize()
    np.testing.assert_array_equal(acc.cpu().numpy(), frame(torch_cuda, "sponza", "shipped", 3, 0))
    t.close()


def test_build_threads_do_not_change_the_tree(torch_cuda):
    """DXRPT_OPT_BVH_THREADS (ABI 4): the parallel SBVH / treelet / collapse build gives the same tree for any
    thread count (tests/test_bvh_build.py checks the layout hash on the CPU); the info reports the phases."""
    sc, sky = scene_bundle("suntemple")
    infos = []
    for threads in (1, 0):
        t = DXRPathTracer(0)
        t.set_option(A.OPT_BVH_THREADS, threads)
        t.initialize_scene(sc, sky)
        infos.append(t.build_rt_acceleration_structure())
        t.close()
    one, auto = infos
    assert one.threads == 1 and auto.threads >= 1
    for f in ("num_nodes", "num_leaves", "num_refs", "max_depth", "sah_cost", "wide_sah", "binary_depth_cap",
              "treelet_passes", "ref_budget_pct"):
        assert getattr(one, f) == getattr(auto, f), f
    assert auto.ref_budget_pct == 115 and auto.treelet_passes == 1 and auto.num_refs >= auto.num_tris
    assert all(auto.phase_ms[k] >= 0.0 for k in range(4)) and sum(auto.phase_ms) <= auto.build_ms * 1.01 + 1.0
