"""The C++ host (dxrpathtracer_amd/lib/dxrpt_render, csrc/tools/dxrpt_render.cpp) drives the same hot path
through the C ABI with no Python: InitializeScene -> BuildRTAccelerationStructure -> RenderRayTracing per
frame (DXRPathTracer.cpp:932-985, 2331-2488, 2024-2090), and with --world the band sharding + RCCL gather
+ un-permute of an N-GPU frame.  Its accumulation target must equal the Python driver's
bit for bit (same scene, sky, constants and progressive samples), and the Python frames are the ones the
oracle parity tests check.  Each CLI run is a child process (one GPU process at a time)."""
import json
import os
import subprocess

import numpy as np
import pytest

import dxrpathtracer_amd as D
from dxrpathtracer_amd.tracer import DXRPathTracer
from tests._common import assert_parity, oracle_scene, scene_bundle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "dxrpathtracer_amd", "lib", "dxrpt_render")


def run_cli(tmp_path, *args):
    out = tmp_path / "accum.f32"
    p = subprocess.run([CLI, *map(str, args), "--dump-accum", str(out)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    return line, np.fromfile(out, dtype=np.float32)


def python_frames(torch, name, W, H, L, frames):
    sc, sky = scene_bundle(name)
    st = sc.settings(MaxPathLength=L)
    t = DXRPathTracer(0)
    try:
        t.initialize_scene(sc, sky)
        t.build_rt_acceleration_structure()
        acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        for f in range(frames):
            t.render_raw(D.make_constants(sc, st, sky, W, H, f % 16), st, acc.data_ptr(), W, H,
                         stream=torch.cuda.current_stream().cuda_stream, lights=D.make_lights(sc))
        torch.cuda.synchronize()
        return acc.cpu().numpy().reshape(-1)
    finally:
        t.close()


@pytest.mark.parametrize("name,W,H,L,frames", [("boxtest", 96, 96, 3, 3), ("sponza", 480, 270, 3, 4),
                                                ("suntemple", 320, 180, 4, 2)])
def test_cli_equals_python_driver(torch_cuda, tmp_path, name, W, H, L, frames):
    assert os.path.exists(CLI), "build first: make -C dxrpathtracer_amd/csrc"
    line, got = run_cli(tmp_path, "--scene", name, "--width", W, "--height", H, "--path-length", L,
                        "--frames", frames, "--warmup", 0)
    assert line["frames"] == frames and line["ms_per_frame"] > 0
    ref = python_frames(torch_cuda, name, W, H, L, frames)
    np.testing.assert_array_equal(got, ref)


def test_cli_one_rank_gather_equals_frame(torch_cuda, tmp_path):
    # --world 1: dxrpt_comm_create of one rank, dxrpt_gather_slabs + dxrpt_unpermute every frame
    W, H, L = 480, 270, 3
    _, plain = run_cli(tmp_path, "--scene", "sponza", "--width", W, "--height", H, "--frames", 3, "--warmup", 0)
    line, gathered = run_cli(tmp_path, "--scene", "sponza", "--width", W, "--height", H, "--frames", 3, "--warmup", 0,
                             "--world", 1, "--rank", 0, "--uid-file", tmp_path / "uid")
    assert line["world"] == 1
    np.testing.assert_array_equal(gathered, plain)


def test_cli_boxtest_matches_oracle(torch_cuda, tmp_path):
    # the CLI's first frame against the oracle directly (BASELINE configs[0]'s scene)
    W, H = 64, 64
    _, got = run_cli(tmp_path, "--scene", "boxtest", "--width", W, "--height", H, "--frames", 1, "--warmup", 0)
    sc, sky = scene_bundle("boxtest")
    st = sc.settings(MaxPathLength=3)
    rtc = D.make_constants(sc, st, sky, W, H, 0)
    ref, _ = oracle_scene("boxtest").render(rtc, st, D.make_lights(sc), W, H)
    assert_parity(got.reshape(H, W, 4), ref, "dxrpt_render boxtest 64x64 L3 s0")


def test_cli_metric_frame_rate(torch_cuda, tmp_path):
    # the metric workload through the C++ host: the shipped schedule (depth split, overlapped frames)
    line, img = run_cli(tmp_path, "--scene", "sponza", "--frames", 16, "--warmup", 4)
    assert line["width"] == 1920 and line["height"] == 1080 and line["max_path_length"] == 3
    assert line["schedule_bits"] & 1 and line["schedule_bits"] & 32 and line["schedule_bits"] & 128, line
    assert np.isfinite(img).all() and line["ms_per_frame"] < 10.0, line
    print(json.dumps(line))
