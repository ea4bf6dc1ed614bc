"""CPU (gloo): the N>1 frame job's failure handling (dxrpathtracer_amd/watchdog.py) and the NativeGather
control flow (distributed.py) around a stub communicator.

The stub has libdxrpt's multi-GPU entry points (dxrpt_comm_*, dxrpt_gather_slabs, dxrpt_unpermute) and
moves the slabs with gloo on host memory, so the pipelined submit / finish / flush sequence bench.py runs
is exercised here without RCCL.  Its failure mode stands in for an RCCL error on one rank: that rank raises,
and every rank must end non-zero with a JSON error line instead of blocking in the next collective."""
import ctypes as C
import json
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Stream:
    cuda_stream = 0

    def wait_stream(self, other):
        pass

    def wait_event(self, ev):
        pass


class _Event:
    def record(self, stream=None):
        pass

    def elapsed_time(self, other):
        return 0.0


def _floats(ptr, n):
    return np.ctypeslib.as_array((C.c_float * n).from_address(ptr.value))


class StubComm:
    """libdxrpt's multi-GPU C ABI over gloo (host memory).  fail_frame: this rank's dxrpt_gather_slabs
    returns an error from that frame on (an RCCL failure on one rank)."""

    def __init__(self, rank, world, fail_frame=None):
        self.rank, self.world, self.fail_frame, self.frames, self.err = rank, world, fail_frame, 0, b""

    def dxrpt_comm_unique_id(self, uid):
        return 0

    def dxrpt_comm_create(self, device, world, rank, uid, comm_ref):
        comm_ref._obj.value = 0x1000 + rank
        return 0

    def dxrpt_comm_info(self, comm, nr_ref, rk_ref):
        nr_ref._obj.value, rk_ref._obj.value = self.world, self.rank
        return 0

    def dxrpt_multi_last_error(self):
        return self.err

    def dxrpt_gather_slabs(self, comm, send, counts, recv, stream):
        f = self.frames
        self.frames += 1
        if self.fail_frame is not None and f >= self.fail_frame:
            self.err = b"stub: ncclSend failed (unhandled system error)"
            return 7
        cnt = [int(counts[r]) for r in range(self.world)]
        mx = max(cnt)
        mine = torch.zeros(mx * 4, dtype=torch.float32)
        mine[:cnt[self.rank] * 4] = torch.from_numpy(_floats(send, cnt[self.rank] * 4).copy())
        bufs = [torch.zeros(mx * 4, dtype=torch.float32) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(mine, bufs, dst=0)
        if self.rank == 0:
            out = _floats(recv, sum(cnt) * 4)
            off = 0
            for r in range(self.world):
                out[off * 4:(off + cnt[r]) * 4] = bufs[r][:cnt[r] * 4].numpy()
                off += cnt[r]
        return 0

    def dxrpt_unpermute(self, recv, tarr, ntiles, full, W, H, stream):
        total = sum(t.w * t.h for t in tarr)
        src = _floats(recv, total * 4).reshape(-1, 4)
        dst = _floats(full, W * H * 4).reshape(-1, 4)
        for t in tarr:
            for yy in range(t.h):
                dst[(t.y0 + yy) * W + t.x0:(t.y0 + yy) * W + t.x0 + t.w] = \
                    src[t.accum_offset + yy * t.accum_pitch:t.accum_offset + yy * t.accum_pitch + t.w]
        return 0

    def dxrpt_comm_destroy(self, comm):
        return 0

    def dxrpt_multi_release(self):
        return 0


def _stub_gather_cls():
    from dxrpathtracer_amd.distributed import NativeGather

    class StubGather(NativeGather):
        def _device_ready(self, device):
            return True

        def _new_stream(self):
            return _Stream()

        def _current_stream(self):
            return _Stream()

        def _event(self, timing=False):
            return _Event()

        def _synchronize(self):
            pass

    return StubGather


def _frame_image(W, H, f):
    return np.arange(W * H * 4, dtype=np.float32).reshape(H, W, 4) + 1000.0 * f


def _worker(rank, world, port, outdir, fail_rank, fail_frame, W, H, frames):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dxrpathtracer_amd.distributed import band_layout
    from dxrpathtracer_amd.watchdog import Watchdog, default_store

    def report(line):
        with open(os.path.join(outdir, f"r{rank}.json"), "a") as fh:
            fh.write(line + "\n")

    wd = Watchdog(rank, world, default_store(), "test metric", report=report, poll_s=0.05)
    try:
        lay = band_layout(W, H, world)
        full = torch.zeros((W * H, 4), dtype=torch.float32) if rank == 0 else None
        with wd.phase("communicator", 60):
            pg = _stub_gather_cls()(lay, rank, 0, full, timing=True,
                                    lib=StubComm(rank, world, fail_frame if rank == fail_rank else None))
            assert pg.comm_ranks == world and pg.comm_rank == rank
        local = torch.zeros((lay.max_count, 4), dtype=torch.float32)
        ok = True
        with wd.phase("frames", 60):
            for f in range(frames):
                img = _frame_image(W, H, f)
                for t in lay.rank_tiles(rank):
                    local[t.accum_offset:t.accum_offset + t.w * t.h] = torch.from_numpy(
                        img[t.y0:t.y0 + t.h, t.x0:t.x0 + t.w].reshape(-1, 4))
                pg.submit(local)
                local.fill_(-1.0)  # the next frame overwrites the accumulation buffer: the snapshot must hold
                if rank == 0 and f > 0:  # frame f-1 un-permuted once frame f was submitted
                    ok &= bool(np.array_equal(full.numpy().reshape(H, W, 4), _frame_image(W, H, f - 1)))
            pg.flush()
            if rank == 0:
                ok &= bool(np.array_equal(full.numpy().reshape(H, W, 4), _frame_image(W, H, frames - 1)))
            _, _, timed = pg.times()
            ok &= timed == frames
        with wd.phase("teardown", 60):
            pg.close()
            dist.barrier()
        with open(os.path.join(outdir, f"r{rank}.ok"), "w") as fh:
            fh.write("1" if ok else "0")
    except BaseException as e:  # noqa: BLE001 -- bench.py's handler
        wd.fail(f"{type(e).__name__}: {e}")
    wd.close()
    dist.destroy_process_group()


def _run(world, tmp_path, fail_rank=None, fail_frame=None, W=40, H=56, frames=4):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path), fail_rank, fail_frame, W, H, frames))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    return codes


@pytest.mark.parametrize("world", [2, 3])
def test_native_gather_control_flow_delivers_every_frame(world, tmp_path):
    # NativeGather's pipelined sequence (snapshot -> dxrpt_gather_slabs -> on the next submit the previous
    # frame's dxrpt_unpermute) with gloo standing in for RCCL: rank 0 holds frame f after submit(f+1)
    # and the last frame after flush(), every rank exits 0 and reports nothing
    codes = _run(world, tmp_path)
    assert codes == [0] * world, codes
    for r in range(world):
        assert (tmp_path / f"r{r}.ok").read_text() == "1"
        assert not (tmp_path / f"r{r}.json").exists()


@pytest.mark.parametrize("world,fail_rank,fail_frame", [(2, 1, 2), (3, 2, 1), (3, 0, 0)])
def test_one_rank_gather_failure_ends_every_rank(world, fail_rank, fail_frame, tmp_path):
    # one rank's dxrpt_gather_slabs fails (an RCCL error): that rank raises and exits 1 with a JSON error
    # line; the others -- blocked in the gather's collective -- see the abort in the rendezvous store (or
    # their own collective error) and exit non-zero with a JSON error line too, within seconds
    t0 = time.time()
    codes = _run(world, tmp_path, fail_rank, fail_frame)
    assert all(c is not None for c in codes), codes
    assert codes[fail_rank] == 1, codes
    assert all(c != 0 for c in codes), codes
    assert time.time() - t0 < 120
    for r in range(world):
        lines = (tmp_path / f"r{r}.json").read_text().splitlines()
        assert len(lines) == 1, lines
        rec = json.loads(lines[0])
        assert rec["value"] is None and rec["metric"] == "test metric" and rec["rank"] == r and rec["n_gpus"] == world
        if r == fail_rank:
            assert rec["error_kind"] == "failed" and "dxrpt_gather_slabs failed" in rec["error"], rec
        assert not (tmp_path / f"r{r}.ok").exists()


def test_phase_timeout_reports_and_exits():
    # a phase past its limit (a collective that never completes) ends the rank with EXIT_TIMEOUT and one
    # JSON line naming the phase; a phase that ends in time does nothing
    from dxrpathtracer_amd.watchdog import EXIT_TIMEOUT, Watchdog
    lines, codes = [], []
    wd = Watchdog(0, 1, None, "m", report=lines.append, exit=codes.append, poll_s=0.02)
    with wd.phase("quick", 5.0):
        time.sleep(0.05)
    assert not codes and not lines
    with wd.phase("stuck collective", 0.1):
        deadline = time.time() + 5
        while not codes and time.time() < deadline:
            time.sleep(0.02)
    wd.close()
    assert codes == [EXIT_TIMEOUT], codes
    rec = json.loads(lines[0])
    assert rec["error_kind"] == "timeout" and rec["phase"] == "stuck collective" and rec["value"] is None


def test_fail_publishes_abort_for_peers():
    # fail() writes the abort record into the store before exiting; a peer's monitor reads it
    from dxrpathtracer_amd.watchdog import ABORT_KEY, EXIT_FAILED, EXIT_PEER, Watchdog
    store = dist.HashStore()
    la, ca, lb, cb = [], [], [], []
    a = Watchdog(0, 2, store, "m", report=la.append, exit=ca.append, poll_s=0.02)
    b = Watchdog(1, 2, store, "m", report=lb.append, exit=cb.append, poll_s=0.02)
    with b.phase("gather", 30):
        a.fail("RuntimeError: dxrpt_gather_slabs failed (7)")
        deadline = time.time() + 5
        while not cb and time.time() < deadline:
            time.sleep(0.02)
    a.close()
    b.close()
    assert ca == [EXIT_FAILED] and cb == [EXIT_PEER], (ca, cb)
    assert json.loads(store.get(ABORT_KEY).decode())["rank"] == 0
    rb = json.loads(lb[0])
    assert rb["error_kind"] == "peer_abort" and rb["origin_rank"] == 0 and rb["phase"] == "gather"
