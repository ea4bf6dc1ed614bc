"""Failure handling for a multi-rank frame job (bench.py --gpus N).

A rank that fails (an RCCL / C-ABI error, a Python exception) or that stays in one phase past its time
limit (a collective that never completes: RCCL blocks on the GPU stream, so the host waits inside
torch.cuda.synchronize or a barrier) must not leave the other ranks blocked in the next collective.
`Watchdog` ends EVERY rank with a non-zero exit and one JSON error line:

  * the failing rank writes an abort record into the job's rendezvous store (torch.distributed's TCP
    store -- it does not go through RCCL, so it still works when a collective is stuck) and exits;
  * a monitor thread on every rank polls that key and its own phase deadline; either ends the rank.

The exit is os._exit from the monitor thread (the main thread may be blocked inside a HIP or RCCL call
that never returns; no exec, no re-launch).  Without a store (one rank) only the deadlines apply.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time

ABORT_KEY = "dxrpt_abort"
EXIT_FAILED = 1    # this rank raised or reported an error
EXIT_TIMEOUT = 3   # this rank's phase passed its time limit
EXIT_PEER = 4      # another rank aborted the job


def default_store():
    """torch.distributed's default (rendezvous) store, or None (no process group / not exposed)."""
    try:
        import torch.distributed as dist
        if not dist.is_initialized():
            return None
        from torch.distributed import distributed_c10d as c10d
        return c10d._get_default_store()
    except Exception:
        return None


class Watchdog:
    """with wd.phase("render", 120): ...   -- the phase must end within 120 s on this rank.
    wd.fail(msg)                        -- abort the job from this rank (every rank exits non-zero).

    `report(line)` writes the JSON error line (default: stdout); `exit(code)` ends the process (default
    os._exit; tests pass a recorder).  `poll_s`: how often the monitor looks at the store and the clock."""

    def __init__(self, rank: int, world: int, store=None, metric: str | None = None, report=None, exit=None,
                 poll_s: float = 0.2):
        self.rank, self.world, self.store, self.metric = rank, world, store, metric
        self.report = report or (lambda line: print(line, flush=True))
        self._exit = exit or os._exit
        self.poll_s = poll_s
        self._phase, self._deadline = "start", None
        self._lock = threading.Lock()
        self._ended = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._monitor, name="dxrpt-watchdog", daemon=True)
        self._thread.start()

    # ---- phases
    def phase(self, name: str, timeout_s: float):
        wd = self

        class _Phase:
            def __enter__(self):
                with wd._lock:
                    self.prev = (wd._phase, wd._deadline)
                    wd._phase, wd._deadline = name, time.monotonic() + float(timeout_s)
                return wd

            def __exit__(self, et, ev, tb):
                with wd._lock:
                    wd._phase, wd._deadline = self.prev
                return False

        return _Phase()

    @property
    def current_phase(self) -> str:
        return self._phase

    # ---- abort paths
    def _line(self, kind: str, msg: str, origin: int) -> str:
        return json.dumps({"metric": self.metric, "value": None, "error": msg, "error_kind": kind, "rank": self.rank,
                           "origin_rank": origin, "n_gpus": self.world, "phase": self._phase})

    def _end(self, kind: str, msg: str, origin: int, code: int, publish: bool):
        with self._lock:
            if self._ended:
                return
            self._ended = True
        if publish and self.store is not None:
            try:
                self.store.set(ABORT_KEY, json.dumps({"rank": self.rank, "phase": self._phase, "kind": kind,
                                                      "msg": msg[:500]}))
            except Exception as e:  # the store itself is gone: the other ranks' deadlines still end them
                print(f"watchdog: could not publish the abort ({e})", file=sys.stderr, flush=True)
        try:
            self.report(self._line(kind, msg, origin))
        finally:
            self._stop.set()
            self._exit(code)

    def fail(self, msg: str):
        """This rank failed: publish the abort, report, exit EXIT_FAILED."""
        self._end("failed", msg, self.rank, EXIT_FAILED, publish=True)

    def close(self):
        """The job finished on this rank: stop monitoring (no exit)."""
        self._stop.set()
        if self._thread is not threading.current_thread():
            self._thread.join(timeout=2 * self.poll_s + 1.0)

    # ---- monitor thread
    def _peer_abort(self):
        if self.store is None:
            return None
        try:
            if self.store.check([ABORT_KEY]):
                return json.loads(self.store.get(ABORT_KEY).decode())
        except Exception:
            return None
        return None

    def _monitor(self):
        while not self._stop.wait(self.poll_s):
            peer = self._peer_abort()
            if peer is not None and not self._ended:
                self._end("peer_abort", f"rank {peer.get('rank')} aborted in phase {peer.get('phase')!r}: "
                                        f"{peer.get('msg')}", int(peer.get("rank", -1)), EXIT_PEER, publish=False)
                return
            with self._lock:
                late = self._deadline is not None and time.monotonic() > self._deadline
                phase = self._phase
            if late and not self._ended:
                self._end("timeout", f"phase {phase!r} passed its time limit (a collective or GPU wait that "
                                      "never completed)", self.rank, EXIT_TIMEOUT, publish=True)
                return
