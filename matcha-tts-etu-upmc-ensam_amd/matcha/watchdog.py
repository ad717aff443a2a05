"""Fail-fast watchdog for the data-parallel step (bench.py's N>1 path).

A rank whose step stops making progress -- a peer that never joins a bucket's all-reduce, an RCCL kernel that
never completes inside the replayed graph -- would otherwise block until the driver's own time limit and leave
no evidence.  ``StepWatchdog`` is a host thread per rank: the step loop and the gradient reducer report
progress (``beat`` / ``note``); when nothing has progressed for the bound of the current phase it prints one
line to stderr naming the rank, the phase, the graph key, the last bucket the host issued and the last step and
bucket the DEVICE completed (``DeviceProgress``: markers written by the graph itself into host-mapped memory,
read without synchronising), then ends the process with ``os._exit(exit_code)`` -- no retry, no re-exec;
torch.distributed.run then stops the other ranks.

The reference has no multi-GPU step (train.py:81-84 trains on one device); DDP's counterpart is torch's
ProcessGroupNCCL watchdog timeout (default 10 minutes, not capturable on this stack -- matcha/dp.py).
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
import time

from matcha import _native as N

N.register("mtts_dp_progress_create", ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p),
                                                     ctypes.POINTER(ctypes.POINTER(ctypes.c_int32))])
N.register("mtts_dp_progress_mark", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p])
N.register("mtts_dp_progress_destroy", ctypes.c_int, [ctypes.c_void_p])


class DeviceProgress:
    """Host-mapped progress slots written by the device in stream order (include/mtts_dp.h).  Slot 0: steps the
    device completed; slot 1: steps * 256 + (index + 1) of the last bucket whose all-reduce completed."""

    SLOTS = 2

    def __init__(self):
        self._h = ctypes.c_void_p()
        self._host = ctypes.POINTER(ctypes.c_int32)()
        N.check(N.lib().mtts_dp_progress_create(self.SLOTS, ctypes.byref(self._h), ctypes.byref(self._host)),
                "mtts_dp_progress_create")

    def mark_step(self, stream) -> None:
        N.check(N.lib().mtts_dp_progress_mark(self._h, 0, -1, stream.cuda_stream), "mtts_dp_progress_mark")

    def mark_bucket(self, k: int, stream) -> None:
        N.check(N.lib().mtts_dp_progress_mark(self._h, 1, k + 1, stream.cuda_stream), "mtts_dp_progress_mark")

    def read(self) -> dict:
        steps, b = int(self._host[0]), int(self._host[1])
        return {"device_steps_done": steps,
                "device_last_bucket_done": (b % 256) - 1 if b else None,
                "device_last_bucket_step": b // 256 if b else None}

    def close(self) -> None:
        if self._h:
            N.lib().mtts_dp_progress_destroy(self._h)
            self._h = ctypes.c_void_p()


class StepWatchdog:
    """Per-rank host watchdog.  ``beat(phase, bound_s=None, **fields)`` records progress (and optionally a new
    bound for the phase that starts); ``note(**fields)`` updates what the report names without counting as
    progress; ``stop()`` ends the thread.  ``device``: an optional DeviceProgress -- a change in what the
    device reports also counts as progress (the host thread is blocked in a synchronise while the replayed
    steps run)."""

    def __init__(self, rank: int, bound_s: float, device: DeviceProgress | None = None, exit_code: int = 3,
                 poll_s: float = 0.25, out=None):
        self.rank = rank
        self.bound_s = float(bound_s)
        self.device = device
        self.exit_code = exit_code
        self.poll_s = poll_s
        self.out = out or sys.stderr
        self.fields: dict = {"phase": "init", "last_step_done": -1, "graph_key": None, "bucket_issued": None,
                             "buckets": None}
        self._lock = threading.Lock()
        self._last = time.monotonic()
        self._dev_seen = None
        self._stop = threading.Event()
        self.fired = False
        self._t = threading.Thread(target=self._run, name=f"mtts-watchdog-r{rank}", daemon=True)
        self._t.start()

    def beat(self, phase: str | None = None, bound_s: float | None = None, **fields) -> None:
        with self._lock:
            if phase is not None:
                self.fields["phase"] = phase
            if bound_s is not None:
                self.bound_s = float(bound_s)
            self.fields.update(fields)
            self._last = time.monotonic()

    def note(self, **fields) -> None:
        with self._lock:
            self.fields.update(fields)

    def stop(self) -> None:
        self._stop.set()
        self._t.join(timeout=5.0)

    def report(self, idle_s: float) -> str:
        with self._lock:
            f = dict(self.fields)
            bound = self.bound_s
        dev = self.device.read() if self.device is not None else {}
        parts = [f"[mtts watchdog] rank {self.rank}: no progress for {idle_s:.1f} s (bound {bound:.0f} s)",
                 f"phase={f.pop('phase')}", f"last_step_done={f.pop('last_step_done')}",
                 f"graph_key={f.pop('graph_key')}",
                 f"bucket_issued={f.pop('bucket_issued')} of {f.pop('buckets')}"]
        parts += [f"{k}={v}" for k, v in sorted(f.items())]
        parts += [f"{k}={v}" for k, v in dev.items()] or ["device=n/a"]
        return "; ".join(parts)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            if self.device is not None:
                d = self.device.read()
                key = (d["device_steps_done"], d["device_last_bucket_done"], d["device_last_bucket_step"])
                if key != self._dev_seen:
                    self._dev_seen = key
                    with self._lock:
                        self._last = time.monotonic()
            with self._lock:
                idle = time.monotonic() - self._last
                bound = self.bound_s
            if idle > bound:
                self.fired = True
                try:
                    print(self.report(idle), file=self.out, flush=True)
                finally:
                    os._exit(self.exit_code)
