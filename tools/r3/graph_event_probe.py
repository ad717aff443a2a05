#!/usr/bin/env python
"""Probe: can HIP timing events be recorded INSIDE a captured graph (hipEventRecordWithFlags with
hipEventRecordExternal -> event-record nodes) and timed after a replay?  If so, bench.py can time each
hot kernel inside the graph replay it benchmarks.  Compares the in-graph event time of a matmul with the
same matmul timed eagerly, and a replay of the graph without the events."""
from __future__ import annotations

import ctypes

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
    hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    a = torch.randn(8192, 8192, device=dev)
    b = torch.randn(8192, 8192, device=dev)
    c = a @ b
    torch.cuda.synchronize()
    evs = []
    for _ in range(4):
        e = ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), 0) == 0  # timing enabled
        evs.append(e)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):
            torch.matmul(a, b, out=c)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        st = torch.cuda.current_stream().cuda_stream
        rc0 = hip.hipEventRecordWithFlags(evs[0], ctypes.c_void_p(st), 1)  # hipEventRecordExternal
        torch.matmul(a, b, out=c)
        rc1 = hip.hipEventRecordWithFlags(evs[1], ctypes.c_void_p(st), 1)
        torch.matmul(a, b, out=c)
        rc2 = hip.hipEventRecordWithFlags(evs[2], ctypes.c_void_p(st), 1)
    print("record rcs", rc0, rc1, rc2)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = ctypes.c_float()
    rc = hip.hipEventElapsedTime(ctypes.byref(t), evs[0], evs[1])
    t2 = ctypes.c_float()
    rc2 = hip.hipEventElapsedTime(ctypes.byref(t2), evs[1], evs[2])
    print("in-graph elapsed rc", rc, t.value, "ms;", rc2, t2.value, "ms")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.matmul(a, b, out=c)
    e1.record()
    torch.cuda.synchronize()
    print("eager per matmul", e0.elapsed_time(e1) / 10, "ms")


if __name__ == "__main__":
    main()
