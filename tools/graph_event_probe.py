"""Probe: does an EXTERNAL event recorded inside a captured HIP graph order work issued outside the
graph (on another stream, after replay()) behind that point of THIS replay?  And can RCCL collectives
be captured (world size 1)?  Prints PASS/FAIL lines; exits non-zero on a stale read."""
import os
import sys

import torch

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
main = torch.cuda.Stream(dev)
side = torch.cuda.Stream(dev)
a = torch.randn(4096, 4096, device=dev)
counter = torch.zeros(1, device=dev)
buf = torch.zeros(1 << 20, device=dev)
out = torch.zeros(1 << 20, device=dev)
ev = torch.cuda.Event(external=True)
PROBE_EVENTS = os.environ.get("PROBE_EVENTS", "0") == "1"  # torch 2.10: "External events are disallowed in rocm"


def body():
    x = a
    for _ in range(40):  # ~several ms of work before the event
        x = torch.tanh(x @ a) * 0.01
    counter.add_(1)
    buf.copy_(counter.expand_as(buf) + x[0, 0] * 0)
    ev.record()
    y = a
    for _ in range(40):  # more work after the event inside the graph
        y = torch.tanh(y @ a) * 0.01
    return y


bad = 0
if PROBE_EVENTS:
  g = torch.cuda.CUDAGraph()
  with torch.cuda.stream(main):
      body()  # warm-up
      torch.cuda.synchronize()
      counter.zero_()
      with torch.cuda.graph(g, stream=main):
          body()
  torch.cuda.synchronize()
  counter.zero_()

  for i in range(1, 9):
      with torch.cuda.stream(main):
          g.replay()
      side.wait_event(ev)
      with torch.cuda.stream(side):
          out.copy_(buf)
      torch.cuda.synchronize()
      got = out[0].item()
      ok = got == float(i) and torch.all(out == out[0]).item()
      bad += not ok
      print(f"replay {i}: side stream read {got} -> {'PASS' if ok else 'FAIL (stale)'}")

  # timing: does the side-stream wait return before the graph's tail finishes (i.e. real overlap)?
  t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
  with torch.cuda.stream(main):
      t0.record(main)
      g.replay()
      t2.record(main)
  side.wait_event(ev)
  t1.record(side)
  torch.cuda.synchronize()
  print(f"graph start -> side release {t0.elapsed_time(t1):.3f} ms, graph start -> graph end {t0.elapsed_time(t2):.3f} ms")

if os.environ.get("PROBE_RCCL", "1") == "1":
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.ones(1 << 20, device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()
    try:
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        with torch.cuda.graph(g2, capture_error_mode=os.environ.get("PROBE_MODE", "thread_local")):
            x.mul_(2.0)
            w = dist.all_reduce(x, async_op=True)  # issued mid-graph, waited after more compute
            z = a
            for _ in range(10):
                z = torch.tanh(z @ a) * 0.01
            w.wait()
            x.add_(z[0, 0] * 0)
        for i in range(3):
            g2.replay()
        torch.cuda.synchronize()
        print("RCCL capture (async all_reduce inside the graph, 3 replays): x[0] =", x[0].item(),
              "PASS" if x[0].item() == 8.0 else "FAIL")
    except Exception as e:  # noqa: BLE001
        print("RCCL capture: FAIL", type(e).__name__, str(e)[:300])
    dist.destroy_process_group()
sys.exit(1 if bad else 0)
