"""The data-parallel watchdog (matcha/watchdog.py) on CPU: two gloo ranks of the Trainer's bucketed
gradient exchange, one of them deliberately stalled before it joins a bucket's all-reduce.  The other rank must
end within the bound with exit code 3 and a stderr line that names its rank, the phase, the step and the bucket it
was blocked in; the stalled rank's own watchdog ends it the same way.  Plus the single-process contract: progress
keeps a watchdog quiet, a stop() ends it, and the report carries every field bench.py's N>1 path sets."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

RANK_SCRIPT = r"""
import os, sys, time
root, rank, world, port, stall_step, stall_bucket, bound = sys.argv[1], *map(int, sys.argv[2:7]), float(sys.argv[7])
sys.path[:0] = [os.path.join(root, "matcha-tts-etu-upmc-ensam_amd"), root, os.path.join(root, "tests")]
import torch, torch.distributed as dist
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
dist.init_process_group("gloo", rank=rank, world_size=world)
from matcha.training import TrainConfig, Trainer, synthetic_batch
from matcha.watchdog import StepWatchdog
from test_distributed_cpu import TinyTTS
torch.manual_seed(0)
tr = Trainer(TinyTTS(), TrainConfig(precision="32-true", graph=False, dp="buckets", bucket_mb=0.001))
wd = StepWatchdog(rank, bound)
tr.watchdog = wd
wd.beat("timed")
for step in range(6):
    if step == stall_step and rank == 1:  # this rank stops before it joins bucket `stall_bucket`'s all-reduce
        real = tr.reducer.comm.all_reduce_
        def stalled(t, _real=real):
            if tr.reducer._issued == stall_bucket:
                time.sleep(600)
            _real(t)
        tr.reducer.comm.all_reduce_ = stalled
    tr.step([synthetic_batch(4, 12, 40, seed=100 + rank + 7 * step, device="cpu")])
    print(f"rank {rank} step {step} done", flush=True)
wd.stop()
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_stalled_rank_is_named_and_peers_exit_within_the_bound():
    port, bound = _free_port(), 4.0
    env = dict(os.environ, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, "-c", RANK_SCRIPT, str(ROOT), str(r), "2", str(port), "2", "1", str(bound)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env) for r in range(2)]
    t0 = time.monotonic()
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=120))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.monotonic() - t0
    codes = [p.returncode for p in procs]
    assert codes == [3, 3], (codes, [o[1][-2000:] for o in outs])
    assert elapsed < 90, elapsed
    for r, (out, err) in enumerate(outs):
        assert "rank %d step 1 done" % r in out  # two good steps first
        assert "step 2 done" not in out
        line = next(l for l in err.splitlines() if l.startswith("[mtts watchdog]"))
        assert f"rank {r}: no progress" in line and "(bound 4 s)" in line
        assert "bucket_issued=1 of 3" in line, line  # the bucket whose all-reduce never completed
        assert "last_step_enqueued=1" in line and "step_enqueueing=2" in line, line
        assert "phase=timed" in line and "device=n/a" in line, line


WD_SCRIPT = r"""
import os, sys, time
sys.path[:0] = [os.path.join(sys.argv[1], "matcha-tts-etu-upmc-ensam_amd")]
from matcha.watchdog import StepWatchdog
wd = StepWatchdog(5, 1.5, poll_s=0.05)
for i in range(8):  # 2 s of steady progress: quiet
    time.sleep(0.25)
    wd.beat("timed", last_step_done=i, graph_key="B32xTx120xTy600")
wd.note(bucket_issued=2, buckets=3)
if sys.argv[2] == "stop":
    wd.stop()
    time.sleep(2.5)
    print("stopped cleanly", flush=True)
    sys.exit(0)
time.sleep(30)
"""


def test_watchdog_quiet_under_progress_fires_when_idle_and_stops():
    r = subprocess.run([sys.executable, "-c", WD_SCRIPT, str(ROOT), "idle"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, r.stderr
    line = r.stderr.strip().splitlines()[-1]
    assert line.startswith("[mtts watchdog] rank 5: no progress for") and "(bound 2 s)" in line, line
    for f in ("phase=timed", "last_step_done=7", "graph_key=B32xTx120xTy600", "bucket_issued=2 of 3"):
        assert f in line, (f, line)
    r = subprocess.run([sys.executable, "-c", WD_SCRIPT, str(ROOT), "stop"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "stopped cleanly" in r.stdout, r.stderr
