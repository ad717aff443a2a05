#!/usr/bin/env python
"""Headline benchmark: Matcha-TTS training step on synthetic LJSpeech-shaped batches.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

`bench.py --gpus N` (N > 1) run without a launcher starts the N ranks itself: before any GPU call it runs
torch.distributed.run as a child process (one rank per GPU, 127.0.0.1, a free port) and exits with the
child's code.  Under a launcher, --gpus must equal WORLD_SIZE.  MTTS_BENCH_SHARED_GPU=1 puts every rank on
cuda:0 over gloo (a rehearsal of the multi-rank path on a one-GPU box; never a reported number).

A step = forward (text encoder, fp32 log-prior lattice, HIP maximum_path, CFM decoder) + backward +
grad-norm clip (1.0) + AdamW on B=32 utterances per GPU (Tx=120, Ty=600, 80 mels; BASELINE config 3),
one process per GPU, data parallel over RCCL.  By default the whole step is one captured HIP graph
replay (N>1: the graph also holds the bucketed RCCL all-reduces, forked off as backward completes
each bucket -- matcha/dp.py -- then clip+AdamW on the averaged flat gradients);
--no-graph runs it eagerly under DDP.  Inputs are resident in HBM before the timed region.
Rank 0 prints ONE JSON line: value = utterances/s over all ranks (max-over-ranks wall time), plus
  roofline      the dominant kernel (decoder conv_gemm_kernel): HIP events around each of its launches
                on the launch stream during one extra eager fwd+bwd after the timed region;
  maximum_path  Mcells/s and roofline_mas (HIP events around maximum_path on the batch's own lattice);
  cpu_baseline  (N=1) the oracle restatement of the reference step (same B, Tx, Ty) and the C
                restatement of the reference MAS (oracle/libmas_oracle.so) timed on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = ROOT / "matcha-tts-etu-upmc-ensam_amd"
sys.path[:0] = [str(PKG), str(ROOT)]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_DENSE_TFLOPS = 2500.0
FP32_MFMA_TFLOPS = 157.3


def decoder_train_flops(B: int, T: int) -> float:
    """3 x (12.05e6 T + 3072 T^2) FLOPs per utterance per train step."""
    return 3.0 * (12.05e6 * T + 3072.0 * T * T) * B


def cpu_baseline(B_cpu: int, Tx: int, Ty: int, budget_s: float) -> dict:
    """Reference CPU path timed on this host: the oracle's fp32 train step (train mode, dropout on)
    + clip + AdamW at the bench's own batch shape, and the MAS (the pinned C restatement)."""
    import numpy as np

    sys.path.insert(0, str(ROOT / "tests"))
    from oracle import matcha_oracle as MO  # cpu_baseline leg only
    import oracle_bind as OB

    def mp(value, mask):
        path, _ = OB.maximum_path(value.detach().numpy(), mask.detach().numpy())
        return torch.from_numpy(path)

    threads = torch.get_num_threads()
    torch.manual_seed(0)
    model = MO.MatchaTTSOracle(150, 80, 192, maximum_path=mp)
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-6)
    from matcha.training import synthetic_batch

    b = synthetic_batch(B_cpu, Tx, Ty, device="cpu")

    def step():
        dur, prior, diff, _ = model(b["x"], b["x_lengths"], b["y"], b["y_lengths"])
        (dur + prior + diff).backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)

    step()
    n, t0 = 0, time.perf_counter()
    while n < 3 or (time.perf_counter() - t0 < budget_s and n < 20):
        step()
        n += 1
    step_s = (time.perf_counter() - t0) / n
    out = {"value": round(B_cpu / step_s, 3), "unit": "utterances/s", "cores": threads, "kind": "port",
           "sample": f"{n} fp32 train steps (fwd+bwd+clip+AdamW, dropout on) of the oracle restatement "
                     f"(oracle/matcha_oracle.py) at B={B_cpu}, Tx={Tx}, Ty={Ty}; {threads} torch threads"}
    # MAS on the host: the C restatement oracle/libmas_oracle.so (pinned bit-exact to the reference
    # Cython, tests/test_oracle_golden.py); the compiled reference itself never travels to the GPU box
    rng = np.random.default_rng(0)
    Bm = 32
    value = rng.normal(-100.0, 10.0, size=(Bm, Tx, Ty)).astype(np.float32)
    t_x = np.full(Bm, Tx, np.int32)
    t_y = np.full(Bm, Ty, np.int32)
    kind = "port"

    def fn():
        OB.mas_batch(value, t_x, t_y)
    fn()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        fn()
        n += 1
    ms = (time.perf_counter() - t0) / n * 1e3
    out["mas"] = {"value": round(Bm * Tx * Ty / ms / 1e3, 1), "unit": "Mcells/s", "kind": kind,
                  "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                  "sample": f"{n} x compute_batch_alignments (oracle/mas_oracle.c) B={Bm} {Tx}x{Ty} "
                            f"({ms:.3f} ms each, incl. copy)"}
    out["cpu_model"] = _cpu_model()
    return out


def mas_chain_bound(Tx: int, Ty: int, mas_ms: float, clock_ghz: float = 2.1) -> dict:
    """Lower bound of the DP kernel that RUNS at this Tx (csrc/mas.hip ws_layout; VERDICT r4 #9: the round-4
    model described the one-wave kernel at every Tx, and the multi-wave kernel "beat" it).
    Tx <= 256 -- one wave per utterance (mas_dp_kernel): a Ty-long dependency chain; per column a lane updates
    its K = 1, 2, 4 rows (Tx <= 64, 128, 256) at about 9 VALU per row on the band edges (5 in interior chunks)
    plus a DPP neighbour exchange, each waiting ~8 cycles for its predecessor at one wave per SIMD.
    Tx > 256 -- eight waves per utterance (mas_dp_mw_kernel), KL = 1, 2, 4, 8 rows per lane (Tx <= 512 ... 4096),
    pipelined one 32-column chunk apart: per column two waves per SIMD each issue ~(5 KL + 4) instructions
    (interior cells + exchange / bookkeeping) at ~4 cycles each -- an ISSUE bound, ignoring the per-chunk
    synchronisation (a wave-to-wave LDS hand-over at KL <= 2, a workgroup barrier above) -- over Ty + 7 * 32
    columns (the pipeline fill).  measured / estimate >= 1 by construction; its size says how far the kernel is
    from the issue bound."""
    if Tx <= 256:
        K = 1 if Tx <= 64 else 2 if Tx <= 128 else 4
        cyc_per_col, cols, shape = (9 * K + 2) * 8, Ty, {"waves": 1, "rows_per_lane": K}
    else:
        KL = 1 if Tx <= 512 else 2 if Tx <= 1024 else 4 if Tx <= 2048 else 8
        cyc_per_col, cols, shape = 2 * (5 * KL + 4) * 4, Ty + 7 * 32, {"waves": 8, "rows_per_lane": KL}
    est_ms = cols * cyc_per_col / (clock_ghz * 1e9) * 1e3
    return {"columns": Ty, "kernel_shape": shape, "model_cycles_per_column": cyc_per_col,
            "estimate_ms": round(est_ms, 4), "measured_ns_per_column": round(mas_ms * 1e6 / Ty, 1),
            "measured_over_estimate": round(mas_ms / est_ms, 2), "clock_ghz_assumed": clock_ghz}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _bucketed_batches(B, Tx, Ty, n, rank, world, dev):
    """n length-bucketed batches for this rank: a synthetic corpus (Ty_i uniform in [Ty/4, Ty], Tx_i about
    Ty_i * Tx / Ty), the data path's LengthBucketBatchSampler (sorted pools, batches dealt over ranks) and
    collate with padding quanta 32 (text) / 256 (frames) -- the shapes a bucketed real-data run replays."""
    from matcha.data_management.ljspeech_datamodule import LengthBucketBatchSampler, collate

    g = torch.Generator().manual_seed(77)
    N = B * world * 64
    ty = (Ty * (0.25 + 0.75 * torch.rand(N, generator=g))).long().clamp(2, Ty)
    tx = torch.minimum((ty.float() * Tx / Ty * (0.8 + 0.2 * torch.rand(N, generator=g))).long().clamp(1, Tx), ty)
    sampler = LengthBucketBatchSampler(ty, B, num_replicas=world, rank=rank, bucket_batches=32, seed=0)
    out = []
    for idx in sampler:
        items = [dict(x=torch.randint(1, 150, (int(tx[i]),), generator=g), y=torch.randn(80, int(ty[i]), generator=g),
                      x_lengths=int(tx[i]), y_lengths=int(ty[i])) for i in idx]
        b = collate(items, x_quantum=32, y_quantum=256)
        out.append({k: v.to(dev) for k, v in b.items()})
        if len(out) == n:
            break
    return out


# kernel families of the step, by the kernel's own name in a rocprofv3 trace
FAMILIES = {
    "gemm": ("conv_gemm_kernel", "conv_gemm_glds_kernel", "conv_gemm_wreg_kernel", "splitk_epilogue_kernel"),
    # weight-gradient GEMMs + the step's batched fixed-order partial sums (reduce_partials_kernel: the split
    # slabs, and the LayerNorm / GroupNorm / bias partials that ride in the same launches)
    "wgrad": ("conv_wgrad_kernel", "reduce_partials_kernel"),
    "attn": ("attn_fwd_kernel", "attn_bwd_dq_kernel", "attn_bwd_dkv_kernel", "attn_drow_kernel",
             "attn_bwd_merged_kernel", "attn_fwd_short_kernel", "attn_bwd_dq_short_kernel", "attn_bwd_dkv_short_kernel"),
}


def _kname(full: str) -> str:
    import re

    m = re.search(r"::(\w+?)(<|\()", full) or re.search(r"(\w+)", full)
    return m.group(1) if m else full[:40]


def graph_replay_profile(args) -> dict:
    """Per-kernel durations INSIDE the graph-replayed step: this script re-run as a child under
    `rocprofv3 --kernel-trace` (warm-up + 4 timed steps, no other measurement), the trace cut at the step
    boundary (one replay = the fwd/bwd graph + the optimizer graph, ending in adamw_update_kernel), summed
    per kernel family over the last complete step.  The parent has made its own measurements already; the
    child runs after them."""
    import csv
    import shutil
    import subprocess
    import tempfile

    rp = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if Path("/opt/rocm/bin/rocprofv3").exists() else None)
    if rp is None:
        return {"error": "rocprofv3 not found"}
    d = tempfile.mkdtemp(prefix="mtts_prof_", dir="/tmp")
    cmd = [rp, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
           str(Path(__file__).resolve()), "--profile-child", "--steps", "4", "--warmup", "2", "--batch", str(args.batch),
           "--tx", str(args.tx), "--ty", str(args.ty), "--precision", args.precision]
    try:
        r = subprocess.run(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"), capture_output=True, text=True,
                           timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "rocprofv3 child timed out"}
    traces = sorted(Path(d).rglob("*kernel_trace.csv"))
    if r.returncode != 0 or not traces:
        return {"error": f"rocprofv3 child rc={r.returncode}: {r.stderr[-300:]}"}
    rows = sorted(csv.DictReader(open(traces[0])), key=lambda x: int(x["Start_Timestamp"]))
    ends = [i for i, x in enumerate(rows) if "adamw_update_kernel" in x["Kernel_Name"]]
    if len(ends) < 2:
        return {"error": "no complete step in the trace"}
    seg = rows[ends[-2] + 1: ends[-1] + 1]
    fam = {k: {"launches": 0, "us": 0.0} for k in FAMILIES}
    per_kernel = {}
    busy, t_end = 0.0, int(seg[0]["Start_Timestamp"])
    for x in seg:
        st_, en_ = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        busy += (en_ - max(st_, t_end)) / 1e3 if en_ > t_end else 0.0
        t_end = max(t_end, en_)
        k = _kname(x["Kernel_Name"])
        per_kernel[k] = per_kernel.get(k, 0.0) + (en_ - st_) / 1e3
        for f, names in FAMILIES.items():
            if k in names:
                fam[f]["us"] += (en_ - st_) / 1e3
                if k not in ("splitk_epilogue_kernel", "reduce_partials_kernel"):
                    fam[f]["launches"] += 1
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    top = sorted(per_kernel.items(), key=lambda kv: -kv[1])[:12]
    shutil.rmtree(d, ignore_errors=True)
    return {"families": fam, "kernels_per_step": len(seg), "step_span_us": round(span, 1),
            "step_busy_us": round(busy, 1), "top_kernels_us": {k: round(v, 1) for k, v in top}}


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn_ranks(n: int) -> int:
    """N ranks for `bench.py --gpus N` without a launcher: torch.distributed.run as a CHILD process (this
    process has made no GPU call and never execs), each rank re-entering this script with WORLD_SIZE set."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--tx", type=int, default=120)
    ap.add_argument("--ty", type=int, default=600)
    ap.add_argument("--precision", default="bf16-parity", choices=["32-true", "bf16-mixed", "bf16-parity"],
                    help="bf16-parity (default): bf16-mixed with split bf16 weight planes (but the decoder FF "
                         "up-projection) and the text encoder's forward on the exact-fp32 MFMA -- alignment exact, "
                         "losses within 1e-4 of 32-true; bf16-mixed: one weight plane (throughput mode, misses the "
                         "loss bar); 32-true: the reference's precision")
    ap.add_argument("--no-graph", action="store_true", help="eager step (DDP) instead of the captured HIP graph")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-synth", action="store_true", help="skip the synthesise (inference) measurement")
    ap.add_argument("--profile-child", action="store_true", help=argparse.SUPPRESS)  # graph_replay_profile's child
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the same-run 32-true line and the reference step shape (B=16 x accumulate 2)")
    ap.add_argument("--no-graph-profile", action="store_true",
                    help="skip the rocprofv3 graph-replay leg (roofline from the eager HIP-event pass only)")
    ap.add_argument("--accumulate", type=int, default=1,
                    help="N > 1: the step is N micro-batches of batch/N with gradient accumulation (the reference's "
                         "train.py:63,88 shape is --batch 32 --accumulate 2); profiling aid, not the headline")
    ap.add_argument("--bucketed", type=int, default=0,
                    help="N > 0: cycle N length-bucketed batches (LengthBucketBatchSampler + collate with padding "
                         "quanta) from a synthetic corpus with Ty in [Ty/4, Ty], Tx ~ Ty * tx/ty; --tx/--ty are "
                         "the corpus maxima (long-form config 5); N <= the Trainer's graph cache")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # MTTS_BENCH_SHARED_GPU=1: every rank on cuda:0 over gloo -- rehearses the multi-rank graph path on
        # a one-GPU box (RCCL refuses two ranks on one device); never used for reported numbers
        if os.environ.get("MTTS_BENCH_SHARED_GPU") == "1":
            local = 0
            torch.cuda.set_device(local)
            from matcha.dp import stdout_to_stderr

            with stdout_to_stderr():  # gloo's connect message stays off the JSON stdout
                dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # N>1: a host watchdog per rank (matcha/watchdog.py) -- a step that makes no progress within
    # the phase's bound prints rank, phase, graph key, last issued bucket and the device's last completed step /
    # bucket to stderr and ends the rank with exit code 3 (torch.distributed.run then stops its peers)
    wd = None
    wd_bounds = {"init_s": float(os.environ.get("MTTS_WATCHDOG_INIT_S", "600")),
                 "warmup_step_s": float(os.environ.get("MTTS_WATCHDOG_WARMUP_S", "300")),
                 "step_s": float(os.environ.get("MTTS_WATCHDOG_S", "60")),
                 "post_s": float(os.environ.get("MTTS_WATCHDOG_POST_S", "900"))}
    if world > 1:
        from matcha.watchdog import StepWatchdog

        wd = StepWatchdog(rank, wd_bounds["init_s"])
        wd.beat("init: process group up")
    if world == 1 and os.environ.get("MTTS_FORCE_DP") == "1":
        # rehearsal of the data-parallel step on one GPU: a world-size-1 RCCL group, so the bucketed
        # all-reduces run (as copies) exactly as at N>1; never used for reported numbers
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)

    import matcha.utils.monotonic_align as MA
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import TrainConfig, Trainer, synthetic_batch

    torch.manual_seed(1234)  # identical init on every rank (DDP also broadcasts rank 0's weights)
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev)
    model.train()
    graph = not args.no_graph
    trainer = Trainer(model, TrainConfig(precision=args.precision, graph=graph, graph_cache=max(4, args.bucketed),
                                         accumulate_grad_batches=args.accumulate))
    if wd is not None:
        from matcha.watchdog import DeviceProgress

        trainer.progress = wd.device = DeviceProgress()
        trainer.watchdog = wd
        wd.beat("warm-up (step 0: backward order, bucket layout, RCCL communicator, graph capture)",
                bound_s=wd_bounds["warmup_step_s"])
    B, Tx, Ty = args.batch, args.tx, args.ty
    if args.bucketed > 0:
        batches = _bucketed_batches(B, Tx, Ty, args.bucketed, rank, world, dev)
        batch = batches[0]
        args.warmup = max(args.warmup, 2 * len(batches))  # every padded shape captured before timing
    else:
        batch = synthetic_batch(B, Tx, Ty, seed=1000 + rank, device=dev)
        batches = [batch]
    acc = args.accumulate
    if acc > 1:  # micro-batches of B / acc (the same synthetic generator, one seed each)
        if args.bucketed or B % acc:
            raise SystemExit("bench.py: --accumulate needs --batch divisible by it and no --bucketed")
        micro = [synthetic_batch(B // acc, Tx, Ty, seed=2000 + i, device=dev) for i in range(acc)]

    mas_events: list = []
    real_mp = MA.maximum_path

    def step_batches(i):
        return micro if acc > 1 else [batches[i % len(batches)]]

    for i in range(args.warmup):
        trainer.step(step_batches(i))
        if wd is not None:  # untimed: each warm-up step completes before the next (a hang names its step)
            torch.cuda.synchronize()
            wd.beat("warm-up", last_step_done=i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if wd is not None:
        wd.beat("timed", bound_s=wd_bounds["step_s"])
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.step(step_batches(i))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0, -(t1 - t0)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    rank_spread = {"step_ms_max_over_ranks": round(float(elapsed[0]) / args.steps * 1e3, 3),
                   "step_ms_min_over_ranks": round(-float(elapsed[1]) / args.steps * 1e3, 3)}
    rank_spread["max_over_min"] = round(float(elapsed[0]) / max(-float(elapsed[1]), 1e-12), 4)
    elapsed = float(elapsed[0].item())
    if wd is not None:
        wd.beat("data-parallel tail measurement", last_step_done=args.warmup + args.steps - 1)
    # the exposed tail bucket: one extra eager fwd+bwd with the reducer armed (every rank, no update)
    dp_tail = trainer.measure_dp_tail(step_batches(0)) if trainer.reducer is not None else None
    if wd is not None:
        wd.beat("after the data-parallel legs (rank-local measurements)", bound_s=wd_bounds["post_s"])
    if args.profile_child:  # under rocprofv3 (graph_replay_profile): the trace is all that is wanted
        return
    losses = trainer.last_losses.tolist()
    if args.bucketed > 0:  # the per-batch measurements below run on batches[0]'s padded shape
        Tx, Ty = int(batch["x"].shape[1]), int(batch["y"].shape[2])

    # time maximum_path with HIP events on THIS batch's fp32 lattice (same kernels, same stream),
    # right after the timed region; the step itself runs the fused lattice + DP
    # (prior_maximum_path), timed beside it
    from matcha.utils.model import sequence_mask

    with torch.no_grad():
        mu_x, _, x_mask = model.encoder(batch["x"], batch["x_lengths"])
        lp = model.log_prior(mu_x, batch["y"])
        y_mask = sequence_mask(batch["y_lengths"], Ty).unsqueeze(1).float()
        am = (x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1).contiguous()
        for _ in range(3):
            real_mp(lp, am)
        mas_events.clear()
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            real_mp(lp, am)
            e1.record()
            mas_events.append((e0, e1))
        fev = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            MA.prior_maximum_path(mu_x, batch["y"], batch["x_lengths"], batch["y_lengths"])
            e1.record()
            fev.append((e0, e1))
    torch.cuda.synchronize()
    fused_ms = sum(a.elapsed_time(b) for a, b in fev) / len(fev)
    # dominant kernel: the decoder's implicit-GEMM conv/linear (conv_gemm_kernel, fwd + dgrad).  One
    # more eager fwd+bwd of the same batch (after the timed region, results discarded) with HIP events
    # around every launch on its stream; algorithmic FLOPs = 2*M*N*K per launch.
    from matcha.models.components import _ops as OPS

    for rep in range(2):
        OPS.LAUNCH_LOG, OPS.WGRAD_LOG, OPS.ATTN_LOG = [], [], []
        trainer._fwd_bwd([batch])
        torch.cuda.synchronize()
    gemm_log, OPS.LAUNCH_LOG = OPS.LAUNCH_LOG, None
    if os.environ.get("MTTS_DUMP_GEMM_LOG"):  # per-launch shapes + eager times (tools/r5/gemm_replay.py input)
        with open(os.environ["MTTS_DUMP_GEMM_LOG"], "w") as fh:
            for e0, e1, fl, pr, nby, info in gemm_log:
                fh.write(json.dumps(dict(info, us=round(e0.elapsed_time(e1) * 1e3, 2), bytes=nby)) + "\n")
    wgrad_log, OPS.WGRAD_LOG = OPS.WGRAD_LOG, None
    attn_log, OPS.ATTN_LOG = OPS.ATTN_LOG, None
    model.zero_grad(set_to_none=False)

    # inference: MatchaTTS.synthesise on the same text batch, 10 Euler steps, the ODE
    # replayed as one HIP graph; length_scale 5 gives LJSpeech-like ~5 frames per token
    synth = None
    if not args.no_synth:
        model.eval()
        amp = torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.precision != "32-true")
        pol = OPS.parity_policy(args.precision == "bf16-parity")
        with torch.inference_mode(), amp, pol:
            xs, xls = batch["x"], batch["x_lengths"]
            for _ in range(2):
                out = model.synthesise(xs, xls, 10, length_scale=5.0)
            torch.cuda.synchronize()
            reps, t0s = 5, time.perf_counter()
            for _ in range(reps):
                out = model.synthesise(xs, xls, 10, length_scale=5.0)
            torch.cuda.synchronize()
            syn_ms = (time.perf_counter() - t0s) / reps * 1e3
        frames = int(out["mel_lengths"].sum().item())
        audio_s = frames * 256 / 22050
        synth = {"n_timesteps": 10, "batch": B, "frames": frames, "padded_frames": int(out["decoder_outputs"].shape[-1]),
                 "ms_per_call": round(syn_ms, 2), "rtf": round(syn_ms / 1e3 / audio_s, 6),
                 "frames_per_s": round(frames / (syn_ms / 1e3), 1),
                 "precision": args.precision,
                 "note": "wall clock incl. host sync for the predicted lengths; random-init weights, length_scale 5"}
        model.train()

    # bf16-mixed vs 32-true with the parity tests' weights and batch (tests/test_headline_gpu.py::
    # test_bench_batch_b32_vs_oracle: recipe weights 43, synthetic batch seed 1000 -- the bench batch --, t / z
    # from a CPU generator seeded 44; the 32-true path equals the CPU oracle there, losses to 0 relative)
    precision_check = None
    if args.precision != "32-true" and not args.bucketed and (B, Tx, Ty) == (32, 120, 600):
        sys.path.insert(0, str(ROOT / "tests"))
        from golden.weights_recipe import apply_recipe

        pm = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev)
        apply_recipe(pm, 43)
        pm.eval()
        pb = synthetic_batch(32, 120, 600, seed=1000, device=dev)
        gen = torch.Generator().manual_seed(44)
        t_inj = torch.rand(32, 1, 1, generator=gen).to(dev)
        z_inj = torch.randn(32, 80, 600, generator=gen).to(dev)
        res = {}
        # (name, autocast, split weight planes, text encoder precision)
        modes = (("32-true", False, False, "bf16"), ("one_plane", True, False, "bf16"),
                 ("split_weights", True, True, "bf16"), ("parity_policy", True, True, OPS.encoder_precision_for_parity()),
                 ("parity_bf16x3_encoder", True, True, "bf16x3"), ("parity_bf16x6_encoder", True, True, "bf16x6"),
                 ("parity_fp32fwd_encoder", True, True, "fp32fwd"), ("parity_fp32_encoder", True, True, "fp32"))
        from matcha.precision import error_attribution, grad_errors, loss_and_grads, precision_context

        trainer_modes = {"32-true": "32-true", "one_plane": "bf16-mixed", "parity_policy": "bf16-parity"}
        with torch.no_grad():
            for name, amp_on, split, enc in modes:
                if name in trainer_modes:  # the Trainer's own numerics (matcha.precision.precision_context)
                    with precision_context(trainer_modes[name], pm):
                        out = pm(pb["x"], pb["x_lengths"], pb["y"], pb["y_lengths"], t=t_inj, z=z_inj)
                else:
                    old = OPS.set_weight_split(split)
                    pm.encoder_precision = enc
                    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp_on):
                        out = pm(pb["x"], pb["x_lengths"], pb["y"], pb["y_lengths"], t=t_inj, z=z_inj)
                    OPS.set_weight_split(old)
                    pm.encoder_precision = None
                res[name] = ([float(v) for v in out[:3]], out[3].detach())
        # gradients + one clip / AdamW update of the benched precision (and the one-plane mode) vs 32-true
        # (matcha/precision.py)
        _, g32, _ = loss_and_grads(pm, pb, "32-true", t=t_inj, z=z_inj)
        params = {n: q.detach() for n, q in pm.named_parameters()}
        grads_check = {}
        for name in ("parity_policy", "one_plane"):
            _, gm, _ = loss_and_grads(pm, pb, trainer_modes[name], t=t_inj, z=z_inj)
            grads_check[name] = {k: (round(v, 7) if isinstance(v, float) else v)
                                 for k, v in grad_errors(gm, g32, params).items()}
        # which module family's bf16 arithmetic the benched precision's gradient error comes from
        run_mode = "parity_policy" if args.precision == "bf16-parity" else "one_plane"
        grads_check["attribution"] = error_attribution(pm, pb, trainer_modes[run_mode], g32, t=t_inj, z=z_inj)
        del pm, g32, gm
        l32, a32 = res["32-true"]

        def errs(name):
            l16, a16 = res[name]
            return {"loss_rel_err": [round(abs(a - b) / abs(b), 7) for a, b in zip(l16, l32)],
                    "alignment_cell_agreement": round(float((a16 == a32).float().mean().item()), 6)}

        precision_check = {
            "bf16_loss_rel_err": errs(run_mode)["loss_rel_err"],
            "run_mode": run_mode,
            "modes": {k: errs(k) for k in ("one_plane", "split_weights", "parity_policy", "parity_bf16x3_encoder",
                                           "parity_bf16x6_encoder", "parity_fp32fwd_encoder", "parity_fp32_encoder")},
            "grads": grads_check,
            "grads_note": "fwd + bwd of the same batch (eval mode) in each precision: gradient vs 32-true's "
                          "(global and per-tensor relative L2 error, the global norm's relative error) and one "
                          "clip(1.0) + AdamW(1e-4) update from zero moments (train.py:85 32-true is the reference "
                          "precision; the bf16 modes' backward runs in bf16).  attribution: the benched precision "
                          "with one module family held in 32-true at a time (matcha/precision.py hold_fp32): "
                          "source_share = 1 - (e_held / e)^2; lands_share = where the squared error sits",
            "losses": ["dur", "prior", "diff"],
            "bar": "alignment bit-exact (agreement 1.0), mel / flow-matching loss within 1e-4 relative (north star)",
            "note": "bf16 modes vs 32-true (= the oracle at this batch) with the parity tests' recipe weights and "
                    "batch, eval mode, same t / z.  one_plane: bf16 weights (the fp32 weights' rounding is the "
                    "error); split_weights: hi + rounding-residual bf16 planes; parity_policy (bench default, "
                    "--precision bf16-parity): split weights + the text encoder's forward fp32-faithful (policy: "
                    "see config.text_encoder_forward; backward bf16); parity_bf16x3_encoder: the encoder forward in "
                    "bf16x3 (split A and W operands, three bf16 MFMAs); parity_bf16x6_encoder: in bf16x6 (three exact "
                    "planes per operand, six MFMAs); parity_fp32fwd_encoder: on the exact-fp32 MFMA (32-true's "
                    "forward arithmetic); parity_fp32_encoder: split weights + the whole text encoder in exact fp32, "
                    "backward too (round 3's policy)"}

    # same-run extra lines (N=1): the reference precision (32-true: exact fp32 MFMA) on the bench workload,
    # and the reference's own step shape -- 2 micro-batches of 16 with gradient accumulation
    # (train.py:63,85,88: batch_size 16, accumulate_grad_batches 2) -- in the bench precision
    extra = None
    if world == 1 and not args.no_extra and not args.bucketed and graph:
        extra = {}
        # (name, Trainer precision, micro-batch, accumulate, MatchaTTS.encoder_precision override)
        lines = [("32-true", "32-true", B, 1, None), ("reference_step_16x2", args.precision, B // 2, 2, None)]
        if args.precision != "32-true":
            lines.append(("bf16_one_plane", "bf16-mixed", B, 1, None) if args.precision == "bf16-parity" else
                         ("bf16_parity", "bf16-parity", B, 1, None))
            lines.append(("bf16_parity_fp32_encoder", "bf16-parity", B, 1, "fp32"))
            if args.precision == "bf16-parity":  # the other fp32-faithful encoder forward: bf16x6 (three planes)
                lines.append(("bf16_parity_alt_encoder", "bf16-parity", B, 1,
                              "fp32fwd" if OPS.encoder_precision_for_parity() == "bf16x6" else "bf16x6"))
        # the data-parallel step's own cost on one GPU: a world-size-1 RCCL group, the bucketed in-graph
        # all-reduces (copies at one rank), the per-bucket side-stream weight-gradient flushes and packing
        lines.append(("dp_forced_n1", args.precision, B, 1, None))
        for name, prec, micro, acc, enc in lines:
            if name == "dp_forced_n1" and not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ["MASTER_PORT"] = str(_free_port())
                dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
            torch.manual_seed(1234)
            m2 = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
            m2.encoder_precision = enc
            tr2 = Trainer(m2, TrainConfig(precision=prec, graph=True, accumulate_grad_batches=acc,
                                          force_dp=name == "dp_forced_n1"))
            bs2 = [synthetic_batch(micro, Tx, Ty, seed=2000 + i, device=dev) for i in range(acc)]
            for _ in range(3):
                tr2.step(bs2)
            n2 = max(5, args.steps // 2)
            torch.cuda.synchronize()
            t0x = time.perf_counter()
            for _ in range(n2):
                tr2.step(bs2)
            torch.cuda.synchronize()
            ms2 = (time.perf_counter() - t0x) / n2 * 1e3
            extra[name] = {"ms_per_step": round(ms2, 3), "utterances_per_s": round(micro * acc / ms2 * 1e3, 2),
                           "steps": n2, "precision": prec, "micro_batch": micro, "accumulate_grad_batches": acc,
                           "weight_planes": 2 if prec == "bf16-parity" else 1,
                           "encoder": enc or (OPS.encoder_precision_for_parity() if prec == "bf16-parity"
                                              else "as the precision"),
                           **({"dp": {"ranks": int(tr2.reducer.comm.ranks), "buckets": len(tr2.reducer.buckets),
                                      "overlapped_in_graph": bool(next(iter(tr2._graphs.values()))["overlap"])}}
                              if tr2.reducer is not None else {}),
                           "losses": [round(v, 5) for v in tr2.last_losses.tolist()]}
            del tr2, m2
        torch.cuda.empty_cache()

    mas_ms = sum(a.elapsed_time(b) for a, b in mas_events) / max(len(mas_events), 1)
    cells = B * Tx * Ty
    mas_gbs = 12.0 * cells / (mas_ms * 1e-3) / 1e9
    step_ms = elapsed / args.steps * 1e3
    flops = decoder_train_flops(B, Ty)
    gemm_peak = FP32_MFMA_TFLOPS if args.precision == "32-true" else BF16_DENSE_TFLOPS
    ridge = gemm_peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    # the kernels' durations inside the graph replay that was benchmarked (rocprofv3 child, N=1 only);
    # the eager HIP-event pass above stays as the secondary figure
    gprof = None
    if world == 1 and not args.no_graph_profile and graph:
        gprof = graph_replay_profile(args)

    def traffic_of(name):
        """PMC HBM bytes per launch of this family on THIS workload (tools/r3/pmc_families.sh ->
        profiles/<round>/<name>_traffic.json: FETCH_SIZE x2 + WRITE_SIZE, separate passes); PMC passes
        serialise kernels, so they are not collected inside the bench."""
        if (B, Tx, Ty) != (32, 120, 600) or args.precision == "32-true" or args.bucketed:
            return None, None
        suffix = "_parity" if args.precision == "bf16-parity" else ""
        found = sorted(ROOT.glob(f"profiles/r*/{name}_traffic{suffix}.json"))
        if not found:
            return None, None
        return json.loads(found[-1].read_text())["traffic_bytes_per_launch"], str(found[-1].relative_to(ROOT))

    mas_traffic = traffic_of("mas")  # tools/r5/pmc_mas.sh: maximum_path on the bench batch's lattice

    def roofline_of(log, fam, kernel, note):
        """Roofline line of one kernel family: algorithmic FLOPs / bytes per step from the eager launch log
        (the same launches the graph replays), time from the graph-replay profile when it ran (else the
        eager HIP events); bound from the arithmetic intensity vs the ridge point."""
        if not log:
            return None
        ms = [r[0].elapsed_time(r[1]) for r in log]
        t_eager = sum(ms) * 1e-3
        fl, by = sum(r[2] for r in log), sum(r[4] for r in log)
        g = (gprof or {}).get("families", {}).get(fam) if gprof and "families" in gprof else None
        src = "graph" if g and g["us"] > 0 else "eager"
        t = g["us"] * 1e-6 if src == "graph" else t_eager
        n = len(log)
        tf, gb = fl / t / 1e12, by / t / 1e9
        ai = fl / max(by, 1)
        traffic, tsrc = traffic_of(fam)
        gl = g["launches"] if g else None
        line = {"kernel": kernel, "timing": src, "launches_per_step": n,
                "graph_launches_per_step": gl,
                "avg_launch_us": round(t / n * 1e6, 2),
                "avg_launch_unit": "per logical launch (one GEMM job of the eager log; the batched weight-gradient "
                                   "launches of the graph hold several jobs each) -- time and bytes over the same jobs",
                "avg_graph_launch_us": round(t / gl * 1e6, 2) if gl else None,
                "algorithmic_flops_per_launch": round(fl / n), "algorithmic_bytes_per_launch": round(by / n),
                "arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(ridge, 1),
                "mfma_tflops": round(tf, 1), "mfma_frac": round(tf / gemm_peak, 4), "hbm_gbs": round(gb, 1),
                "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": tsrc,
                "eager_events": {"avg_launch_us": round(t_eager / n * 1e6, 2), "hbm_gbs": round(by / t_eager / 1e9, 1),
                                 "frac": round(by / t_eager / 1e9 / HBM_PEAK_GBS, 4)},
                "note": note}
        if ai < ridge:
            return {"bound": "hbm", "achieved": round(gb, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gb / HBM_PEAK_GBS, 4), **line}
        return {"bound": "mfma", "achieved": round(tf, 1), "peak": gemm_peak, "unit": "TFLOP/s",
                "frac": round(tf / gemm_peak, 4), **line}

    gemm_roofline = roofline_of(
        gemm_log, "gemm", "conv_gemm_kernel + conv_gemm_glds_kernel + conv_gemm_wreg_kernel (+ splitk_epilogue_kernel): "
        "decoder + encoder implicit-GEMM conv / linear, forward and dgrad",
        "time = the family's kernel time in one graph-replayed step (rocprofv3 trace of this command's child) / "
        "launches; bytes = A rows read once + packed W (both planes when split) + C written (+ aux / residual / "
        "pre-activation streams) per launch; FLOP = 2 M N K")
    roofline_wgrad = roofline_of(
        wgrad_log, "wgrad", "conv_wgrad_kernel + reduce_partials_kernel (weight-gradient GEMMs, batched up to 12 jobs "
        "per launch, and the step's batched fixed-order partial sums, which also hold the LayerNorm / GroupNorm gamma / "
        "beta partials)",
        "2 M N K FLOP; bytes = dY + unique A rows + dW; graph time includes the whole batched reduce (the norms' "
        "partial sums too: an upper bound on the GEMMs' own time)")
    roofline_attn = roofline_of(
        attn_log, "attn", "attn_fwd + backward (Drow pre-pass + merged dQ / dK-dV launch) kernels, long (decoder) and short (encoder, T <= 128)",
        "FLOP = 4 B H T^2 D fwd, 8 B H T^2 D bwd (standard flash-attention accounting, recomputation not counted); "
        "bytes = q, k, v, o (+ dO, dq, dk, dv) once")

    if rank == 0:
        rec = {
            "metric": "training utterances/sec (whole node) + maximum_path Mcells/sec, LJSpeech batch=32",
            "value": round(world * B * args.steps / elapsed, 2),
            "unit": "utterances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.precision == "32-true" else "bf16",
            "data": "synthetic LJSpeech-shaped batches (random tokens/mels, ragged lengths), random-init weights",
            "config": {"workload": f"MatchaTTS train step (encoder + MAS + CFM decoder fwd/bwd + clip + AdamW), "
                                   f"B={B}/GPU, Tx={Tx}, Ty={Ty}, 80 mels",
                       "model": "MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192)",
                       "global_batch": world * B, "seq_len": Ty, "text_len": Tx, "parallelism": f"dp{world}",
                       "precision": args.precision, "hip_graph": graph,
                       "weight_planes": 2 if (args.precision == "bf16-parity" or
                                              (OPS.weight_split_enabled() and args.precision == "bf16-mixed")) else 1,
                       **({"text_encoder_forward": OPS.encoder_precision_for_parity() + " (backward bf16)"}
                          if args.precision == "bf16-parity" else {}),
                       **({"bucketed_batches": [[int(v) for v in (b["x"].shape[1], b["y"].shape[2],
                                                                     b["x_lengths"].min(), b["y_lengths"].min())]
                                                for b in batches],
                           "bucketed_note": "per batch: padded Tx, padded Ty, min x_len, min y_len "
                                            "(LengthBucketBatchSampler, collate quanta 32 / 256); corpus maxima "
                                            f"Tx={args.tx}, Ty={args.ty}; the per-call lines below use batch 0"}
                          if args.bucketed > 0 else {})},
            "maximum_path": {"value": round(world * cells / mas_ms / 1e3, 1), "unit": "Mcells/s (whole node)",
                             "ms_per_call": round(mas_ms, 4), "calls": len(mas_events),
                             "fused_prior_maximum_path_ms": round(fused_ms, 4),
                             "fused_note": "what the step runs: log-prior lattice from mu_x / y + DP + durations "
                                           "+ frame rows (mtts_prior_maximum_path)"},
            "roofline": gemm_roofline,
            "roofline_wgrad": roofline_wgrad,
            "roofline_attn": roofline_attn,
            "graph_replay_profile": gprof,
            "extra_configs": extra,
            "roofline_mas": {"kernel": "mas_transpose_kernel + mas_dp_kernel (Tx <= 256) / mas_dp_mw_kernel + mas_expand_kernel (maximum_path)",
                             "bound": "hbm",
                             "achieved": round(mas_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(mas_gbs / HBM_PEAK_GBS, 4), "traffic": mas_traffic[0],
                             "traffic_source": mas_traffic[1],
                             "traffic_unit": "HBM bytes per maximum_path call (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                             "algorithmic_bytes_per_launch": 12 * cells,
                             "chain_bound": mas_chain_bound(Tx, Ty, mas_ms),
                             "note": "12 B/cell (value+mask read, path write); the API premasks + transposes the "
                                     "lattice once (column-major DP loads) from Tx > 128; the DP is chain / issue "
                                     "bound: one wave per utterance up to Tx = 256, eight pipelined waves beyond "
                                     "(chain_bound names the kernel shape that ran)"},
            "decoder_mfma": {"train_flops_per_step": flops,
                             "achieved_tflops_step": round(flops / (step_ms * 1e-3) / 1e12, 2),
                             "peak_tflops": FP32_MFMA_TFLOPS if args.precision == "32-true" else BF16_DENSE_TFLOPS},
            "losses": [round(v, 5) for v in losses],
            "dp": None if trainer.reducer is None else {
                "ranks": int(trainer.reducer.comm.ranks), "transport": type(trainer.reducer.comm).__name__,
                "backend": trainer.reducer.comm.backend,
                "rccl_version": getattr(trainer.reducer.comm, "version", None),
                "shared_gpu": os.environ.get("MTTS_BENCH_SHARED_GPU") == "1",
                "buckets": len(trainer.reducer.buckets), "bucket_mb": trainer.cfg.bucket_mb,
                "flat_floats": trainer.reducer.flat.numel(),
                "overlapped_in_graph": bool(next(iter(trainer._graphs.values()))["overlap"]) if trainer._graphs else None,
                "rank_step_time": rank_spread,
                "tail": dp_tail,
                "agree_shapes": trainer.cfg.agree_shapes,
                "agree_shapes_note": "on (default): every rank pads to the max padded Tx / Ty over ranks, so all ranks "
                                     "replay one graph; a rank's losses then depend on its peers' padded lengths "
                                     "(GroupNorm statistics, conv bias in padded frames -- SURVEY 0.6)",
                "grad_semantics": "after a step each .grad holds the SUM over ranks; the fused clip + AdamW applies "
                                  "the 1 / world mean (GradBucketReducer.mean_grads() gives DDP's means)",
                "watchdog": None if wd is None else dict(wd_bounds, exit_code=wd.exit_code)},
            "precision_check": precision_check,
            "synthesise": synth,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(B, Tx, Ty, args.cpu_budget)
        print(json.dumps(rec), flush=True)
    if wd is not None:
        wd.beat("teardown", bound_s=120.0)
    if dist.is_initialized():
        dist.destroy_process_group()
    if wd is not None:
        wd.stop()


if __name__ == "__main__":
    main()
