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
    """The DP is a Ty-long dependency chain per utterance (one wave each, utterances in parallel on
    their own CUs): per column a lane updates its K = ceil(Tx / 64) rows (about 9 dependent VALU
    instructions per row -- score, compare, select, add, band test, backpointer shift/or) plus one
    DPP neighbour exchange, each waiting ~8 cycles for its predecessor at one wave per SIMD.  The
    estimate is that chain's length; measured / estimate near 1 means the kernel runs at its chain
    bound, not at HBM speed (which the 12 B/cell roofline would ask for)."""
    K = 1
    while 64 * K < Tx:
        K *= 2
    cyc_per_col = (9 * K + 2) * 8
    est_ms = Ty * cyc_per_col / (clock_ghz * 1e9) * 1e3
    return {"columns": Ty, "rows_per_lane": K, "model_cycles_per_column": cyc_per_col,
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
    ap.add_argument("--precision", default="bf16-mixed", choices=["32-true", "bf16-mixed"])
    ap.add_argument("--no-graph", action="store_true", help="eager step (DDP) instead of the captured HIP graph")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-synth", action="store_true", help="skip the synthesise (inference) measurement")
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
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
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
    trainer = Trainer(model, TrainConfig(precision=args.precision, graph=graph, graph_cache=max(4, args.bucketed)))
    B, Tx, Ty = args.batch, args.tx, args.ty
    if args.bucketed > 0:
        batches = _bucketed_batches(B, Tx, Ty, args.bucketed, rank, world, dev)
        batch = batches[0]
        args.warmup = max(args.warmup, 2 * len(batches))  # every padded shape captured before timing
    else:
        batch = synthetic_batch(B, Tx, Ty, seed=1000 + rank, device=dev)
        batches = [batch]

    mas_events: list = []
    real_mp = MA.maximum_path

    for i in range(args.warmup):
        trainer.step([batches[i % len(batches)]])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.step([batches[i % len(batches)]])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
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
    wgrad_log, OPS.WGRAD_LOG = OPS.WGRAD_LOG, None
    attn_log, OPS.ATTN_LOG = OPS.ATTN_LOG, None
    model.zero_grad(set_to_none=False)
    gemm_ms = [r[0].elapsed_time(r[1]) for r in gemm_log]
    gemm_flops = sum(r[2] for r in gemm_log)
    gemm_bytes = sum(r[4] for r in gemm_log)
    gemm_avg_us = sum(gemm_ms) / max(len(gemm_ms), 1) * 1e3
    gemm_tflops = gemm_flops / (sum(gemm_ms) * 1e-3) / 1e12 if gemm_ms else 0.0

    # inference: MatchaTTS.synthesise on the same text batch, 10 Euler steps, the ODE
    # replayed as one HIP graph; length_scale 5 gives LJSpeech-like ~5 frames per token
    synth = None
    if not args.no_synth:
        model.eval()
        amp = torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.precision == "bf16-mixed")
        with torch.inference_mode(), amp:
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

    # bf16-mixed vs 32-true on the bench batch (SURVEY 7 "hard parts"): the same weights, tokens, mels and
    # injected t / z, eval mode; the 32-true product path equals the CPU oracle at this batch (losses to
    # 0 relative, alignment bit-exact: tests/test_headline_gpu.py::test_bench_batch_b32_vs_oracle)
    precision_check = None
    if args.precision == "bf16-mixed":
        model.eval()
        gen = torch.Generator(device=dev).manual_seed(44)
        t_inj = torch.rand(B, 1, 1, generator=gen, device=dev)
        z_inj = torch.randn(B, 80, Ty, generator=gen, device=dev)
        res = {}
        with torch.no_grad():
            for prec in ("32-true", "bf16-mixed"):
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec == "bf16-mixed"):
                    out = model(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"], t=t_inj, z=z_inj)
                res[prec] = ([float(v) for v in out[:3]], out[3].detach())
        model.train()
        l32, a32 = res["32-true"]
        l16, a16 = res["bf16-mixed"]
        precision_check = {
            "bf16_loss_rel_err": [round(abs(a - b) / abs(b), 6) for a, b in zip(l16, l32)],
            "losses": ["dur", "prior", "diff"],
            "alignment_cell_agreement": round(float((a16 == a32).float().mean().item()), 6),
            "note": "bf16-mixed vs the 32-true path (= the oracle at this batch) on the bench batch, eval mode, "
                    "same t / z; the duration loss moves with MAS boundary flips (tests/test_headline_gpu.py)"}

    mas_ms = sum(a.elapsed_time(b) for a, b in mas_events) / max(len(mas_events), 1)
    cells = B * Tx * Ty
    mas_gbs = 12.0 * cells / (mas_ms * 1e-3) / 1e9
    step_ms = elapsed / args.steps * 1e3
    flops = decoder_train_flops(B, Ty)
    # roofline.traffic: PMC-measured HBM bytes per conv_gemm launch on THIS workload (tools/pmc_traffic.sh
    # -> profiles/<round>/conv_gemm_traffic.json); PMC passes serialize kernels, so not collected here
    traffic, traffic_src = None, None
    if (B, Tx, Ty, args.precision) == (32, 120, 600, "bf16-mixed"):
        found = sorted(ROOT.glob("profiles/r*/conv_gemm_traffic.json"))
        if found:
            traffic = json.loads(found[-1].read_text())["traffic_bytes_per_launch"]
            traffic_src = str(found[-1].relative_to(ROOT))
    gemm_peak = FP32_MFMA_TFLOPS if args.precision == "32-true" else BF16_DENSE_TFLOPS

    # roofline model of the dominant kernel: attainable = min(MFMA peak, AI x HBM peak).  At this
    # workload's arithmetic intensity (algorithmic FLOPs / algorithmic bytes) the GEMMs sit below the
    # ridge point (peak / 8 TB/s), so the binding roof is HBM; the MFMA fraction is reported beside it
    gemm_time_s = sum(gemm_ms) * 1e-3
    ai = gemm_flops / max(gemm_bytes, 1)
    ridge = gemm_peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    gemm_gbs = gemm_bytes / gemm_time_s / 1e9 if gemm_ms else 0.0
    common = {"kernel": "conv_gemm_kernel (decoder + encoder implicit-GEMM conv/linear, fwd + dgrad)",
              "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC, FETCH_SIZE x2 + WRITE_SIZE)",
              "traffic_source": traffic_src,
              "algorithmic_bytes_per_launch": round(gemm_bytes / max(len(gemm_log), 1)),
              "algorithmic_flops_per_launch": round(gemm_flops / max(len(gemm_log), 1)),
              "arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(ridge, 1),
              "launches_per_step": len(gemm_log), "avg_launch_us": round(gemm_avg_us, 2),
              "algorithmic_flops_per_step": gemm_flops,
              "mfma_tflops": round(gemm_tflops, 1), "mfma_frac": round(gemm_tflops / gemm_peak, 4),
              "note": "achieved over sum of launch durations (HIP events on the launch stream, one eager "
                      "fwd+bwd of the bench batch); bytes = A read once + W + C written (+ aux/residual/"
                      "pre-activation streams) per launch"}
    if ai < ridge:
        gemm_roofline = {"bound": "hbm", "achieved": round(gemm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gemm_gbs / HBM_PEAK_GBS, 4), **common}
    else:
        gemm_roofline = {"bound": "mfma", "achieved": round(gemm_tflops, 1), "peak": gemm_peak,
                         "unit": "TFLOP/s", "frac": round(gemm_tflops / gemm_peak, 4), **common}

    def roofline_of(log, kernel, note):
        """Roofline line of a launch log: bound from the arithmetic intensity vs the ridge point."""
        if not log:
            return None
        ms = [r[0].elapsed_time(r[1]) for r in log]
        t = sum(ms) * 1e-3
        fl, by = sum(r[2] for r in log), sum(r[4] for r in log)
        tf, gb = fl / t / 1e12, by / t / 1e9
        ai = fl / max(by, 1)
        line = {"kernel": kernel, "launches_per_step": len(log), "avg_launch_us": round(sum(ms) / len(ms) * 1e3, 2),
                "algorithmic_flops_per_launch": round(fl / len(log)), "algorithmic_bytes_per_launch": round(by / len(log)),
                "arithmetic_intensity_flop_per_byte": round(ai, 1), "ridge_flop_per_byte": round(ridge, 1),
                "mfma_tflops": round(tf, 1), "hbm_gbs": round(gb, 1), "traffic": None, "note": note}
        if ai < ridge:
            return {"bound": "hbm", "achieved": round(gb, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gb / HBM_PEAK_GBS, 4), **line}
        return {"bound": "mfma", "achieved": round(tf, 1), "peak": gemm_peak, "unit": "TFLOP/s",
                "frac": round(tf / gemm_peak, 4), **line}

    roofline_wgrad = roofline_of(
        wgrad_log, "conv_wgrad_kernel + wgrad slab reduce (weight-gradient GEMMs, decoder + encoder)",
        "HIP events around each mtts_conv_wgrad call (one eager fwd+bwd of the bench batch); 2*M*N*K FLOP; "
        "bytes = dY + unique A rows + dW; each call includes its fp32 partial-slab reduce (this eager pass does "
        "not defer the sums)")
    roofline_attn = roofline_of(
        attn_log, "attn_fwd_kernel / attn_bwd_dq_kernel + attn_bwd_dkv_kernel (decoder + encoder attention)",
        "HIP events around each mtts_attention_fwd / _bwd call; FLOP = 4 B H T^2 D fwd, 8 B H T^2 D bwd "
        "(standard flash-attention accounting, recomputation not counted)")

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
            "roofline_mas": {"kernel": "mas_dp_kernel + mas_expand_kernel (maximum_path)", "bound": "hbm",
                             "achieved": round(mas_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(mas_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                             "algorithmic_bytes_per_launch": 12 * cells,
                             "chain_bound": mas_chain_bound(Tx, Ty, mas_ms),
                             "note": "12 B/cell (value+mask read, path write); chain-bound: one wave per utterance"},
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
                "overlapped_in_graph": bool(next(iter(trainer._graphs.values()))["overlap"]) if trainer._graphs else None},
            "precision_check": precision_check,
            "synthesise": synth,
        }
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(B, Tx, Ty, args.cpu_budget)
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
