"""Per-wave phase timeline of one register-staged GEMM launch (diagnostic build: MTTS_GEMM_TIMELINE=1,
lib/libmtts_hip_tl.so; see the g_tl comment in csrc/conv_gemm.hip).

python tools/r5/gemm_timeline.py --match M,N,K,flags,act [--cfg 3] [--out OUT.json]

Replays the bench step's launch of that shape (tools/r5/gemm_replay.py's synthetic operands), then reads the
100 MHz wall-clock stamps each wave's lane 0 wrote: kernel start, prologue done, per K step (loads issued, MFMAs
issued, LDS stored, barrier passed), loop end, epilogue end.  Prints where the waves' time goes and how many waves
each SIMD held over the launch."""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent
os.environ.setdefault("MTTS_LIB", str(ROOT / "matcha-tts-etu-upmc-ensam_amd" / "lib" / "libmtts_hip_tl.so"))
sys.path[:0] = [str(ROOT / "tools" / "r5")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gemm_replay as G  # noqa: E402
from matcha import _native as N  # noqa: E402

SLOTS, WAVES, STEPS = 128, 16384, 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", default=str(ROOT / "profiles" / "r05" / "gemm_log_parity.jsonl"))
    ap.add_argument("--match", required=True)
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    want = [int(x) for x in args.match.split(",")]
    r = next(json.loads(l) for l in open(args.log) if l.startswith("{") and
             [json.loads(l)[k] for k in ("M", "N", "K", "flags", "act")] == want)
    fn = N.lib().mtts_gemm_timeline_read
    fn.restype, fn.argtypes = ctypes.c_longlong, [ctypes.c_void_p]
    A, Wp, C, kw = G.make_case(r)
    for _ in range(5):
        G.run(r, A, Wp, C, kw, args.cfg)
    torch.cuda.synchronize()
    assert fn(None) > 0
    torch.cuda.synchronize()
    G.run(r, A, Wp, C, kw, args.cfg)
    torch.cuda.synchronize()
    buf = np.zeros(WAVES * SLOTS, dtype=np.int64)
    assert fn(buf.ctypes.data) == buf.nbytes
    t = buf.reshape(WAVES, SLOTS)
    live = t[:, 1] > 0
    t = t[live]
    nw = len(t)
    hw = t[:, 0] & 0xFFFFFFFF
    smid = t[:, 0] >> 32
    simd = (hw >> 4) & 3
    t0 = t[:, 1].min()
    tick_us = 0.01  # 100 MHz
    start, pro, lend, epi = t[:, 1], t[:, 2], t[:, SLOTS - 2], t[:, SLOTS - 1]
    nk = 0
    while nk < STEPS and (t[:, 3 + 4 * nk] > 0).all():
        nk += 1
    ph = {"load": [], "mfma": [], "store": [], "barrier": []}
    prev = pro
    for k in range(nk):
        l_, c_, s_, b_ = (t[:, 3 + 4 * k + i] for i in range(4))
        ph["load"].append(l_ - prev)
        ph["mfma"].append(c_ - l_)
        ph["store"].append(s_ - c_)
        ph["barrier"].append(b_ - s_)
        prev = b_
    res = {
        "shape": args.match, "cfg": args.cfg, "waves": int(nw), "steps_recorded": nk,
        "kernel_us": float((epi.max() - t0) * tick_us),
        "wave_life_us_mean": float(((epi - start) * tick_us).mean()),
        "start_spread_us": float((start.max() - t0) * tick_us),
        "prologue_us_mean": float(((pro - start) * tick_us).mean()),
        "loop_us_mean": float(((lend - pro) * tick_us).mean()),
        "epilogue_us_mean": float(((epi - lend) * tick_us).mean()),
        "per_step_us_mean": {k: float(np.mean(v) * tick_us) for k, v in ph.items()},
        "per_step_us_p90": {k: float(np.percentile(np.stack(v), 90) * tick_us) for k, v in ph.items()},
        "cus": int(len(np.unique(smid))),
    }
    # waves resident per SIMD over time (sampled every 0.5 us)
    key = smid * 4 + simd
    ts = np.arange(t0, epi.max(), 50)
    occ = []
    for x in ts:
        alive = (start <= x) & (epi > x)
        if alive.any():
            _, cnt = np.unique(key[alive], return_counts=True)
            occ.append((float((x - t0) * tick_us), float(cnt.mean()), int(alive.sum())))
    res["simd_occupancy"] = occ[:: max(1, len(occ) // 20)]
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
