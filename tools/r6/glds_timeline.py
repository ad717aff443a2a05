"""Per-wave phase timeline of one LDS-DMA GEMM launch (conv_gemm_glds_kernel; diagnostic build
MTTS_GEMM_TIMELINE=1 -> lib/libmtts_hip_tl.so, see g_tlg in csrc/conv_gemm_glds.hip).

python tools/r6/glds_timeline.py --match M,N,K,ntaps,flags [--cfg -1] [--out OUT.json]

Replays the bench step's launch of that shape (tools/r5/gemm_replay.py's synthetic operands) and reads the 100 MHz
stamps each wave's lane 0 wrote: start, prologue issued, per K step (DMAs landed + barrier passed, MFMAs issued),
loop end, epilogue end.  Prints where the waves' time goes and the tile count per CU."""
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

SLOTS, WAVES, STEPS = 128, 16384, 60


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log", default=str(ROOT / "profiles" / "r05" / "gemm_log_parity.jsonl"))
    ap.add_argument("--match", required=True)
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    want = [int(x) for x in args.match.split(",")]
    r = next(json.loads(l) for l in open(args.log) if l.startswith("{") and
             [json.loads(l)[k] for k in ("M", "N", "K", "ntaps", "flags")] == want)
    fn = N.lib().mtts_glds_timeline_read
    fn.restype, fn.argtypes = ctypes.c_longlong, [ctypes.c_void_p]
    A, Wp, C, kw = G.make_case(r)
    for _ in range(5):
        G.run(r, A, Wp, C, kw, args.cfg)
    torch.cuda.synchronize()
    assert fn(None) > 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    G.run(r, A, Wp, C, kw, args.cfg)
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(WAVES * SLOTS, dtype=np.int64)
    assert fn(buf.ctypes.data) == buf.nbytes
    t = buf.reshape(WAVES, SLOTS)
    t = t[t[:, 1] > 0]
    nw = len(t)
    smid = t[:, 0] >> 32
    hw = t[:, 0] & 0xFFFFFFFF
    simd = (hw >> 4) & 3
    t0 = t[:, 1].min()
    tick = 0.01  # us per 100 MHz tick
    start, pro, lend, epi = t[:, 1], t[:, 2], t[:, SLOTS - 2], t[:, SLOTS - 1]
    nk = 0
    while nk < STEPS and (t[:, 3 + 2 * nk] > 0).all():
        nk += 1
    wait, comp = [], []
    prev = pro
    for k in range(nk):
        b_, c_ = t[:, 3 + 2 * k], t[:, 4 + 2 * k]
        wait.append(b_ - prev)
        comp.append(c_ - b_)
        prev = c_
    wait, comp = np.stack(wait) * tick, np.stack(comp) * tick
    _, per_cu = np.unique(smid, return_counts=True)
    res = {
        "shape": args.match, "cfg": args.cfg, "waves": int(nw), "steps_recorded": nk,
        "event_us": e0.elapsed_time(e1) * 1e3,
        "kernel_us": float((epi.max() - t0) * tick),
        "wave_life_us_mean": float(((epi - start) * tick).mean()),
        "start_spread_us": float((start.max() - t0) * tick),
        "start_quantiles_us": [float(np.percentile((start - t0) * tick, q)) for q in (10, 50, 90, 100)],
        "prologue_issue_us_mean": float(((pro - start) * tick).mean()),
        "first_wait_us_mean": float(wait[0].mean()) if nk else None,
        "loop_us_mean": float(((lend - pro) * tick).mean()),
        "epilogue_us_mean": float(((epi - lend) * tick).mean()),
        "per_step_wait_us_mean": float(wait[1:].mean()) if nk > 1 else None,
        "per_step_compute_us_mean": float(comp.mean()) if nk else None,
        "per_step_wait_us_by_k": [round(float(x), 3) for x in wait.mean(axis=1)],
        "cus": int(len(per_cu)), "waves_per_cu_max": int(per_cu.max()), "waves_per_cu_min": int(per_cu.min()),
    }
    key = smid * 4 + simd
    ts = np.arange(t0, epi.max(), 50)
    occ = []
    for x in ts:
        alive = (start <= x) & (epi > x)
        if alive.any():
            _, cnt = np.unique(key[alive], return_counts=True)
            occ.append((round(float((x - t0) * tick), 2), round(float(cnt.mean()), 2), int(alive.sum())))
    res["simd_occupancy"] = occ[:: max(1, len(occ) // 16)]
    print(json.dumps(res, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
