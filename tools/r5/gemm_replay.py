"""Replays the bench step's GEMM launches (bench.py with MTTS_DUMP_GEMM_LOG=path) on synthetic operands of the
same shapes, flags and epilogues: graph-timed per schedule (20 back-to-back launches per graph, the kernel
boundary included), each candidate's output compared with the FIRST schedule's (max abs difference relative to
its max |value|, and bitwise).

python tools/r5/gemm_replay.py LOG.jsonl [--cfgs -1,64,65] [--top N] [--out OUT.jsonl]"""
import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT / "tools")]
from matcha.models.components import _ops as O  # noqa: E402

dev = torch.device("cuda")


def t_ev(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3


KEYS = ("M", "N", "K", "cin", "ntaps", "in_stride", "out_stride", "out_off", "prec", "flags", "act", "pre", "res", "drop",
        "asc", "cs", "bias", "aux", "nb", "Ti", "To", "To_full", "lda", "ldc", "ldr", "Kp", "offs")


def make_case(r, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed + r["M"] + 7 * r["N"] + r["K"])
    F = r["flags"]
    a16, c16, ws, pre16 = bool(F & 2), bool(F & 4), bool(F & 0x40), bool(F & 0x10)
    nb, Ti, To, To_full = r["nb"], r["Ti"], r["To"], r["To_full"]
    N, Kp = r["N"], r["Kp"]
    A = torch.randn(nb, Ti, r["lda"], generator=g).to(dev)
    A = A.bfloat16() if a16 else A
    wdt = torch.bfloat16 if r["prec"] == 1 else torch.float32
    w = (torch.randn(N, Kp, generator=g) / (r["K"] ** 0.5)).to(dev)
    if ws:
        hi = w.bfloat16()
        Wp = torch.cat([hi, (w - hi.float()).bfloat16()]).contiguous()
    else:
        Wp = w.to(wdt).contiguous()
    if ws:
        Wp._mtts_w_split = True
    kw = {}
    if r["asc"]:
        lens = torch.randint(Ti // 2, Ti + 1, (nb,), generator=g)
        kw["a_scale"] = (torch.arange(Ti)[None] < lens[:, None]).float().to(dev)
    if r["bias"]:
        kw["bias"] = torch.randn(N, generator=g).to(dev)
    if r["res"]:
        ldr = r["ldr"] or N
        kw["residual"] = torch.randn(nb, To_full, ldr, generator=g).to(dev)[..., :N] if ldr != N else \
            torch.randn(nb, To_full, N, generator=g).to(dev)
    if r["cs"]:
        kw["c_scale"] = (torch.rand(nb, To_full, generator=g) > 0.2).float().to(dev)
    if r["pre"]:
        kw["C_pre"] = torch.empty(nb, To_full, r["ldc"], device=dev, dtype=torch.bfloat16 if pre16 else torch.float32)
    if r["aux"]:
        kw["aux"] = torch.randn(nb, To_full, r["ldc"], generator=g).to(dev)
        kw["aux"] = kw["aux"].bfloat16() if pre16 else kw["aux"]
    if r["drop"]:
        kw["dropout_p"] = 0.1
        kw["seed"] = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
    kw["act"] = r["act"]
    C = torch.zeros(nb, To_full, r["ldc"], device=dev, dtype=torch.bfloat16 if c16 else torch.float32)
    return A, Wp, C, kw


def run(r, A, Wp, C, kw, cfg):
    O._gemm(A, r["Ti"], r["To"], r["nb"], r["in_stride"], r["offs"], r["cin"], Wp, r["Kp"], r["N"], C, r["To_full"],
            r["out_stride"], r["out_off"], prec=r["prec"], tile_cfg=cfg, **kw)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--cfgs", default="-1,64,65,66,67,68,69")
    ap.add_argument("--top", type=int, default=1000)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only-bf16", action="store_true")
    ap.add_argument("--only-fp32", action="store_true")
    ap.add_argument("--match", default=None, help="M,N,K,flags,act: replay only this launch shape")
    ap.add_argument("--plain", type=int, default=0, help="with --match: N plain (ungraphed) launches per schedule "
                    "instead of the timing, for rocprofv3 counter passes")
    args = ap.parse_args()
    rows = [json.loads(l) for l in open(args.log) if l.startswith("{")]
    uniq = {}
    for r in rows:
        k = tuple(json.dumps(r.get(x)) for x in KEYS)
        e = uniq.setdefault(k, dict(r, count=0, us_sum=0.0))
        e["count"] += 1
        e["us_sum"] += r["us"]
    cases = sorted(uniq.values(), key=lambda e: -e["us_sum"])[: args.top]
    cfgs = [int(c) for c in args.cfgs.split(",")]
    out = open(args.out, "w") if args.out else None
    tot = {c: 0.0 for c in cfgs}
    for r in cases:
        if (args.only_bf16 and r["prec"] != 1) or (args.only_fp32 and r["prec"] != 0):
            continue
        if args.match and [int(x) for x in args.match.split(",")] != [r[k] for k in ("M", "N", "K", "flags", "act")]:
            continue
        if args.match and args.plain:
            A, Wp, C, kw = make_case(r)
            for cfg in cfgs:
                for _ in range(args.plain):
                    run(r, A, Wp, C, kw, cfg)
                torch.cuda.synchronize()
            print(json.dumps(dict(match=args.match, cfgs=cfgs, launches=args.plain)), flush=True)
            break
        A, Wp, C, kw = make_case(r)
        res = {}
        ref = None
        for cfg in cfgs:
            C.zero_()
            try:
                run(r, A, Wp, C, kw, cfg)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                res[cfg] = dict(err=str(e)[:80])
                continue
            outc = C.float().clone()
            if ref is None:
                ref = outc
            d = (outc - ref).abs().max().item()
            scale = ref.abs().max().item() + 1e-30
            us = t_ev(lambda: run(r, A, Wp, C, kw, cfg))
            res[cfg] = dict(us=round(us, 2), rel=d / scale, bitwise=bool(torch.equal(outc, ref)))
        best = min((v["us"] for v in res.values() if "us" in v), default=None)
        for c in cfgs:
            v = res.get(c, {})
            tot[c] += v["us"] * r["count"] if "us" in v else (res.get(-1, {}).get("us", 0) * r["count"])
        line = dict({k: r[k] for k in ("M", "N", "K", "ntaps", "flags", "act", "prec", "count")}, res=res, best=best)
        print(json.dumps(line), flush=True)
        if out:
            out.write(json.dumps(line) + "\n")
    print(json.dumps({"total_us_per_step_by_cfg (missing = cfg -1)": {c: round(v, 1) for c, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
