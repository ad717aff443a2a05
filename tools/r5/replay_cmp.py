"""Per-shape table of two replay runs (tools/r5/gemm_replay.py --out): the heuristic (-1) of each and every
other schedule of the second, with the per-step totals.  python tools/r5/replay_cmp.py OLD.jsonl NEW.jsonl"""
import json
import sys


def load(p):
    out = {}
    for l in open(p):
        r = json.loads(l)
        if "res" in r:
            out[(r["M"], r["N"], r["K"], r["flags"], r["act"], r["ntaps"])] = r
    return out


old, new = load(sys.argv[1]), load(sys.argv[2])
tot = {}
for k, r in new.items():
    o = old.get(k, {}).get("res", {}).get("-1", {}).get("us")
    row = [f"{o}"]
    for c, v in r["res"].items():
        us = v.get("us")
        row.append(f"{c}:{us}{'' if v.get('bitwise', True) else '(!)'}")
        tot[c] = tot.get(c, 0) + (us if us is not None else r["res"]["-1"]["us"]) * r["count"]
    tot["old"] = tot.get("old", 0) + (o or 0) * r["count"]
    tot["best"] = tot.get("best", 0) + min(v["us"] for v in r["res"].values() if "us" in v) * r["count"]
    print(k, r["count"], " ".join(row))
print({c: round(v, 1) for c, v in tot.items()})
