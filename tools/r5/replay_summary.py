"""Summarises a gemm_replay.py log: one line per shape, time per schedule (!BAD where the output differs)."""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "res" not in d:
        print(line.strip())
        continue
    r = d["res"]
    ok = {c: v for c, v in r.items() if "us" in v}
    best = min(ok, key=lambda c: ok[c]["us"]) if ok else None
    cells = []
    for c, v in r.items():
        if "us" not in v:
            cells.append(f"{c}:-")
            continue
        bad = "" if v["rel"] < 2e-2 else "!BAD%.2g" % v["rel"]
        cells.append(f"{c}:{v['us']:.1f}{bad}{'*' if c == best else ''}")
    print(d["M"], d["N"], d["K"], d["ntaps"], hex(d["flags"]), d["act"], "x%d" % d["count"], "|", " ".join(cells))
