#!/usr/bin/env python
"""Which weights' bf16 rounding moves the losses: first order, rounding W to bf16 changes a loss L by
dL = sum(dW * dL/dW), with dW a rounding error of about |W| * 2^-9 / sqrt(3) rms (uniform relative error),
so Var(dL) per weight tensor ~ (2^-9)^2 / 3 * sum((W * G)^2).  Computed in fp32 (32-true) on the parity
tests' recipe weights and the bench batch, for the prior and the diff loss separately; prints the tensors
ranked by their share of the variance (cumulative), as JSON lines."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tests")]

import torch  # noqa: E402

from golden.weights_recipe import apply_recipe  # noqa: E402
from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import synthetic_batch  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev)
    apply_recipe(model, 43)
    model.eval()
    b = {k: v.to(dev) for k, v in synthetic_batch(32, 120, 600, seed=1000, device="cpu").items()}
    gen = torch.Generator().manual_seed(44)
    t = torch.rand(32, 1, 1, generator=gen).to(dev)
    z = torch.randn(32, 80, 600, generator=gen).to(dev)
    gemm_w = {n: p for n, p in model.named_parameters() if p.dim() >= 2 and "embedding" not in n}
    for li, lname in ((1, "prior"), (2, "diff")):
        model.zero_grad(set_to_none=True)
        out = model(b["x"], b["x_lengths"], b["y"], b["y_lengths"], t=t, z=z)
        loss = out[li]
        loss.backward()
        var = {n: float(((p.detach() * p.grad) ** 2).sum()) * (2 ** -9) ** 2 / 3 for n, p in gemm_w.items()
               if p.grad is not None}
        tot = sum(var.values())
        cum = 0.0
        rows = []
        for n, v in sorted(var.items(), key=lambda kv: -kv[1]):
            cum += v
            rows.append({"param": n, "share": round(v / tot, 4), "cum": round(cum / tot, 4)})
        print(json.dumps({"loss": lname, "value": float(loss), "pred_rel_err_rms": (tot ** 0.5) / float(loss),
                          "n_tensors": len(rows), "ranked": rows[:40]}), flush=True)


if __name__ == "__main__":
    main()
