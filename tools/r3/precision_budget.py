#!/usr/bin/env python
"""bf16-mixed error budget of the train-step losses (VERDICT r2 "what's next" #2).

For each storage configuration (environment switches read at import, so each runs in its own process)
the product's bf16-mixed forward on the recipe weights is compared with its 32-true forward (which equals
the CPU oracle bit for bit at these batches: tests/test_headline_gpu.py).  Four bf16 runs separate the
error sources:
  full        bf16-mixed as the bench runs it
  align32     the same, with the fp32 run's alignment (MAS result) forced: no MAS boundary flips
  enc32       the fp32 run's encoder outputs (mu_x, logw) forced: decoder-only error (alignment then equal)
  dec32       bf16 encoder, fp32 alignment, fp32 decoder: encoder-only error on prior / duration
Prints one JSON line per (configuration, batch).

    python tools/r3/precision_budget.py [config ...]      (default: every configuration)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CONFIGS = {
    "default": {},
    "split": {"MTTS_W_SPLIT": "1"},
    "split_encfp32": {"MTTS_W_SPLIT": "1", "MTTS_BUDGET_ENC_FP32": "1"},
    "preln_fp32": {"MTTS_PRELN_N16": "0"},
    "attn_io_fp32": {"MTTS_ATTN_IO16": "0"},
    "ffn_fp32": {"MTTS_FF_FP32_HIDDEN": "1", "MTTS_FF_FP32_PRE": "1"},
    "resnet_fp32": {"MTTS_RESNET_BF16_STORE": "0"},
    "all_storage_fp32": {"MTTS_PRELN_N16": "0", "MTTS_ATTN_IO16": "0", "MTTS_FF_FP32_HIDDEN": "1",
                         "MTTS_FF_FP32_PRE": "1", "MTTS_RESNET_BF16_STORE": "0"},
}
CASES = [(32, 120, 600, 1000), (8, 512, 4096, 7)]


def child(name: str) -> None:
    sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tests")]
    import torch

    import matcha.utils.monotonic_align as MA
    from golden.weights_recipe import apply_recipe
    from matcha.models.matcha_tts import MatchaTTS
    from matcha.training import synthetic_batch

    dev = torch.device("cuda:0")
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev)
    model.encoder_fp32 = os.environ.get("MTTS_BUDGET_ENC_FP32") == "1"
    apply_recipe(model, 43)
    model.eval()
    real_pmp, real_enc = MA.prior_maximum_path, model.encoder.forward
    for B, Tx, Ty, seed in CASES:
        b = synthetic_batch(B, Tx, Ty, seed=seed, device="cpu")
        gen = torch.Generator().manual_seed(44)
        t = torch.rand(B, 1, 1, generator=gen).to(dev)
        z = torch.randn(B, 80, Ty, generator=gen).to(dev)
        b = {k: v.to(dev) for k, v in b.items()}
        saved = {}

        def rec_pmp(*a, **k):
            saved["align"] = real_pmp(*a, **k)
            return saved["align"]

        def rec_enc(*a, **k):
            saved["enc"] = real_enc(*a, **k)
            return saved["enc"]

        def run(bf16: bool):
            with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                dur, prior, diff, attn = model(b["x"], b["x_lengths"], b["y"], b["y_lengths"], t=t, z=z)
            return [float(dur), float(prior), float(diff)], attn

        MA.prior_maximum_path, model.encoder.forward = rec_pmp, rec_enc
        l32, a32 = run(False)
        MA.prior_maximum_path, model.encoder.forward = real_pmp, real_enc
        out = {"config": name, "batch": [B, Tx, Ty], "losses_fp32": l32}

        def rel(l16):
            return [abs(x - y) / abs(y) for x, y in zip(l16, l32)]

        l16, a16 = run(True)
        out["full"] = rel(l16)
        out["full_cells_differing"] = int((a16 != a32).sum())
        MA.prior_maximum_path = lambda *a, **k: saved["align"]  # noqa: E731
        out["align32"] = rel(run(True)[0])
        MA.prior_maximum_path = real_pmp
        model.encoder.forward = lambda *a, **k: saved["enc"]  # noqa: E731
        out["enc32"] = rel(run(True)[0])
        model.encoder.forward = real_enc
        # bf16 encoder only: the decoder forced to fp32 by running its loss outside autocast
        dec = model.decoder.compute_loss_and_prior

        def dec_fp32(*a, **k):
            with torch.autocast("cuda", enabled=False):
                return dec(*[v.float() if torch.is_tensor(v) and v.is_floating_point() else v for v in a], **k)

        model.decoder.compute_loss_and_prior = dec_fp32
        MA.prior_maximum_path = lambda *a, **k: saved["align"]  # noqa: E731
        out["dec32"] = rel(run(True)[0])
        MA.prior_maximum_path = real_pmp
        del model.decoder.compute_loss_and_prior
        # weight rounding vs activation rounding: the GEMM weights (conv / linear, not the embedding lookup)
        # rounded to bf16 in both runs
        if name == "default":
            saved_w = {}
            with torch.no_grad():
                for n_, p_ in model.named_parameters():
                    if p_.dim() >= 2 and "embedding" not in n_:
                        saved_w[n_] = p_.detach().clone()
                        p_.copy_(p_.bfloat16().float())
            lr32, _ = run(False)
            lr16, _ = run(True)
            with torch.no_grad():
                for n_, p_ in model.named_parameters():
                    if n_ in saved_w:
                        p_.copy_(saved_w[n_])
            out["wround_fp32_vs_fp32"] = rel(lr32)  # the effect of rounding the weights alone
            out["wround_bf16_vs_wround_fp32"] = [abs(x - y) / abs(y) for x, y in zip(lr16, lr32)]  # activations alone
        print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    names = sys.argv[1:] or list(CONFIGS)
    rc = 0
    for name in names:
        env = dict(os.environ, **CONFIGS[name])
        r = subprocess.run([sys.executable, __file__, "--child", name], env=env, timeout=600)
        rc = rc or r.returncode
    sys.exit(rc)


if __name__ == "__main__":
    main()
