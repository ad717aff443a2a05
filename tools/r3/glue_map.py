#!/usr/bin/env python
"""Which Python op launches each non-HIP (torch / library) kernel of the train step: one eager fwd+bwd of
the bench batch (the graph step replays the same launches) under torch.profiler, kernels grouped by the
launching aten op and the Python frames above it.  Writes gpurun_out/<tag>/glue_map.txt."""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import TrainConfig, Trainer, synthetic_batch  # noqa: E402

OURS = ("conv_", "attn_", "layernorm", "gn_mish", "mas_", "log_prior", "pack_", "rope_", "dropout_apply",
        "act_dropout", "splitk", "reduce_partials", "embedding_", "loss_", "adamw", "cfm_", "time_emb",
        "expand_rows", "colsum", "mel_")


def main():
    out = Path(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "glue_map.txt")
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
    tr = Trainer(model, TrainConfig(precision="bf16-mixed", graph=False))
    b = synthetic_batch(32, 120, 600, seed=1000, device=dev)
    for _ in range(2):
        tr._fwd_bwd([b])
        model.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr._fwd_bwd([b])
        torch.cuda.synchronize()
    lines, glue, n_all = [], [], 0
    for e in prof.events():
        for k in getattr(e, "kernels", []) or []:
            n_all += 1
            if not any(t in k.name for t in ("at::native", "Cijk", "CatArray", "rocclr", "Memset", "Memcpy")):
                continue  # one of ours (csrc/*.hip)
            chain, parent = [e.name], e.cpu_parent
            while parent is not None and len(chain) < 4:
                chain.append(parent.name)
                parent = parent.cpu_parent
            stack = [s_ for s_ in (e.stack or []) if "matcha" in s_][:3]
            glue.append((k.duration, k.name, chain, stack))
    lines.append(f"kernels {n_all}, non-HIP {len(glue)}: {sum(g[0] for g in glue):.1f} us (eager, profiled)")
    for dur, name, chain, stack in glue:
        lines.append(f"{dur:8.1f} us  {name[:60]:60s} <- {' < '.join(chain)} | {' ; '.join(stack)}")
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text("\n".join(lines) + "\n")
    print("\n".join(lines[:80]))


if __name__ == "__main__":
    main()
