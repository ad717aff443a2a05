"""Workload of tools/r5/pmc_mas.sh: maximum_path(value, mask) on the bench batch's own fp32 lattice (B=32,
120x600, the bench's model init and precision, as bench.py times it): one warm-up and two logged calls.
Writes the calls' algorithmic bytes (12 B per padded cell: value + mask read, path written) to argv[1]."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import torch  # noqa: E402

import matcha.utils.monotonic_align as MA  # noqa: E402
from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import synthetic_batch  # noqa: E402
from matcha.utils.model import sequence_mask  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(1234)
m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
B, Tx, Ty = 32, 120, 600
b = synthetic_batch(B, Tx, Ty, seed=1000, device=dev)
with torch.no_grad():
    mu_x, _, x_mask = m.encoder(b["x"], b["x_lengths"])
    lp = m.log_prior(mu_x, b["y"])
    y_mask = sequence_mask(b["y_lengths"], Ty).unsqueeze(1).float()
    am = (x_mask.unsqueeze(-1) * y_mask.unsqueeze(2)).squeeze(1).contiguous()
    torch.cuda.synchronize()
    for _ in range(3):  # warm-up + two logged calls
        MA.maximum_path(lp, am)
    torch.cuda.synchronize()
out = {"mas": {"launches": 2, "algorithmic_bytes": 2 * 12.0 * B * Tx * Ty, "algorithmic_flops": 0},
       "passes": 2, "warmup_passes": 1, "precision": os.environ.get("PMC_PREC", "bf16-parity")}
Path(sys.argv[1]).write_text(json.dumps(out))
print(json.dumps(out))
