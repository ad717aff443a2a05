"""Workload of tools/r3/pmc_families.sh: one warm-up and two logged eager bf16 fwd+bwd passes of the bench
batch (B=32, 120x600, the bench's model init).  Writes the launches' algorithmic bytes / FLOPs per family
(the _ops launch logs: GEMM, weight gradient, attention) to the JSON path in argv[1]."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import os  # noqa: E402

import torch  # noqa: E402

from matcha.models.components import _ops as O  # noqa: E402
from matcha.models.matcha_tts import MatchaTTS  # noqa: E402
from matcha.training import TrainConfig, Trainer, synthetic_batch  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(1234)
m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
# PMC_PREC=bf16-parity (round 4): the bench default's precision (bench.py reads *_traffic_parity.json for it)
tr = Trainer(m, TrainConfig(precision=os.environ.get("PMC_PREC", "bf16-mixed"), graph=False))
b = synthetic_batch(32, 120, 600, seed=1000, device=dev)
tr._fwd_bwd([b])
m.zero_grad(set_to_none=True)
torch.cuda.synchronize()
logs = {"gemm": [], "wgrad": [], "attn": []}
for _ in range(2):
    O.LAUNCH_LOG, O.WGRAD_LOG, O.ATTN_LOG = [], [], []
    tr._fwd_bwd([b])
    m.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    logs["gemm"] += O.LAUNCH_LOG
    logs["wgrad"] += O.WGRAD_LOG
    logs["attn"] += O.ATTN_LOG
O.LAUNCH_LOG = O.WGRAD_LOG = O.ATTN_LOG = None
out = {f: {"launches": len(v), "algorithmic_bytes": sum(x[4] for x in v), "algorithmic_flops": sum(x[2] for x in v)}
       for f, v in logs.items()}
out["passes"] = 2
out["precision"] = os.environ.get("PMC_PREC", "bf16-mixed")
out["warmup_passes"] = 1  # profiled too: pmc_families_summary.py drops its dispatches
Path(sys.argv[1]).write_text(json.dumps(out))
print(json.dumps(out))
