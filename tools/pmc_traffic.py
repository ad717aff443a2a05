"""One eager bf16 fwd+bwd of the bench batch (B=32, 120x600): the conv_gemm launches whose HBM traffic
tools/pmc_traffic.sh measures with rocprofv3 PMC passes.  Writes the launches' algorithmic bytes and
FLOPs (the LAUNCH_LOG hook) to the JSON path given as argv[1]."""
import json, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import torch
from matcha.models.matcha_tts import MatchaTTS
from matcha.models.components import _ops as O
from matcha.training import TrainConfig, Trainer, synthetic_batch

dev = torch.device("cuda")
torch.manual_seed(1234)
m = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).train()
tr = Trainer(m, TrainConfig(precision="bf16-mixed", graph=False))
b = synthetic_batch(32, 120, 600, seed=1000, device=dev)
tr._fwd_bwd([b])  # warm-up (same launches)
torch.cuda.synchronize()
O.LAUNCH_LOG = []
tr._fwd_bwd([b])
torch.cuda.synchronize()
log, O.LAUNCH_LOG = O.LAUNCH_LOG, None
out = {"launches_per_pass": len(log), "algorithmic_bytes_per_pass": sum(x[4] for x in log),
       "algorithmic_flops_per_pass": sum(x[2] for x in log), "passes": 2}
Path(sys.argv[1]).write_text(json.dumps(out))
print(json.dumps(out))
