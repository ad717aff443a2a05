"""Per-utterance MAS diagnosis vs the oracle: dp lattice match, first diverging column."""
import sys
from pathlib import Path
import numpy as np, torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT), str(ROOT / "tests")]
import oracle_bind as O
from matcha.utils.monotonic_align import maximum_path_c
for (B, Tx, Ty) in [(3, 20, 50), (3, 64, 200), (3, 65, 200), (3, 120, 600), (2, 120, 120), (2, 200, 400)]:
    rng = np.random.default_rng(Tx + Ty)
    value = rng.normal(-100, 10, size=(B, Tx, Ty)).astype(np.float32)
    t_x = np.array([Tx] + [max(1, Tx - 5 * b) for b in range(1, B)], np.int32)
    t_y = np.array([Ty] + [max(int(t_x[b]), Ty - 7 * b) for b in range(1, B)], np.int32)
    ep, edp = O.mas_batch(value, t_x, t_y)
    v = torch.from_numpy(value).cuda(); p = torch.zeros(value.shape, dtype=torch.int32, device="cuda")
    maximum_path_c(p, v, torch.from_numpy(t_x).cuda(), torch.from_numpy(t_y).cuda())
    gp, gdp = p.cpu().numpy(), v.cpu().numpy()
    for b in range(B):
        dpok = np.array_equal(gdp[b].view(np.uint32), edp[b].view(np.uint32))
        pok = np.array_equal(gp[b], ep[b])
        msg = f"B{B} {Tx}x{Ty} b={b} tx={t_x[b]} ty={t_y[b]} dp_ok={dpok} path_ok={pok}"
        if not dpok:
            bad = np.argwhere(gdp[b].view(np.uint32) != edp[b].view(np.uint32))
            msg += f" first_dp_bad(x,y)={bad[np.lexsort((bad[:,0], bad[:,1]))][0].tolist()} n={len(bad)}"
        if not pok:
            gi = gp[b, :, :t_y[b]].argmax(0); ei = ep[b, :, :t_y[b]].argmax(0)
            d = np.nonzero(gi != ei)[0]
            msg += f" path_cols_bad={len(d)} last_bad_col={d.max() if len(d) else -1} gpu_idx={gi[d.max()] if len(d) else -1} ref_idx={ei[d.max()] if len(d) else -1}"
            msg += f" gpu_colsum_ok={(gp[b].sum(0)[:t_y[b]]==1).all()}"
        print(msg, flush=True)
