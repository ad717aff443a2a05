"""The fused pre-LN sub-blocks' GEMMs and weight gradients at the train step's shapes (M = 32 x 600 and
32 x 300), fp32 vs bf16 operand storage, every schedule (graph-timed).  One JSON line per (op, storage,
schedule); the `best` lines summarise.  python tools/preln_shapes.py > log"""
import json, math, sys
from pathlib import Path
import torch
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd")]
from matcha.models.components import _ops as O

dev = torch.device("cuda")


def t_ev(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters): fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3): g.replay()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * iters) * 1e3


P = O.PREC_BF16
seed = torch.tensor([12345, 678], dtype=torch.int32, device=dev)
ONLY = sys.argv[1].split(",") if len(sys.argv) > 1 and __name__ == "__main__" else None


def gemm_case(name, M, K, N, a16, c16=False, act=O.ACT_NONE, pre=False, aux=False, res=False, bias=True):
    A = torch.randn(M, K, device=dev)
    A = A.to(torch.bfloat16) if a16 else A
    w = torch.randn(N, K, device=dev) / math.sqrt(K)
    Wp, Kp = O.pack_weight(w, P)
    b = torch.randn(N, device=dev) if bias else None
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if c16 else torch.float32)
    Cp = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if pre else None
    ax = torch.randn(M, N, device=dev).to(torch.bfloat16) if aux else None
    r = torch.randn(M, N, device=dev) if res else None
    cands = [-1] + list(range(32, 48)) if a16 else [-1, 7, 12] + list(range(32, 48))
    best = None
    allc = {}
    for cfg in cands:
        run = lambda: O._gemm(A, M, M, 1, 1, [0], K, Wp, Kp, N, C, M, prec=P, bias=b, act=act, C_pre=Cp, aux=ax,
                              residual=r, seed=seed, tile_cfg=cfg)
        try:
            run(); torch.cuda.synchronize()
        except Exception:
            continue
        us = t_ev(run)
        allc[cfg] = round(us, 1)
        if cfg == -1:
            dflt = us
        if best is None or us < best[1]:
            best = (cfg, us)
    print(json.dumps({"op": name, "M": M, "A": "bf16" if a16 else "fp32", "default_us": round(dflt, 1),
                      "best_cfg": best[0], "best_us": round(best[1], 1),
                      "tflops_default": round(2 * M * N * K / dflt / 1e6, 1), "all": allc}), flush=True)


def wgrad_case(name, M, K, N, a16, y16):
    A = torch.randn(M, K, device=dev)
    A = A.to(torch.bfloat16) if a16 else A
    dY = torch.randn(M, N, device=dev)
    dY = dY.to(torch.bfloat16) if y16 else dY
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    res = {}
    for kb, tb, dp in [(-1, -1, -1), (32, -1, 1), (32, -1, 2), (64, -1, 2), (32, 512, 2), (32, 1024, 2), (64, 256, 2)]:
        run = lambda: O._wgrad(dY, M, 1, 0, A, M, M, 1, 1, [0], K, N, dw, (K, 1, 0), prec=P, db=db,
                               rows_per_step=kb, target_blocks=tb, depth=dp)
        try:
            run(); torch.cuda.synchronize()
        except Exception as e:
            continue
        res[(kb, tb, dp)] = round(t_ev(run), 1)
    best = min(res, key=res.get)
    print(json.dumps({"op": name, "M": M, "A": "bf16" if a16 else "fp32", "dY": "bf16" if y16 else "fp32",
                      "default_us": res[(-1, -1, -1)], "best": list(best), "best_us": res[best]}), flush=True)


if __name__ == "__main__":
  for M in (19200, 9600):
      for a16 in (False, True):
          if not ONLY or "gemm" in ONLY:
              gemm_case("qkv", M, 256, 768, a16, bias=False)
              gemm_case("ff1_gelu", M, 256, 1024, a16, c16=True, act=O.ACT_GELU, pre=True)
              gemm_case("ff_dgrad_dz_dn", M, 1024, 256, a16, bias=False)
          if not ONLY or "wgrad" in ONLY:
              wgrad_case("dW_qkv", M, 256, 768, a16, False)
              for y16 in (False, True):
                  wgrad_case("dW1", M, 256, 1024, a16, y16)
      if not ONLY or "gemm" in ONLY:
          for c16 in (False, True):  # dgelu producing dz fp32 / bf16
              A = None
              gemm_case("ff2_dgrad_dgelu_C" + ("16" if c16 else "32"), M, 256, 1024, False, c16=c16, act=O.ACT_DGELU,
                        aux=True, bias=False)
