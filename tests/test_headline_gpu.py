"""The bench configuration (BASELINE config 3: Tx=120, Ty=600) pinned against the reference in both
precisions.

* headline_golden.npz: the REFERENCE MatchaTTS.forward (matcha_tts.py:247-325) at B=4, 120x600,
  fp32, eval mode, t / z replayed from the seed (tests/golden/_decoder_golden.py headline_case).
* B=32 (the bench batch): the product against the CPU oracle restatement (oracle/matcha_oracle.py,
  itself pinned to the reference fixtures) on the same weights, tokens, mels, t and z.

32-true: alignment bit-exact, each loss within 1e-4 relative (the north star's bar).
bf16-parity (the bench default since round 4): bf16-mixed with split bf16 weight planes
(MTTS_GEMM_F_W_SPLIT: the fp32 weights' static rounding -- the dominant bf16 loss error, tools/r3/
precision_budget.py -- drops out) and the text encoder's FORWARD on the exact-fp32 MFMA with fp32 weights
(precise_forward("fp32"): 32-true's forward arithmetic), backward bf16: the encoder's activation rounding
decided every alignment near-tie.  Bar: alignment bit-exact and every loss (duration included) within 1e-4
relative.  bf16-parity-fp32enc: round 3's policy (the whole encoder in exact fp32, backward too), same bar.
bf16-parity-bf16x3: the encoder forward in bf16x3 (MTTS_GEMM_F_A_SPLIT, A_hi W_hi + A_hi W_lo + A_lo W_hi,
~16 significant bits): losses at the bar, but at B=4 one alignment near-tie of the reference fixture
flipped (agreement 0.99968, round-4 GPU run) -- measured, held to the one-plane agreement bound.
bf16-mixed one plane (the throughput mode): measured 2.3e-4 .. 3.3e-4 (prior / diff at B=32, 512x4096)
-> bound 5e-4, documented as missing the bar; its duration loss moves with MAS boundary flips (3e-3 at
B=32, 9.9e-2 at B=4 -> bound 0.15) -- under a perturbed lattice near-tied DP decisions flip and move row
boundaries by a frame, which moves log(duration) by up to log 2 for short rows, so its alignment is
compared cell by cell (BF16_ATTN_AGREE).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
import torch

from golden._decoder_golden import attn_row_starts
from golden.weights_recipe import apply_recipe

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GH = np.load(Path(__file__).parent / "golden" / "headline_golden.npz")
FP32_LOSS_RTOL = 1e-4       # north star: mel / flow-matching loss within 1e-4 relative
PARITY_RTOL = np.array([1e-4, 1e-4, 1e-4])    # bf16-parity (dur, prior, diff): every loss at the bar
BF16_LOSS_RTOL = np.array([0.15, 5e-4, 5e-4])  # bf16-mixed, one weight plane: measured, misses the bar
BF16_ATTN_AGREE = 0.99      # one plane: fraction of [Tx, Ty] alignment cells equal to the fp32 reference path
# precision -> (bf16 autocast, split weight planes, MatchaTTS.encoder_precision)
MODES = {"32-true": (False, False, "bf16"), "bf16-mixed": (True, False, "bf16"),
         "bf16-parity": (True, True, "fp32fwd"), "bf16-parity-fp32enc": (True, True, "fp32"),
         "bf16-parity-bf16x3": (True, True, "bf16x3"), "bf16-parity-bf16x6": (True, True, "bf16x6")}
# bf16x6 is not at the bar: measured B=4 alignment 0.99990 (2 of 437 durations moved), duration loss 4e-4
PARITY_MODES = ("bf16-parity", "bf16-parity-fp32enc")
# The at-bar modes' BACKWARD is bf16: their gradients pinned against the reference fixture's
# per-tensor gradient norms (B=4) and the 32-true step's gradients / AdamW update (B=32, below).  Bounds from
# the round-5 GPU measurement (profiles/r05/grads/); the B=32 bounds at measured + 50 % (round 6, VERDICT r5 #4:
# re-measured unchanged on HEAD, profiles/r06/).  bf16-parity measured: B=4 global norm 3.3e-4, per-tensor norms
# median 4.3e-4 / max 1.9e-2; B=32 vs 32-true: ||g - g32|| / ||g32|| 2.99e-3, global norm 4.28e-5, update 7.58e-2
# (the first Adam step is ~lr * sign(g): near-zero entries flip; bf16-mixed 0.107)
GRAD_NORM_GLOBAL_RTOL = 1e-3
GRAD_NORM_MEDIAN_RTOL = 1.5e-3
GRAD_NORM_MAX_RTOL = 6e-2
B32_GRAD_GLOBAL_RTOL = 4.5e-3  # ||g - g32|| / ||g32||
B32_GRAD_NORM_RTOL = 6.5e-5    # | ||g|| - ||g32|| | / ||g32||
B32_UPDATE_RTOL = 0.114        # one clip + AdamW step from zero moments


def run_precision(model, precision, fn):
    """fn() under `precision` (MODES): 32-true; bf16-mixed (one weight plane); bf16-parity (split weight
    planes + the text encoder's forward in exact fp32, backward bf16 -- the bench default);
    bf16-parity-fp32enc (split weight planes + the whole text encoder in exact fp32, round 3's policy);
    bf16-parity-bf16x3 / -bf16x6 (split weight planes + the encoder forward in bf16x3 / bf16x6: both
    flip alignment cells at B=4, so they are held to the one-plane bounds)."""
    from matcha.models.components import _ops as O
    from matcha.precision import precision_context

    if precision in ("32-true", "bf16-mixed", "bf16-parity"):  # the Trainer's own precisions, its contexts
        with precision_context(precision, model):
            return fn()
    amp, split, enc = MODES[precision]
    old = O.set_weight_split(split)
    model.encoder_precision = enc
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            return fn()
    finally:
        O.set_weight_split(old)
        model.encoder_precision = None


def check_bf16(precision, err, agree):
    """The at-bar modes: alignment bit-exact, every loss within 1e-4; one plane: the measured bounds."""
    if precision in PARITY_MODES:
        assert agree == 1.0, f"{precision}: alignment not exact ({agree})"
        assert (err <= PARITY_RTOL).all(), err
    else:
        assert (err <= BF16_LOSS_RTOL).all(), err
        assert agree >= BF16_ATTN_AGREE


def _run(model, x, xl, y, yl, t, z, precision):
    def fn():
        dur, prior, diff, attn = model(x, xl, y, yl, t=t, z=z)
        (dur + prior + diff).backward()
        return dur, prior, diff, attn

    dur, prior, diff, attn = run_precision(model, precision, fn)
    torch.cuda.synchronize()
    return np.array([dur.item(), prior.item(), diff.item()]), attn.detach().cpu().numpy()


def _product(seed):
    from matcha.models.matcha_tts import MatchaTTS

    model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(DEV)
    apply_recipe(model, seed)
    model.eval()
    return model


def _agree(attn, ref_attn, xl, yl):
    """Fraction of valid [t_x, t_y] cells where two 0/1 alignments agree."""
    same = total = 0
    for b in range(attn.shape[0]):
        a, r = attn[b, : xl[b], : yl[b]], ref_attn[b, : xl[b], : yl[b]]
        same += int((a == r).sum())
        total += a.size
    return same / total


@pytest.mark.parametrize("precision", list(MODES))
def test_headline_b4_vs_reference(precision):
    model = _product(41)
    g = lambda k: torch.from_numpy(GH[k]).to(DEV)  # noqa: E731
    got, attn = _run(model, g("h_x"), g("h_x_lengths"), g("h_y"), g("h_y_lengths"), g("h_t"), g("h_z"), precision)
    want = GH["h_losses"]
    err = np.abs(got - want) / np.abs(want)
    rows = attn_row_starts(attn.astype(np.int8))
    print(f"{precision}: losses {got} reference {want} rel err {err}")
    if precision == "32-true":
        np.testing.assert_array_equal(rows, GH["h_attn_rows"])
        assert (err <= FP32_LOSS_RTOL).all(), err
        gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for _, p in model.named_parameters()])
        np.testing.assert_allclose(gn, GH["h_grad_norms"], rtol=5e-3, atol=1e-6)
    else:
        import oracle_bind as OB

        xl, yl = GH["h_x_lengths"], GH["h_y_lengths"]
        ref_attn = OB.row_start_to_path(GH["h_attn_rows"], xl, yl, attn.shape[-1])
        agree = _agree(attn.astype(np.int8), ref_attn, xl, yl)
        with torch.no_grad():
            enc32 = model.encoder(g("h_x"), g("h_x_lengths"))
            with torch.autocast("cuda", dtype=torch.bfloat16):
                enc16 = model.encoder(g("h_x"), g("h_x_lengths"))
        m = enc32[2]
        d_logw = ((enc16[1] - enc32[1]) * m).abs().max().item()
        r_mu = ((enc16[0] - enc32[0]) * m).norm().item() / (enc32[0] * m).norm().item()
        dur16 = attn.astype(np.int64).sum(-1)
        dur32 = ref_attn.astype(np.int64).sum(-1)
        print(f"bf16 alignment agreement {agree:.5f}; rows whose duration moved {(dur16 != dur32).sum()} of "
              f"{int(xl.sum())}; max |logw16 - logw32| {d_logw:.4f}; mu_x rel err {r_mu:.2e}")
        check_bf16(precision, err, agree)
        # gradients of the same backward against the reference's own (fp32 CPU) per-parameter gradient norms
        gn = np.array([p.grad.double().norm().item() if p.grad is not None else 0.0 for _, p in model.named_parameters()])
        ref = GH["h_grad_norms"]
        big = ref > 1e-3 * ref.max()  # tensors whose gradient is not ~0 (a relative error of ~0 is noise)
        rel = np.abs(gn - ref)[big] / ref[big]
        tot = abs(np.sqrt((gn ** 2).sum()) - np.sqrt((ref ** 2).sum())) / np.sqrt((ref ** 2).sum())
        print(f"{precision}: grad norms vs reference: global {tot:.2e}, per tensor median {np.median(rel):.2e} "
              f"max {rel.max():.2e} ({int(big.sum())} tensors)")
        if precision in PARITY_MODES:
            assert tot <= GRAD_NORM_GLOBAL_RTOL, tot
            assert np.median(rel) <= GRAD_NORM_MEDIAN_RTOL, np.median(rel)
            assert rel.max() <= GRAD_NORM_MAX_RTOL, rel.max()


_B32 = {}


def _oracle_b32():
    """The CPU oracle's fp32 forward at the bench batch (B=32, 120x600), computed once per session."""
    if not _B32:
        import oracle_bind as OB
        from matcha.training import synthetic_batch
        from oracle import matcha_oracle as MO

        def mp(value, mask):
            return torch.from_numpy(OB.maximum_path(value.detach().float().numpy(), mask.detach().float().numpy())[0])

        ref = MO.MatchaTTSOracle(150, 80, 192, maximum_path=mp)
        apply_recipe(ref, 43)
        ref.eval()
        b = synthetic_batch(32, 120, 600, seed=1000, device="cpu")
        gen = torch.Generator().manual_seed(44)
        t = torch.rand(32, 1, 1, generator=gen)
        z = torch.randn(32, 80, 600, generator=gen)
        with torch.no_grad():
            dur, prior, diff, attn = ref(b["x"], b["x_lengths"], b["y"], b["y_lengths"], t=t, z=z)
        _B32.update(batch=b, t=t, z=z, losses=np.array([float(dur), float(prior), float(diff)]),
                    attn=attn.numpy().astype(np.int8))
    return _B32


@pytest.mark.parametrize("precision", list(MODES))
def test_bench_batch_b32_vs_oracle(precision):
    o = _oracle_b32()
    model = _product(43)
    b = {k: v.to(DEV) for k, v in o["batch"].items()}
    got, attn = _run(model, b["x"], b["x_lengths"], b["y"], b["y_lengths"], o["t"].to(DEV), o["z"].to(DEV), precision)
    err = np.abs(got - o["losses"]) / np.abs(o["losses"])
    xl, yl = o["batch"]["x_lengths"].numpy(), o["batch"]["y_lengths"].numpy()
    agree = _agree(attn.astype(np.int8), o["attn"], xl, yl)
    print(f"B=32 {precision}: losses {got} oracle {o['losses']} rel err {err} alignment agreement {agree:.6f}")
    if precision == "32-true":
        np.testing.assert_array_equal(attn.astype(np.int8), o["attn"])
        assert (err <= FP32_LOSS_RTOL).all(), err
    else:
        check_bf16(precision, err, agree)
    assert all(p.grad is None or torch.isfinite(p.grad).all() for p in model.parameters())


@pytest.mark.parametrize("precision", PARITY_MODES[:1] + ("bf16-mixed",))
def test_bench_batch_b32_grads_vs_32true(precision):
    """The benched step's product is a parameter UPDATE: its gradients (bf16 backward) and one clip + AdamW step
    against the 32-true step's on the bench batch (recipe weights 43, eval mode, same t / z).  32-true's own
    gradients are pinned element-wise to the oracle (test_model_gpu.py::test_matcha_gradients_elementwise_vs_oracle)."""
    from matcha.precision import grad_errors, loss_and_grads

    o = _oracle_b32()
    model = _product(43)
    b = {k: v.to(DEV) for k, v in o["batch"].items()}
    t, z = o["t"].to(DEV), o["z"].to(DEV)
    _, g32, _ = loss_and_grads(model, b, "32-true", t=t, z=z)
    _, g16, _ = loss_and_grads(model, b, precision, t=t, z=z)
    params = {n: p.detach() for n, p in model.named_parameters()}
    e = grad_errors(g16, g32, params)
    print(f"B=32 {precision} gradients vs 32-true: {e}")
    if precision in PARITY_MODES:
        assert e["global_rel_err"] <= B32_GRAD_GLOBAL_RTOL, e
        assert e["norm_rel_err"] <= B32_GRAD_NORM_RTOL, e
        assert e["update_rel_err"] <= B32_UPDATE_RTOL, e
    assert e["global_rel_err"] < 0.5, e  # one plane: measured, finite and in range


def test_bench_batch_b32_grad_error_attribution():
    """Where the bf16-parity gradient error comes from (matcha/precision.py error_attribution): holding one module
    family in 32-true removes that family's share.  Measured (round 6, B=32 bench batch): global 2.99e-3; held
    decoder 1.50e-3 (source 75 %), text encoder 2.60e-3 (24 %), decoder Resnet1D blocks 2.62e-3 (23 %), FeedForward
    2.81e-3 (12 %), attention 2.83e-3 (10 %) -- diffuse: no family carries a majority but the decoder as a whole."""
    from matcha.precision import HOLD_FAMILIES, error_attribution, loss_and_grads

    o = _oracle_b32()
    model = _product(43)
    b = {k: v.to(DEV) for k, v in o["batch"].items()}
    t, z = o["t"].to(DEV), o["z"].to(DEV)
    _, g32, _ = loss_and_grads(model, b, "32-true", t=t, z=z)
    a = error_attribution(model, b, "bf16-parity", g32, t=t, z=z)
    print(f"B=32 bf16-parity gradient error attribution: {a}")
    assert a["global_rel_err"] <= B32_GRAD_GLOBAL_RTOL
    assert set(a["held"]) == set(HOLD_FAMILIES)
    assert abs(sum(a["lands_share"].values()) - 1.0) < 1e-3
    held = {k: v["global_rel_err"] for k, v in a["held"].items()}
    for fam in HOLD_FAMILIES:  # holding any family in 32-true never makes the error worse (beyond noise)
        assert held[fam] <= a["global_rel_err"] * 1.02, (fam, held[fam], a["global_rel_err"])
    assert held["decoder"] <= 0.7 * a["global_rel_err"]  # the decoder's bf16 backward is the largest source
    sub = sum(a["held"][f]["source_share"] for f in ("decoder_resnets", "decoder_attention", "decoder_ff"))
    assert sub <= a["held"]["decoder"]["source_share"] + 0.05  # the decoder's parts do not exceed the whole
