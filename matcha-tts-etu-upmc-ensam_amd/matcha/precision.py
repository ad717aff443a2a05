"""Precision modes of the train step and the error of a mode's gradients / optimizer update against 32-true.

The Trainer's precisions ("32-true", "bf16-mixed", "bf16-parity") as context managers, so that a test or the
bench computes a forward + backward with exactly the step's numerics outside the Trainer, and the comparisons
the bench line reports as ``precision_check.grads`` (the benched bf16-parity step's gradients
and AdamW update against the reference precision, ``train.py:85`` ``precision: 32-true``):

* ``global_rel_err``      ||g - g32|| / ||g32|| over every parameter gradient, flattened;
* ``norm_rel_err``        | ||g|| - ||g32|| | / ||g32||  (the clip threshold's input,
                          ``baselightningmodule.py:244-245`` logs it as grad_norm);
* ``tensor_rel_err``      per parameter tensor ||g_t - g32_t|| / ||g32_t||: max (and which) and median;
* ``update_rel_err``      one clip(1.0) + AdamW(1e-4, (0.9, 0.999), 1e-8, wd 1e-6) step from zero moments on
                          both gradient sets: ||dtheta - dtheta32|| / ||dtheta32||.

Attribution: ``hold_fp32(model, family)`` runs one module family's forward AND backward in
32-true's arithmetic (autocast off around it: exact-fp32 MFMA, fp32-stored activations, fp32 weight operands)
while the rest of the model keeps the benched precision; ``error_attribution`` reports, per family, how much of
the global gradient error disappears when that family is held (its "source" share, 1 - (e_held / e)^2) and how
the squared error of the un-held run is distributed over the parameters' owners (where it "lands").

Measurement code: no oracle, no reference import; the parameters of the model are left unchanged.
"""
from __future__ import annotations

import contextlib

import torch

from matcha.models.components import _ops as O

PRECISIONS = ("32-true", "bf16-mixed", "bf16-parity")


@contextlib.contextmanager
def precision_context(precision: str, model=None):
    """The Trainer's numerics for `precision` (Trainer._autocast): bf16 autocast for the bf16 modes, plus
    _ops.parity_policy() (split weight planes but the decoder FF up-projection, the text encoder's forward on
    the exact-fp32 MFMA) for bf16-parity.  `model.encoder_precision` is cleared to the ambient default for the
    duration (restored after)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision {precision!r} not in {PRECISIONS}")
    old_enc = getattr(model, "encoder_precision", None) if model is not None else None
    if model is not None:
        model.encoder_precision = None
    old_split = O.set_weight_split(False)
    try:
        with contextlib.ExitStack() as st:
            if precision != "32-true":
                st.enter_context(torch.autocast("cuda", dtype=torch.bfloat16))
            if precision == "bf16-parity":
                st.enter_context(O.parity_policy())
            yield
    finally:
        O.set_weight_split(old_split)
        if model is not None:
            model.encoder_precision = old_enc


# module families of MatchaTTS for the attribution (hold_fp32): the text encoder (its forward is already exact fp32
# under bf16-parity, so holding it removes its bf16 backward), the whole decoder, and the decoder's three GEMM
# families -- Resnet1D blocks (k=3 convs, GroupNorm+Mish, res_conv), the pre-LN attention sub-blocks (LN, q|k|v,
# attention, out-projection) and the pre-LN FeedForward sub-blocks (LN, GELU up-projection, down-projection)
HOLD_FAMILIES = ("text_encoder", "decoder", "decoder_resnets", "decoder_attention", "decoder_ff")


def _fp32_wrap(fn):
    def run(*a, **k):
        with torch.autocast("cuda", enabled=False):
            return fn(*a, **k)
    return run


@contextlib.contextmanager
def hold_fp32(model, family: str | None):
    """Inside a precision_context: `family` (HOLD_FAMILIES) runs forward and backward in 32-true's arithmetic; the
    ops capture their precision at the forward, so the backward follows.  None: nothing held."""
    if family is None:
        yield
        return
    if family not in HOLD_FAMILIES:
        raise ValueError(f"family {family!r} not in {HOLD_FAMILIES}")
    from matcha.models.components import decoder as D

    patches = []  # (owner, attribute, original)
    if family == "text_encoder":
        old = model.encoder_precision
        model.encoder_precision = "fp32"
    elif family == "decoder":
        patches += [(D.Decoder, "forward_tm"), (D.Decoder, "forward_tm_packed")]
    elif family == "decoder_resnets":
        patches += [(D.Resnet1D, "forward_tm")]
    elif family == "decoder_attention":
        patches += [(O, "preln_attention_tm")]
    elif family == "decoder_ff":
        patches += [(O, "preln_ff_tm")]
    saved = [(o, a, getattr(o, a)) for o, a in patches]
    for o, a, f in saved:
        setattr(o, a, _fp32_wrap(f))
    try:
        yield
    finally:
        for o, a, f in saved:
            setattr(o, a, f)
        if family == "text_encoder":
            model.encoder_precision = old


def loss_and_grads(model, batch, precision: str, t=None, z=None, hold: str | None = None):
    """(dur, prior, diff) losses and {name: fp32 gradient} of one forward + backward of `model` on `batch`
    under `precision` (the existing .grad are replaced, then restored to None); hold: a family kept in 32-true
    (hold_fp32)."""
    for p in model.parameters():
        p.grad = None
    with precision_context(precision, model), hold_fp32(model, hold):
        dur, prior, diff, attn = model(batch["x"], batch["x_lengths"], batch["y"], batch["y_lengths"], t=t, z=z)
        (dur + prior + diff).backward()
    grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}
    for p in model.parameters():
        p.grad = None
    return [float(v.detach()) for v in (dur, prior, diff)], grads, attn.detach()


def _adamw_delta(params: dict, grads: dict, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, wd=1e-6, max_norm=1.0):
    """Parameter change of one clip_grad_norm_(max_norm) + AdamW step from zero moments (torch's formulas, in
    float64 so the comparison measures the gradients, not this arithmetic)."""
    names = [n for n in params if n in grads]
    g = {n: grads[n].double() for n in names}
    total = torch.sqrt(sum((v * v).sum() for v in g.values()))
    scale = min(1.0, max_norm / (float(total) + 1e-6))
    out = {}
    b1, b2 = betas
    for n in names:
        gn = g[n] * scale
        m = (1 - b1) * gn
        v = (1 - b2) * gn * gn
        mhat, vhat = m / (1 - b1), v / (1 - b2)
        p = params[n].double()
        out[n] = -lr * wd * p - lr * mhat / (vhat.sqrt() + eps)
    return out


def grad_errors(grads: dict, ref: dict, params: dict | None = None) -> dict:
    """The module docstring's comparisons of `grads` against `ref` (same parameter names)."""
    names = [n for n in ref if n in grads]
    flat = torch.cat([grads[n].reshape(-1).double() for n in names])
    flat_ref = torch.cat([ref[n].reshape(-1).double() for n in names])
    nref = float(flat_ref.norm())
    per = []
    for n in names:
        d = float((grads[n].double() - ref[n].double()).norm())
        r = float(ref[n].double().norm())
        per.append((d / r if r > 0 else (0.0 if d == 0 else float("inf")), n))
    per.sort()
    out = {"global_rel_err": float((flat - flat_ref).norm()) / nref,
           "norm_rel_err": abs(float(flat.norm()) - nref) / nref,
           "tensor_rel_err_max": per[-1][0], "tensor_rel_err_max_param": per[-1][1],
           "tensor_rel_err_median": per[len(per) // 2][0], "tensors": len(per)}
    if params is not None:
        d = _adamw_delta(params, grads)
        d_ref = _adamw_delta(params, ref)
        num = torch.sqrt(sum(((d[n] - d_ref[n]) ** 2).sum() for n in d_ref))
        den = torch.sqrt(sum((d_ref[n] ** 2).sum() for n in d_ref))
        out["update_rel_err"] = float(num / den)
    return out


def _owner(name: str) -> str:
    """The attribution family a parameter belongs to (where its gradient error lands)."""
    if name.startswith("encoder."):
        return "text_encoder"
    if ".attn1." in name or ".norm1." in name:
        return "decoder_attention"
    if ".ff." in name or ".norm3." in name:
        return "decoder_ff"
    parts = name.split(".")
    if len(parts) > 4 and parts[2] in ("Downsampling_Blocks", "Mid_Blocks", "Upsampling_Blocks") and parts[4] == "0":
        return "decoder_resnets"
    return "decoder_other"  # sampling convs, final head, time MLP


def error_attribution(model, batch, precision: str, ref: dict, t=None, z=None) -> dict:
    """Per family: the global gradient error of `precision` with the family held in 32-true, its source share
    1 - (e_held / e)^2 (the fraction of the squared error that family's bf16 arithmetic causes, interactions
    aside), and where the un-held squared error lands (share per owning family)."""
    _, g, _ = loss_and_grads(model, batch, precision, t=t, z=z)
    names = [n for n in ref if n in g]
    sq = {n: float(((g[n].double() - ref[n].double()) ** 2).sum()) for n in names}
    nref2 = sum(float((ref[n].double() ** 2).sum()) for n in names)
    e2 = sum(sq.values())
    lands = {}
    for n, v in sq.items():
        lands[_owner(n)] = lands.get(_owner(n), 0.0) + v
    out = {"global_rel_err": (e2 / nref2) ** 0.5,
           "lands_share": {k: round(v / e2, 4) for k, v in sorted(lands.items())} if e2 > 0 else {},
           "held": {}}
    for fam in HOLD_FAMILIES:
        _, gh, _ = loss_and_grads(model, batch, precision, t=t, z=z, hold=fam)
        eh2 = sum(float(((gh[n].double() - ref[n].double()) ** 2).sum()) for n in names)
        out["held"][fam] = {"global_rel_err": round((eh2 / nref2) ** 0.5, 7),
                            "source_share": round(1.0 - eh2 / e2, 4) if e2 > 0 else 0.0}
    return out
