"""Deterministic, name-keyed parameter recipe shared by the fixture generator and the tests.

Every parameter is drawn from numpy's default_rng(seed ^ crc32(name)), so any module with the
reference's parameter names (the reference itself, the oracle, the product model) receives the same
weights, independent of construction order or device.  Test infrastructure only."""
from __future__ import annotations

import zlib

import numpy as np
import torch


def param_array(name: str, shape: tuple, seed: int) -> np.ndarray:
    rng = np.random.default_rng((seed * 1_000_003) ^ zlib.crc32(name.encode()))
    leaf = name.rsplit(".", 1)[-1]
    n = int(np.prod(shape)) if shape else 1
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        a = rng.normal(0.0, 1.0 / np.sqrt(fan_in), size=shape)
    elif "norm" in name or leaf == "weight":
        # GroupNorm / LayerNorm affine weights and other 1-D weights
        a = 1.0 + 0.1 * rng.standard_normal(size=shape)
    else:
        a = 0.05 * rng.standard_normal(size=shape)
    del n
    return a.astype(np.float32)


@torch.no_grad()
def apply_recipe(module: torch.nn.Module, seed: int) -> None:
    for name, p in module.named_parameters():
        p.copy_(torch.from_numpy(param_array(name, tuple(p.shape), seed)).to(p.device, p.dtype))


def named_arrays(module: torch.nn.Module, seed: int) -> dict:
    return {n: param_array(n, tuple(p.shape), seed) for n, p in module.named_parameters()}
