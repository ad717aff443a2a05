"""Generates the golden fixtures under tests/golden/ from the REFERENCE itself (run in the dev
container, where /root/reference exists; the fixtures are committed and travel to the GPU box).

    make -C oracle ref                      # compiles the reference core.pyx into oracle/_ref/
    python tests/golden/make_golden.py mas  # MAS fixtures from the compiled Cython
    python tests/golden/make_golden.py decoder  # decoder/CFM/MatchaTTS fixtures (see _decoder_golden.py)
    python tests/golden/make_golden.py headline # MatchaTTS.forward at the bench shape (B=4, 120x600)
    python tests/golden/make_golden.py synth    # MatchaTTS.synthesise with the z draw replayed

MAS fixtures (mas_golden.npz) -- outputs of compute_batch_alignments (core.pyx:101-128) and of the
reference wrapper maximum_path (__init__.py:40-55):
  random_*   : N(-100, 10^2) lattices, ragged lengths, shapes (1,1) ... (120,600)      [SURVEY 8c-i]
  ties_*     : integer lattices randint(-2, 1) -- pin the `>=` -> diagonal tie rule     [8c-ii]
  zero3x6    : all-zero 3x6 known answer                                                [8c-iii]
  dp_*       : the Cython-mutated values lattice (bit patterns) for the small cases     [8c-iv]
  masked_*   : maximum_path() with a mask that has holes inside the rectangle (value*mask)
  large_*    : B=32 120x600 and B=8 512x4096 from numpy default_rng recipes; row starts + SHA-256
               of the int8 path                                                         [8c-v]
Paths are stored as int32 row starts (row x covers [start[x], start[x+1]-1], last row to t_y-1;
-1 = no path), which determines the dense path exactly.
"""
from __future__ import annotations

import hashlib
import importlib.util
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = Path("/root/reference")


def load_cython_core():
    so = sorted((ROOT / "oracle" / "_ref").glob("core*.so"))
    if not so:
        raise SystemExit("oracle/_ref/core*.so missing: run `make -C oracle ref` first")
    spec = importlib.util.spec_from_file_location("core", so[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def path_to_row_start(path: np.ndarray) -> np.ndarray:
    """[B,Tx,Ty] {0,1} -> int32 [B,Tx] first column per row (-1 if the row is empty)."""
    B, Tx, Ty = path.shape
    rs = np.full((B, Tx), -1, np.int32)
    nz = path != 0
    has = nz.any(axis=2)
    first = nz.argmax(axis=2)
    rs[has] = first[has]
    return rs


def ref_maximum_path(core, value: np.ndarray, mask: np.ndarray) -> np.ndarray:
    """The reference wrapper (__init__.py:40-55) with numpy in place of torch (same arithmetic)."""
    v = (value * mask).astype(np.float32)
    path = np.zeros_like(v).astype(np.int32)
    t_x = mask.sum(1)[:, 0].astype(np.int32)
    t_y = mask.sum(2)[:, 0].astype(np.int32)
    core.compute_batch_alignments(path, v, t_x, t_y)
    return path


def lengths_mask(B, Tx, Ty, t_x, t_y):
    m = np.zeros((B, Tx, Ty), np.float32)
    for b in range(B):
        m[b, : t_x[b], : t_y[b]] = 1.0
    return m


def ragged(rng, B, Tx, Ty):
    """lengths ~ U[0.7 max, max], element 0 = max, t_x <= t_y."""
    t_x = np.maximum(1, (Tx * rng.uniform(0.7, 1.0, B)).astype(np.int32))
    t_y = np.maximum(1, (Ty * rng.uniform(0.7, 1.0, B)).astype(np.int32))
    t_x[0], t_y[0] = Tx, Ty
    t_y = np.maximum(t_y, t_x)
    return t_x.astype(np.int32), t_y.astype(np.int32)


def large_lattice(seed, B, Tx, Ty):
    """Recipe shared with tests/test_mas_gpu.py (regenerated there, never stored raw)."""
    rng = np.random.default_rng(seed)
    value = rng.normal(-100.0, 10.0, size=(B, Tx, Ty)).astype(np.float32)
    t_x, t_y = ragged(rng, B, Tx, Ty)
    return value, t_x, t_y


def make_mas():
    core = load_cython_core()
    rng = np.random.default_rng(1234)
    out: dict[str, np.ndarray] = {}
    shapes = [(1, 1), (1, 5), (5, 5), (3, 4), (7, 8), (30, 100), (120, 600)]
    for Tx, Ty in shapes:
        B = 4
        value = rng.normal(-100.0, 10.0, size=(B, Tx, Ty)).astype(np.float32)
        t_x, t_y = ragged(rng, B, Tx, Ty)
        path = np.zeros((B, Tx, Ty), np.int32)
        dp = value.copy()
        core.compute_batch_alignments(path, dp, t_x, t_y)
        key = f"random_{Tx}x{Ty}"
        out[key + "_value"] = value
        out[key + "_tx"], out[key + "_ty"] = t_x, t_y
        out[key + "_rowstart"] = path_to_row_start(path)
        if Tx * Ty <= 30 * 100:
            out[key + "_dp"] = dp
        else:
            out[key + "_dpsha"] = np.frombuffer(hashlib.sha256(dp.tobytes()).digest(), np.uint8)
    # tie-heavy integer lattices
    for i in range(3):
        B, Tx, Ty = 8, 10, 25
        value = rng.integers(-2, 1, size=(B, Tx, Ty)).astype(np.float32)
        t_x, t_y = ragged(rng, B, Tx, Ty)
        path = np.zeros((B, Tx, Ty), np.int32)
        dp = value.copy()
        core.compute_batch_alignments(path, dp, t_x, t_y)
        key = f"ties_{i}"
        out[key + "_value"], out[key + "_tx"], out[key + "_ty"] = value, t_x, t_y
        out[key + "_rowstart"] = path_to_row_start(path)
        out[key + "_dp"] = dp
    # all-zero 3x6 known answer
    value = np.zeros((1, 3, 6), np.float32)
    path = np.zeros((1, 3, 6), np.int32)
    core.compute_batch_alignments(path, value.copy(), np.array([3], np.int32), np.array([6], np.int32))
    out["zero3x6_path"] = path.astype(np.int8)
    # maximum_path() wrapper with holes in the mask inside the rectangle (pins value*mask)
    B, Tx, Ty = 4, 20, 60
    value = rng.normal(-5.0, 3.0, size=(B, Tx, Ty)).astype(np.float32)
    t_x, t_y = ragged(rng, B, Tx, Ty)
    mask = lengths_mask(B, Tx, Ty, t_x, t_y)
    holes = (rng.random((B, Tx, Ty)) < 0.2).astype(np.float32)
    holes[:, 0, :] = 0.0
    holes[:, :, 0] = 0.0
    mask = mask * (1.0 - holes)
    out["masked_value"], out["masked_mask"] = value, mask.astype(np.float32)
    out["masked_rowstart"] = path_to_row_start(ref_maximum_path(core, value, mask))
    # large recipes
    for name, seed, (B, Tx, Ty) in (("large_b32", 7, (32, 120, 600)), ("large_long", 8, (8, 512, 4096))):
        value, t_x, t_y = large_lattice(seed, B, Tx, Ty)
        path = np.zeros((B, Tx, Ty), np.int32)
        core.compute_batch_alignments(path, value, t_x, t_y)
        out[name + "_shape"] = np.array([seed, B, Tx, Ty], np.int64)
        out[name + "_tx"], out[name + "_ty"] = t_x, t_y
        out[name + "_rowstart"] = path_to_row_start(path)
        out[name + "_pathsha"] = np.frombuffer(hashlib.sha256(path.astype(np.int8).tobytes()).digest(),
                                               np.uint8)
    np.savez_compressed(HERE / "mas_golden.npz", **out)
    print("wrote", HERE / "mas_golden.npz", sum(v.nbytes for v in out.values()), "bytes raw")


if __name__ == "__main__":
    what = sys.argv[1:] or ["mas"]
    if "mas" in what:
        make_mas()
    if "decoder" in what:
        sys.path.insert(0, str(HERE))
        import _decoder_golden  # noqa: E402

        _decoder_golden.main()
    if "headline" in what or "synth" in what:
        sys.path.insert(0, str(HERE))
        import _decoder_golden  # noqa: E402

        if "headline" in what:
            _decoder_golden.main_headline()
        if "synth" in what:
            _decoder_golden.main_synth()
