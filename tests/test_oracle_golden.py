"""The CPU oracle (oracle/mas_oracle.c) against the golden vectors produced by the compiled reference
Cython (tests/golden/make_golden.py).  Pins the oracle before any GPU result is compared with it."""
from __future__ import annotations

import hashlib
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as O

G = np.load(Path(__file__).parent / "golden" / "mas_golden.npz")
RANDOM = sorted({k[: -len("_value")] for k in G.files if k.startswith("random_") and k.endswith("_value")})
TIES = sorted({k[: -len("_value")] for k in G.files if k.startswith("ties_") and k.endswith("_value")})


def _check_case(key):
    value, t_x, t_y = G[key + "_value"], G[key + "_tx"], G[key + "_ty"]
    paths, dp = O.mas_batch(value, t_x, t_y)
    exp = O.row_start_to_path(G[key + "_rowstart"], t_x, t_y, value.shape[2])
    np.testing.assert_array_equal(paths.astype(np.int8), exp)
    if key + "_dp" in G.files:  # Cython-mutated lattice, bit for bit
        np.testing.assert_array_equal(dp.view(np.uint32), G[key + "_dp"].view(np.uint32))
    else:
        assert hashlib.sha256(dp.tobytes()).digest() == G[key + "_dpsha"].tobytes()


@pytest.mark.parametrize("key", RANDOM)
def test_oracle_random(key):
    _check_case(key)


@pytest.mark.parametrize("key", TIES)
def test_oracle_ties(key):
    _check_case(key)


def test_oracle_zero_known_answer():
    # Cython on an all-zero 3x6 lattice takes the diagonal on ties
    paths, _ = O.mas_batch(np.zeros((1, 3, 6), np.float32), np.array([3]), np.array([6]))
    np.testing.assert_array_equal(paths.astype(np.int8), G["zero3x6_path"])
    np.testing.assert_array_equal(paths[0], [[1, 1, 1, 1, 0, 0], [0, 0, 0, 0, 1, 0], [0, 0, 0, 0, 0, 1]])


def test_oracle_maximum_path_masked():
    path, t = O.maximum_path(G["masked_value"], G["masked_mask"])
    exp = O.row_start_to_path(G["masked_rowstart"], t[:, 0], t[:, 1], path.shape[2])
    np.testing.assert_array_equal(path.astype(np.int8), exp)


@pytest.mark.parametrize("name", ["large_b32", "large_long"])
def test_oracle_large_recipe(name):
    from golden.make_golden import large_lattice

    seed, B, Tx, Ty = (int(v) for v in G[name + "_shape"])
    value, t_x, t_y = large_lattice(seed, B, Tx, Ty)
    np.testing.assert_array_equal(t_x, G[name + "_tx"])
    np.testing.assert_array_equal(t_y, G[name + "_ty"])
    paths, _ = O.mas_batch(value, t_x, t_y)
    assert hashlib.sha256(paths.astype(np.int8).tobytes()).digest() == G[name + "_pathsha"].tobytes()
    exp = O.row_start_to_path(G[name + "_rowstart"], t_x, t_y, Ty)
    np.testing.assert_array_equal(paths.astype(np.int8), exp)
