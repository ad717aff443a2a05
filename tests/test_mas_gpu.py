"""HIP maximum_path / compute_batch_alignments against the CPU oracle and the Cython golden vectors.

Bar: bit-exact (paths and, for the low-level API, the mutated DP lattice)."""
from __future__ import annotations

import hashlib
from pathlib import Path

import numpy as np
import pytest
import torch

import oracle_bind as O

pytestmark = pytest.mark.gpu

G = np.load(Path(__file__).parent / "golden" / "mas_golden.npz")
DEV = "cuda:0"


def _mp():
    from matcha.utils.monotonic_align import maximum_path, maximum_path_c

    return maximum_path, maximum_path_c


def gpu_path(value: np.ndarray, mask: np.ndarray):
    maximum_path, _ = _mp()
    v = torch.from_numpy(value).to(DEV)
    m = torch.from_numpy(mask).to(DEV)
    p, rs, ln = maximum_path(v, m, return_row_start=True)
    torch.cuda.synchronize()
    return p.cpu().numpy(), rs.cpu().numpy(), ln.cpu().numpy()


def gpu_batch(value: np.ndarray, t_x, t_y):
    _, maximum_path_c = _mp()
    v = torch.from_numpy(np.ascontiguousarray(value, np.float32)).to(DEV)
    p = torch.zeros(value.shape, dtype=torch.int32, device=DEV)
    maximum_path_c(p, v, torch.from_numpy(np.asarray(t_x, np.int32)).to(DEV),
                   torch.from_numpy(np.asarray(t_y, np.int32)).to(DEV))
    torch.cuda.synchronize()
    return p.cpu().numpy(), v.cpu().numpy()


CASES = sorted({k[: -len("_value")] for k in G.files
                if (k.startswith("random_") or k.startswith("ties_")) and k.endswith("_value")})


@pytest.mark.parametrize("key", CASES)
def test_golden_low_level(key):
    value, t_x, t_y = G[key + "_value"], G[key + "_tx"], G[key + "_ty"]
    paths, dp = gpu_batch(value, t_x, t_y)
    exp = O.row_start_to_path(G[key + "_rowstart"], t_x, t_y, value.shape[2])
    np.testing.assert_array_equal(paths.astype(np.int8), exp)
    if key + "_dp" in G.files:
        np.testing.assert_array_equal(dp.view(np.uint32), G[key + "_dp"].view(np.uint32))
    else:
        assert hashlib.sha256(dp.tobytes()).digest() == G[key + "_dpsha"].tobytes()


@pytest.mark.parametrize("key", CASES)
def test_golden_maximum_path(key):
    value, t_x, t_y = G[key + "_value"], G[key + "_tx"], G[key + "_ty"]
    B, Tx, Ty = value.shape
    mask = O.lengths_mask(B, Tx, Ty, t_x, t_y)
    path, rs, ln = gpu_path(value, mask)
    np.testing.assert_array_equal(ln[:, 0], t_x)
    np.testing.assert_array_equal(ln[:, 1], t_y)
    exp = O.row_start_to_path(G[key + "_rowstart"], t_x, t_y, Ty)
    np.testing.assert_array_equal(path, exp.astype(np.float32))
    np.testing.assert_array_equal(rs, G[key + "_rowstart"])


def test_zero_lattice_known_answer():
    path, _, _ = gpu_path(np.zeros((1, 3, 6), np.float32), np.ones((1, 3, 6), np.float32))
    np.testing.assert_array_equal(path.astype(np.int8), G["zero3x6_path"])


def test_mask_with_holes_multiplies_value():
    path, _, ln = gpu_path(G["masked_value"], G["masked_mask"])
    exp = O.row_start_to_path(G["masked_rowstart"], ln[:, 0], ln[:, 1], path.shape[2])
    np.testing.assert_array_equal(path.astype(np.int8), exp)


@pytest.mark.parametrize("name", ["large_b32", "large_long"])
def test_large_recipes(name):
    from golden.make_golden import large_lattice

    seed, B, Tx, Ty = (int(v) for v in G[name + "_shape"])
    value, t_x, t_y = large_lattice(seed, B, Tx, Ty)
    mask = O.lengths_mask(B, Tx, Ty, t_x, t_y)
    path, rs, _ = gpu_path(value, mask)
    np.testing.assert_array_equal(rs, G[name + "_rowstart"])
    assert hashlib.sha256(path.astype(np.int8).tobytes()).digest() == G[name + "_pathsha"].tobytes()


def _rand_case(rng, B, Tx, Ty, ties=False):
    if ties:
        value = rng.integers(-2, 1, size=(B, Tx, Ty)).astype(np.float32)
    else:
        value = rng.normal(-100.0, 10.0, size=(B, Tx, Ty)).astype(np.float32)
    t_x = rng.integers(1, Tx + 1, size=B).astype(np.int32)
    t_y = np.array([rng.integers(min(t, Ty), Ty + 1) for t in t_x], np.int32)
    t_x = np.minimum(t_x, t_y)
    return value, t_x, t_y


@pytest.mark.parametrize("Tx,Ty", [(1, 1), (2, 3), (63, 64), (64, 64), (65, 130), (127, 129),
                                   (128, 128), (129, 301), (200, 203), (255, 600), (256, 257),
                                   (257, 700), (300, 999), (511, 1001), (512, 512), (77, 33 * 32 + 5),
                                   (513, 600), (700, 1501), (1024, 1024), (1000, 2100), (1025, 1100),
                                   (1500, 2999), (2048, 2048), (2047, 4096), (2049, 2100), (3000, 3333),
                                   (4095, 4095), (4096, 4200)])
def test_random_vs_oracle(Tx, Ty):
    """Every DP specialisation -- the one-wave kernel (Tx <= 64) and the multi-wave one (2 / 4 / 8 waves,
    1 / 2 / 4 / 8 rows per lane, up to Tx = 4096) --, odd Ty (scalar loads), LDS- and HBM-resident
    backpointers, square lattices (forced diagonal), partial last 32-column chunks, and ties."""
    rng = np.random.default_rng(Tx * 10007 + Ty)
    for ties in (False, True):
        value, t_x, t_y = _rand_case(rng, 3, Tx, max(Ty, Tx), ties)
        Ty_ = value.shape[2]
        t_y = np.maximum(t_y, t_x)
        exp_p, exp_dp = O.mas_batch(value, t_x, t_y)
        got_p, got_dp = gpu_batch(value, t_x, t_y)
        np.testing.assert_array_equal(got_p, exp_p)
        np.testing.assert_array_equal(got_dp.view(np.uint32), exp_dp.view(np.uint32))
        mask = O.lengths_mask(3, Tx, Ty_, t_x, t_y)
        path, _, _ = gpu_path(value, mask)
        np.testing.assert_array_equal(path, exp_p.astype(np.float32))


def test_undefined_reference_cases_give_zero_paths():
    """t_x > t_y and empty masks are UB in the Cython (core.pyx:37-41); defined as no path here."""
    B, Tx, Ty = 3, 10, 8
    value = np.random.default_rng(0).normal(size=(B, Tx, Ty)).astype(np.float32)
    t_x = np.array([10, 0, 5], np.int32)
    t_y = np.array([8, 8, 8], np.int32)
    mask = O.lengths_mask(B, Tx, Ty, t_x, t_y)
    path, rs, ln = gpu_path(value, mask)
    assert path[0].sum() == 0 and path[1].sum() == 0
    exp_p, _ = O.mas_batch(value[2:], t_x[2:], t_y[2:])
    np.testing.assert_array_equal(path[2:], exp_p.astype(np.float32))
    assert (rs[0] == -1).all() and (rs[1] == -1).all()


def test_properties_full_size_and_dtypes():
    """Size-independent properties at the bench shape (B=32, 120x600): one 1 per column y < t_y,
    monotone, (0,0) and (t_x-1,t_y-1) on the path; fp16/bf16 value return value's dtype."""
    maximum_path, _ = _mp()
    rng = np.random.default_rng(5)
    B, Tx, Ty = 32, 120, 600
    value = rng.normal(-100.0, 10.0, size=(B, Tx, Ty)).astype(np.float32)
    t_x = np.maximum(1, (Tx * rng.uniform(0.7, 1.0, B)).astype(np.int32))
    t_y = np.maximum(t_x, (Ty * rng.uniform(0.7, 1.0, B)).astype(np.int32))
    mask = O.lengths_mask(B, Tx, Ty, t_x, t_y)
    path, rs, _ = gpu_path(value, mask)
    for b in range(B):
        col = path[b].sum(0)
        assert (col[: t_y[b]] == 1).all() and (col[t_y[b]:] == 0).all()
        assert path[b, 0, 0] == 1 and path[b, t_x[b] - 1, t_y[b] - 1] == 1
        idx = path[b, :, : t_y[b]].argmax(0)
        assert (np.diff(idx) >= 0).all() and (np.diff(idx) <= 1).all()
    for dt in (torch.float16, torch.bfloat16, torch.float64):
        v = torch.from_numpy(value).to(DEV, dt)
        m = torch.from_numpy(mask).to(DEV)
        p = maximum_path(v, m)
        assert p.dtype == dt
        ref, _ = O.maximum_path((v * m).float().cpu().numpy(), mask)
        np.testing.assert_array_equal(p.float().cpu().numpy(), ref)


def test_no_host_sync_and_stream_ordering():
    """maximum_path enqueues on the current stream only: results are right on a side stream."""
    maximum_path, _ = _mp()
    rng = np.random.default_rng(9)
    value = rng.normal(-100.0, 10.0, size=(4, 50, 200)).astype(np.float32)
    mask = O.lengths_mask(4, 50, 200, np.array([50, 40, 30, 20]), np.array([200, 150, 100, 60]))
    exp, _ = O.maximum_path(value, mask)
    s = torch.cuda.Stream()
    v = torch.from_numpy(value).to(DEV)
    m = torch.from_numpy(mask).to(DEV)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        p = maximum_path(v, m)
    s.synchronize()
    np.testing.assert_array_equal(p.cpu().numpy(), exp)


# ---------------------------------------------------------------- fused prior lattice + MAS
@pytest.mark.parametrize("B,C,Tx,Ty", [(4, 80, 13, 37), (3, 80, 64, 65), (2, 80, 200, 1000), (32, 80, 120, 600),
                                       (2, 16, 1, 5), (3, 80, 300, 301)])
def test_prior_maximum_path_vs_oracle(B, C, Tx, Ty):
    """mtts_prior_maximum_path: the masked lattice is bit-identical to the numpy restatement of
    matcha_tts.py:277-282 (oracle/prior_oracle.py), the path bit-identical to the CPU oracle's
    maximum_path on that lattice, durations == path.sum(-1), col_row == the path's row per frame."""
    from matcha.utils.monotonic_align import prior_maximum_path
    from oracle import prior_oracle as PO

    rng = np.random.default_rng(B * 1000 + Tx + Ty)
    mu = rng.normal(0.0, 1.0, size=(B, C, Tx)).astype(np.float32)
    y = rng.normal(0.0, 1.0, size=(B, C, Ty)).astype(np.float32)
    xl = rng.integers(max(1, Tx // 2), Tx + 1, size=B).astype(np.int64)
    yl = np.maximum(rng.integers(max(1, Ty // 2), Ty + 1, size=B), xl).astype(np.int64)
    xl[0], yl[0] = Tx, Ty
    d = lambda a: torch.from_numpy(a).to(DEV)  # noqa: E731
    attn, dur, col_row, rs, lens, lat = prior_maximum_path(d(mu), d(y), d(xl), d(yl), return_lattice=True)
    torch.cuda.synchronize()
    exp_lat, mask = PO.log_prior_lattice(mu, y, xl, yl)
    np.testing.assert_array_equal(lat.cpu().numpy().view(np.uint32), exp_lat.view(np.uint32))
    exp_path, exp_t = O.maximum_path(exp_lat, mask)
    np.testing.assert_array_equal(attn.cpu().numpy(), exp_path)
    np.testing.assert_array_equal(lens.cpu().numpy(), exp_t)
    np.testing.assert_array_equal(dur.cpu().numpy(), PO.durations(exp_path))
    np.testing.assert_array_equal(col_row.cpu().numpy(), PO.col_row(exp_path))
    # without return_lattice the lattice is written transposed for the DP's column-major loads: same outputs
    got = prior_maximum_path(d(mu), d(y), d(xl), d(yl))
    for a, b in zip(got, (attn, dur, col_row, rs, lens)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("Tx,Ty", [(1, 1), (5, 7), (64, 64), (120, 600), (129, 301), (257, 700), (512, 4096),
                                   (1025, 1100), (2049, 2100), (4096, 4100)])
def test_transposed_and_row_major_lattice_agree(Tx, Ty, monkeypatch):
    """maximum_path(value, mask) with the DP on the premasked transposed lattice (default: one coalesced
    transpose, column-major loads) and on the row-major one (MTTS_MAS_TR=0: lane-per-row loads, value * mask
    formed in the DP): identical paths, row starts and lengths, both bit-exact vs the oracle."""
    rng = np.random.default_rng(Tx * 31 + Ty)
    value, t_x, t_y = _rand_case(rng, 3, Tx, Ty, ties=Tx % 2 == 0)
    mask = O.lengths_mask(3, Tx, value.shape[2], t_x, np.maximum(t_y, t_x))
    outs = {}
    for tr in ("1", "0"):
        monkeypatch.setenv("MTTS_MAS_TR", tr)
        outs[tr] = gpu_path(value, mask)
    for a, b in zip(outs["1"], outs["0"]):
        np.testing.assert_array_equal(a, b)
    exp_p, _ = O.maximum_path(value, mask)
    np.testing.assert_array_equal(outs["1"][0], exp_p)


def test_prior_lattice_matches_torch_formula():
    """Against the reference's own formula (matcha_tts.py:277-282 in float64): fp32 rounding only."""
    from matcha.utils.monotonic_align import prior_maximum_path

    g = torch.Generator().manual_seed(5)
    B, C, Tx, Ty = 4, 80, 50, 211
    mu = torch.randn(B, C, Tx, generator=g)
    y = torch.randn(B, C, Ty, generator=g)
    xl = torch.tensor([50, 31, 17, 50])
    yl = torch.tensor([211, 150, 99, 60])
    *_, lat = prior_maximum_path(mu.to(DEV), y.to(DEV), xl.to(DEV), yl.to(DEV), return_lattice=True)
    m, yy = mu.double(), y.double()
    factor = -0.5 * torch.ones_like(m)
    ref = (torch.matmul(factor.transpose(1, 2), yy ** 2) - torch.matmul(2.0 * (factor * m).transpose(1, 2), yy)
           + torch.sum(factor * m ** 2, 1).unsqueeze(-1) - 0.5 * np.log(2 * np.pi) * C)
    am = ((torch.arange(Tx)[None, :, None] < xl[:, None, None]) & (torch.arange(Ty)[None, None, :] < yl[:, None, None]))
    ref = ref * am
    err = (lat.cpu().double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-6, err


def test_expand_rows_matches_bmm_and_its_gradient():
    """mu_y = attn^T @ mu_x as a gather: forward bitwise equal to the bmm on the one-hot attn;
    backward (segment sums) equal to the bmm's gradient in float64 to fp32 rounding."""
    from matcha.utils.monotonic_align import expand_rows, prior_maximum_path

    g = torch.Generator().manual_seed(9)
    B, C, Tx, Ty = 5, 80, 40, 173
    mu = torch.randn(B, C, Tx, generator=g).to(DEV)
    y = torch.randn(B, C, Ty, generator=g).to(DEV)
    xl = torch.tensor([40, 33, 1, 20, 39], device=DEV)
    yl = torch.tensor([173, 100, 7, 20, 140], device=DEV)
    attn, dur, col_row, rs, lens = prior_maximum_path(mu, y, xl, yl)
    a = mu.clone().requires_grad_(True)
    out = expand_rows(a, col_row, rs, lens)
    ref = torch.matmul(attn.transpose(1, 2), mu.transpose(1, 2)).transpose(1, 2)
    assert torch.equal(out, ref)
    gy = torch.randn(B, C, Ty, generator=g).to(DEV)
    (out * gy).sum().backward()
    gref = torch.matmul(gy.double(), attn.double().transpose(1, 2))
    err = (a.grad.double() - gref).abs().max().item() / gref.abs().max().item()
    assert err < 1e-6, err


def test_text_length_limit_is_a_clear_error():
    """Beyond MTTS_MAS_MAX_TX (8192 rows; the reference Cython has no cap) the wrapper refuses with a
    ValueError naming the limit instead of a native shape error; compute_batch_alignments (the row-major
    lattice it mutates) keeps 4096 and says so."""
    import torch

    from matcha.utils.monotonic_align import maximum_path, maximum_path_c

    v = torch.zeros(1, 8193, 8200, device="cuda")
    with pytest.raises(ValueError, match="8192"):
        maximum_path(v, torch.ones_like(v))
    del v
    v = torch.zeros(1, 4097, 4100, device="cuda")
    paths = torch.zeros(1, 4097, 4100, dtype=torch.int32, device="cuda")
    t = torch.tensor([4097], dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError, match="4096"):
        maximum_path_c(paths, v, t, torch.tensor([4100], dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("Tx,Ty", [(4097, 4500), (6000, 6001), (8192, 8192)])
def test_long_text_vs_oracle(Tx, Ty):
    """Round 6: maximum_path beyond 4096 text rows (the multi-wave DP at 16 rows per lane, backpointers in HBM, the
    backtrack from LDS slot copies) is bit-exact with the oracle, ties included."""
    rng = np.random.default_rng(Tx + 3 * Ty)
    for ties in (False, True):
        value, t_x, t_y = _rand_case(rng, 1, Tx, Ty, ties)
        t_x[0], t_y[0] = Tx, Ty
        mask = O.lengths_mask(1, Tx, Ty, t_x, t_y)
        exp_p, _ = O.mas_batch(value, t_x, t_y)
        path, _, _ = gpu_path(value, mask)
        np.testing.assert_array_equal(path, exp_p.astype(np.float32))
