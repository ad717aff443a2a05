"""Fast-iteration harness for the multi-wave MAS DP (csrc/mas.hip mas_dp_mw_kernel, transposed premasked lattice):
extracts the kernel and its helpers from mas.hip into a small HIP file with a launcher (seconds to build instead of
the ~20 minutes of the whole mas.hip), runs it on random lattices, checks the row starts bit for bit against the
C oracle (oracle/mas_oracle.c, the checker) and times it; MTTS_MAS_STAMPS splits the time into forward DP and
backtrack per utterance.

build (here):   python tools/r6/mas_probe.py build            -> tools/r6/_mas_probe.so (git-ignored)
run (GPU box):  python tools/r6/mas_probe.py run [--configs 8x512x4096,...] [--iters 20]"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent.parent
CSRC = ROOT / "matcha-tts-etu-upmc-ensam_amd" / "csrc"
SO = Path(__file__).resolve().parent / "_mas_probe.so"

LAUNCHER = r'''
}  // namespace
template <int KL>
static void go(MasArgs a, int B, size_t shmem, hipStream_t st) {
    auto k = mas_dp_mw_kernel<KL, 8, true, false, false, false, true>;
    if (shmem > 64 * 1024) hipFuncSetAttribute(reinterpret_cast<const void *>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
    hipLaunchKernelGGL(k, dim3(B), dim3(512), shmem, st, a);
}
extern "C" int probe_mw(const float *lat, const int *txs, const int *tys, int *lengths, int *row_start, unsigned *bits,
                        int B, int Tx, int Ty, int Txp, int nch, float neg, void *stream) {
    MasArgs a{};
    a.value = lat; a.t_xs = txs; a.t_ys = tys; a.lengths = lengths; a.row_start = row_start; a.bits = bits;
    a.Tx = Tx; a.Ty = Ty; a.Txp = Txp; a.nch = nch; a.premasked = 1; a.neg = neg; a.tr_ld = Txp;
    const size_t shmem = mw_backtrack_bufs(a, (size_t)Txp * 4 + (size_t)kEdgeRing * 8 * 32 * 4);
    hipStream_t st = (hipStream_t)stream;
    const int KL = Txp / 512;
    if (KL == 1) go<1>(a, B, shmem, st); else if (KL == 2) go<2>(a, B, shmem, st);
    else if (KL == 4) go<4>(a, B, shmem, st); else if (KL == 8) go<8>(a, B, shmem, st); else go<16>(a, B, shmem, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
extern "C" int probe_stamps(long long *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(mas_probe_stamps), sizeof(long long) * 4 * n) == hipSuccess ? 0 : -1;
}
'''


def build(so=SO):
    src = (CSRC / "mas.hip").read_text().splitlines(keepends=True)
    h = next(i for i, l in enumerate(src) if l.startswith("template <int K, int C, int D, bool PM, bool VEC, bool LDS_BITS"))
    s = next(i for i, l in enumerate(src) if l.startswith("// MTTS_MAS_STAMPS"))
    e = next(i for i, l in enumerate(src) if l.startswith("// Dense writer"))
    m0 = next(i for i, l in enumerate(src) if l.startswith("// dynamic LDS past 64 KiB"))
    m1 = next(i for i, l in enumerate(src) if l.startswith("size_t mw_backtrack_bufs"))
    m2 = next(i for i in range(m1, len(src)) if src[i].startswith("}"))
    out = Path("/tmp/mas_probe.hip")
    out.write_text("#define MTTS_MAS_STAMPS 1\n" + "".join(src[:h]) + "".join(src[s:e]) + "".join(src[m0:m2 + 1]) + LAUNCHER)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", f"-I{ROOT / 'include'}",
           f"-I{CSRC}", "-ffp-contract=off", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", str(out), "-o", str(so)]
    subprocess.run(cmd, check=True)
    print(so)


def run(configs, iters, so=SO):
    import numpy as np
    import torch

    sys.path[:0] = [str(ROOT / "tests"), str(ROOT)]
    import oracle_bind as OB

    lib = ctypes.CDLL(str(so))
    P = ctypes.c_void_p
    lib.probe_mw.argtypes = [P, P, P, P, P, P] + [ctypes.c_int] * 5 + [ctypes.c_float, P]
    lib.probe_stamps.argtypes = [P, ctypes.c_int]
    neg = -1e9
    for cfg in configs:
        B, Tx, Ty = map(int, cfg.split("x"))
        Txp = max(512, 1 << (Tx - 1).bit_length())  # 64 lanes x 8 waves x KL rows
        nch = (Ty + 31) // 32
        rng = np.random.default_rng(B + Tx + Ty)
        t_x = np.maximum(1, (Tx * rng.uniform(0.7, 1.0, B)).astype(np.int32)); t_x[0] = Tx
        t_y = np.maximum(t_x, (Ty * rng.uniform(0.7, 1.0, B)).astype(np.int32)); t_y[0] = Ty
        value = rng.normal(-100.0, 10.0, size=(B, Tx, Ty)).astype(np.float32)
        mask = np.zeros_like(value)
        for b in range(B):
            mask[b, : t_x[b], : t_y[b]] = 1
        pm = value * mask
        lat = np.zeros((B, Ty, Txp), np.float32)
        lat[:, :, :Tx] = pm.transpose(0, 2, 1)
        d = torch.device("cuda")
        g_lat = torch.from_numpy(lat).to(d)
        g_tx, g_ty = torch.from_numpy(t_x).to(d), torch.from_numpy(t_y).to(d)
        g_len = torch.zeros(B, 2, dtype=torch.int32, device=d)
        g_rs = torch.full((B, Tx), -7, dtype=torch.int32, device=d)
        g_bits = torch.zeros(B * nch * Txp, dtype=torch.int32, device=d)
        st = torch.cuda.current_stream().cuda_stream
        args = (g_lat.data_ptr(), g_tx.data_ptr(), g_ty.data_ptr(), g_len.data_ptr(), g_rs.data_ptr(), g_bits.data_ptr(),
                B, Tx, Ty, Txp, nch, ctypes.c_float(neg), st)
        assert lib.probe_mw(*args) == 0
        torch.cuda.synchronize()
        path, _ = OB.maximum_path(value, mask)
        want = np.full((B, Tx), -1, np.int32)
        for b in range(B):
            for x in range(t_x[b]):
                ys = np.nonzero(path[b, x])[0]
                want[b, x] = ys[0] if len(ys) else -1
        got = g_rs.cpu().numpy()
        exact = bool(np.array_equal(np.where(want >= 0, got, -1), want))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            lib.probe_mw(*args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        stamps = np.zeros(4 * B, np.int64)
        assert lib.probe_stamps(stamps.ctypes.data, B) == 0
        s = stamps.reshape(B, 4)
        dp_us = (s[:, 1] - s[:, 0]) * 0.01
        bt_us = (s[:, 2] - s[:, 1]) * 0.01
        print(json.dumps({"so": Path(so).name, "config": cfg, "bit_exact_row_starts": exact, "kernel_ms": round(ms, 4),
                          "dp_us_max": round(float(dp_us.max()), 1), "backtrack_us_max": round(float(bt_us.max()), 1),
                          "dp_ns_per_column_b0": round(float(dp_us[0]) * 1e3 / Ty, 1)}), flush=True)


if __name__ == "__main__":
    so = SO
    for i, x in enumerate(sys.argv):
        if x == "--so":
            so = Path(sys.argv[i + 1])
    if sys.argv[1] == "build":
        build(so)
    else:
        cfgs = "8x512x4096,8x1024x4096"
        iters = 20
        for i, x in enumerate(sys.argv):
            if x == "--configs":
                cfgs = sys.argv[i + 1]
            if x == "--iters":
                iters = int(sys.argv[i + 1])
        run(cfgs.split(","), iters, so)
