"""Builds lib/libmtts_hip.so (gfx950 only) from csrc/ with hipcc, in tree.

    python build_native.py [--force] [-j N]

Incremental: an object is rebuilt when its source or a project header it includes (transitively) is newer.
The .so is git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
# MTTS_BUILD_VARIANT=pk: a diagnostic build WITH packed-fp32 VALU ops (lib/libmtts_hip_pk.so, loaded
# only through MTTS_LIB by tools/wgrad_debug.py to reproduce the fault documented in DESIGN.md §9)
VARIANT = os.environ.get("MTTS_BUILD_VARIANT", "")
OBJ = PKG / "build" / ("obj_" + VARIANT if VARIANT else "obj")
LIB = PKG / "lib" / ("libmtts_hip_" + VARIANT + ".so" if VARIANT else "libmtts_hip.so")
ARCH = "gfx950"

# -packed-fp32-ops: no v_pk_{add,mul,fma}_f32 -- a performance choice: beside MFMAs a packed-fp32 VALU
# op costs more issue cycles than two scalar ones (MI355X_MICROARCH.md), the step ran 1.7 % faster.
# Correctness does not depend on it any more: the wgrad fault the flag once masked (v_pk_mul_f32 of
# dY by an op_sel-swapped mask pair) is removed in the source, and the pk variant
# below passes every op test.  The host pass ignores the feature (warning).
COMMON = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
          "-Wall", "-Wno-unused-function"]
if VARIANT != "pk":
    COMMON += ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
# Per-file extra flags.  The MAS DP must not contract value*mask + best into an FMA (bit parity with
# the Cython, core.pyx:80 / __init__.py:45).
EXTRA = {
    "mas.hip": ["-ffp-contract=off"],
    "cfm_prep.hip": ["-ffp-contract=off"],  # phi_t and the time embedding round like torch (no fma)
    "losses.hip": ["-ffp-contract=off"],  # u = x1 - (1 - sigma) z and the prior term: torch's roundings
}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (need ROCm with gfx950 support)")


def sources() -> list[Path]:
    return sorted([p for p in CSRC.iterdir() if p.suffix in (".hip", ".cpp")])


def _deps(src: Path, seen: set | None = None) -> set:
    """The project headers `src` includes, transitively (#include "..." found in csrc/ or include/)."""
    seen = set() if seen is None else seen
    for line in src.read_text(errors="ignore").splitlines():
        line = line.strip()
        if line.startswith("#include \""):
            name = line.split('"')[1]
            for d in (CSRC, INCLUDE):
                h = d / name
                if h.exists() and h not in seen:
                    seen.add(h)
                    _deps(h, seen)
                    break
    return seen


def _newest_header(src: Path) -> float:
    return max((h.stat().st_mtime for h in _deps(src)), default=0.0)


def _compile(src: Path, force: bool) -> Path:
    obj = OBJ / (src.name + ".o")
    if not force and obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, _newest_header(src)):
        return obj
    lang = ["-x", "hip"] if src.suffix == ".hip" else ["-x", "hip"]
    cmd = [_hipcc(), *COMMON, *EXTRA.get(src.name, []), *os.environ.get("MTTS_EXTRA_HIPCC_FLAGS", "").split(),
           *lang, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    LIB.parent.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, len(srcs))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        tmp = LIB.with_suffix(".so.tmp")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs), "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    args = ap.parse_args()
    try:
        print(build(args.force, args.j))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
