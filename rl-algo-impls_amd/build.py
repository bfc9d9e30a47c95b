"""Build recipe for the gfx950 C-ABI library (librai_amd.so).

hipcc cross-compiles every csrc/*.hip for --offload-arch=gfx950 and links one
shared library into lib/ in-tree (the .so travels to the GPU box with the repo
snapshot; nothing is installed into site-packages).  Runs on a CPU-only host.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = PKG / "build" / "obj"
LIBNAME = "librai_amd.so"
ARCH = os.environ.get("RAI_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

COMMON_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-Wall",
    "-Wno-unused-function",
    "-munsafe-fp-atomics",
]
# Files whose numerics must follow the reference's rounding sequence exactly.
NO_CONTRACT = {"gae.hip", "gae_traj.hip", "optim.hip", "loss.hip"}


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def lib_path(variant: str = "") -> Path:
    if variant:
        return LIBDIR / LIBNAME.replace(".so", f"_{variant}.so")
    override = os.environ.get("RAI_AMD_LIB")
    return Path(override) if override else LIBDIR / LIBNAME


# "alt": an A/B build of the same sources with extra -D flags from RAI_ALT_FLAGS (tools/ab_bench.sh;
# diagnostic, never loaded by the product)
VARIANT_FLAGS = {"": [], "stamps": ["-DRAI_STAMPS"], "alt": os.environ.get("RAI_ALT_FLAGS", "").split()}


def _compile(src: Path, variant: str = "") -> Path:
    objdir = OBJDIR if not variant else OBJDIR.parent / f"obj_{variant}"
    objdir.mkdir(parents=True, exist_ok=True)
    obj = objdir / (src.stem + ".o")
    deps = [src, CSRC / "common.h", PKG.parent / "include" / "rai_amd.h"]
    deps += list(CSRC.glob("*.h"))
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps if d.exists()):
        return obj
    flags = list(COMMON_FLAGS) + VARIANT_FLAGS[variant]
    if src.name in NO_CONTRACT:
        flags.append("-ffp-contract=off")
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


def build(verbose: bool = False, variant: str = "") -> Path:
    """Build librai_amd.so (variant "" = the shipped library; "stamps" = the per-phase
    cycle-stamp diagnostic build, lib/librai_amd_stamps.so, never loaded by the product)."""
    OBJDIR.mkdir(parents=True, exist_ok=True)
    LIBDIR.mkdir(parents=True, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, variant), srcs))
    out = lib_path(variant) if variant else LIBDIR / LIBNAME
    if out.exists() and out.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return out
    tmp = out.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *map(str, objs), "-o", str(tmp),
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    if verbose:
        print(f"built {out}")
    return out


if __name__ == "__main__":
    print(build(verbose=True, variant=sys.argv[1] if len(sys.argv) > 1 else ""))
