"""In-tree build of the gfx950 kernel library (`_la_kernels.so`).

Plain hipcc, no hipify, no torch headers: the kernels expose a C ABI that
`localai_amd.ops` binds with ctypes.  The library links against the HIP runtime that
PyTorch-ROCm itself loaded (same soname, torch/lib first on the rpath), so a process
never carries two HIP runtimes.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB = HERE / "_la_kernels.so"
ARCH = os.environ.get("LOCALAI_AMD_ARCH", "gfx950")


def _torch_lib() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return str(Path(spec.origin).parent / "lib")


# per-file hipcc flags: the prefill GEMM's dequant runs beside MFMAs, where the packed
# v_pk_fma_f32 the SLP vectoriser forms issues slower than two scalar FMAs (profiles/r5_prefill_gemm.md)
FILE_FLAGS = {"gemm_bs.hip": ["-fno-slp-vectorize"]}


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _digest() -> str:
    h = hashlib.sha256()
    for p in sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.h"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(ARCH.encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def _hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    return "hipcc"


def build(force: bool = False, verbose: bool = False, jobs: int = 8) -> Path:
    return _build_lib(LIB, [], force, verbose, jobs)


def build_variant(name: str, defines, verbose: bool = False, jobs: int = 8) -> Path:
    """An A/B build of the same sources with extra -D flags into ops/<name> (selected at run time
    by LOCALAI_AMD_KLIB=<name>), e.g. build_variant("_la_kernels_wnt.so", ["LA_W_AUX=2"])."""
    return _build_lib(HERE / name, list(defines), False, verbose, jobs)


def _build_lib(LIB: Path, defines, force: bool, verbose: bool, jobs: int) -> Path:
    stamp = LIB.with_suffix(".stamp")
    dig = _digest() + ("".join(defines) if defines else "")
    if not force and LIB.exists() and stamp.exists() and stamp.read_text().strip() == dig:
        return LIB
    objdir = HERE / ("build" if not defines else "build_" + LIB.stem)
    objdir.mkdir(exist_ok=True)
    flags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wno-unused-result",
             "-I", str(CSRC)] + [f"-D{d}" for d in defines]

    def compile_one(src: Path) -> Path:
        obj = objdir / (src.stem + ".o")
        cmd = [_hipcc(), *flags, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, _sources()))
    tl = _torch_lib()
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
           f"-L{tl}", "-l:libamdhip64.so", f"-Wl,-rpath,{tl}"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    stamp.write_text(dig)
    return LIB


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
