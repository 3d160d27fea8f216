"""Build the native engine core (`_la_core*.so`, C++17 + pybind11) in-tree with g++."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRCS = sorted(HERE.glob("*.cpp"))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
LIB = HERE / f"_la_core{EXT}"


def _digest() -> str:
    h = hashlib.sha256()
    for p in SRCS:
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False, sanitize: bool = False) -> Path:
    stamp = HERE / "_la_core.stamp"
    dig = _digest() + ("-asan" if sanitize else "")
    if not force and LIB.exists() and stamp.exists() and stamp.read_text().strip() == dig:
        return LIB
    import pybind11
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-sign-compare",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    if sanitize:
        flags += ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
    tmp = str(LIB) + ".tmp"
    cmd = [cxx, *flags, *map(str, SRCS), "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, LIB)
    stamp.write_text(dig)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, sanitize="--asan" in sys.argv))
