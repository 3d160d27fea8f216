"""Build the native engine core (`_la_core*.so`, C++17 + pybind11) in-tree with g++."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
# module name -> sources
MODULES = {"_la_core": ["engine_core.cpp", "grammar.cpp", "http_server.cpp"]}
HEADERS = ["text_stream.h"]
LIB = HERE / f"_la_core{EXT}"


def _digest(srcs) -> str:
    h = hashlib.sha256()
    for p in srcs:
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False, sanitize: bool = False) -> Path:
    for name in MODULES:
        build_module(name, force, verbose, sanitize)
    return LIB


# AddressSanitizer + UndefinedBehaviorSanitizer build of the native core (host code only), kept apart
# from the production module: tests/test_native_sanitizers.py reruns the native test files against it
# in a child interpreter with the ASan runtime preloaded
ASAN_DIR = HERE / "_asan"


def build_module(name: str, force: bool = False, verbose: bool = False, sanitize: bool = False) -> Path:
    SRCS = [HERE / s for s in MODULES[name]]
    out_dir = ASAN_DIR if sanitize else HERE
    out_dir.mkdir(exist_ok=True)
    LIB = out_dir / f"{name}{EXT}"
    stamp = out_dir / f"{name}.stamp"
    dig = _digest(SRCS + [HERE / h for h in HEADERS]) + ("-asan" if sanitize else "")
    if not force and LIB.exists() and stamp.exists() and stamp.read_text().strip() == dig:
        return LIB
    import pybind11
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-sign-compare",
             f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    if sanitize:
        flags = [f for f in flags if f != "-O2"] + ["-O1", "-fsanitize=address,undefined",
                                                    "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g"]
    tmp = str(LIB) + ".tmp"
    cmd = [cxx, *flags, *map(str, SRCS), "-o", tmp, "-lpthread"]
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
