"""The native core (scheduler / paged-KV manager, GBNF automaton, detokenizing stop matcher, HTTP
server) under AddressSanitizer + UndefinedBehaviorSanitizer (the reference runs no
sanitizer at all).  The host-only sanitized build (native/_build.py ASAN_DIR) is loaded in a child
interpreter with the ASan runtime preloaded, and the native test files run against it; any
out-of-bounds access, use-after-free or undefined behaviour aborts the child."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
NATIVE_TESTS = ["tests/test_native_core.py", "tests/test_grammar.py", "tests/test_http_native_protocol.py"]


def _runtime(name: str) -> str:
    r = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else ""


@pytest.mark.timeout(1200)  # includes the sanitized rebuild after a native source change
def test_native_core_under_asan_ubsan():
    asan = _runtime("libasan.so")
    if not asan:
        pytest.skip("no libasan runtime on this host")
    from localai_amd.native import _build
    _build.build_module("_la_core", sanitize=True)  # in this process: the child only loads it
    # libstdc++ right behind the ASan runtime: CPython does not link it, and ASan's __cxa_throw
    # interceptor must resolve the real one at start-up (C++ exceptions -> Python ValueError)
    preload = " ".join(p for p in (asan, _runtime("libstdc++.so.6")) if p)
    env = dict(os.environ, LOCALAI_AMD_NATIVE_ASAN="1", LD_PRELOAD=preload,
               # CPython's own allocations are not instrumented: leak reports would be its noise
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        *NATIVE_TESTS], cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout[-4000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in out and "runtime error" not in out, out
    assert r.returncode == 0, out
    assert " passed" in r.stdout, out
