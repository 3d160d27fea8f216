"""Native (C++/pybind11) runtime: engine core (scheduler, paged-KV manager, detokenizing
stop matcher) and the HTTP/1.1 front end with SSE token sinks.  Built in-tree on first import."""
import os

from . import _build

if os.environ.get("LOCALAI_AMD_NATIVE_ASAN") == "1":
    # sanitizer runs only (tests/test_native_sanitizers.py): the ASan/UBSan build, loaded under
    # the module's own name from its separate directory; the ASan runtime must be preloaded
    import importlib.util

    _p = _build.build_module("_la_core", sanitize=True)
    _spec = importlib.util.spec_from_file_location("localai_amd.native._la_core", _p)
    core = importlib.util.module_from_spec(_spec)
    _spec.loader.exec_module(core)
else:
    try:
        from . import _la_core as core  # noqa: F401
    except ImportError:
        _build.build_module("_la_core")
        from . import _la_core as core  # noqa: F401


def http():
    """The HTTP server / SSE sink classes (compiled into the same module as the engine core, so
    the engine's native token emitter can drive the sinks directly)."""
    return core
