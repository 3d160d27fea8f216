"""Native (C++/pybind11) runtime: engine core (scheduler, paged-KV manager, detokenizing
stop matcher) and the HTTP/1.1 front end with SSE token sinks.  Built in-tree on first import."""
from . import _build

try:
    from . import _la_core as core  # noqa: F401
except ImportError:
    _build.build_module("_la_core")
    from . import _la_core as core  # noqa: F401


def http():
    """The HTTP server / SSE sink classes (compiled into the same module as the engine core, so
    the engine's native token emitter can drive the sinks directly)."""
    return core
