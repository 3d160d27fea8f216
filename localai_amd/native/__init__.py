"""Native (C++/pybind11) engine core.  Built in-tree on first import."""
from . import _build

try:
    from . import _la_core as core  # noqa: F401
except ImportError:
    _build.build()
    from . import _la_core as core  # noqa: F401
