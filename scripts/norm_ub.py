"""Upper bound of fusing add_norm into the decode GEMVs: bench.py (engine mode) with every
add_norm of a 1-2 row batch replaced by a no-op returning a cached tensor (WRONG numerics; timing
only).  Usage: python scripts/norm_ub.py --mode engine --concurrency 1 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402

_real = ops.add_norm
_cache = {}


def fake(residual, add, weight, bias, eps, mode=0, out=None, want_out=True):
    T, D = residual.shape
    if T > 2 or not residual.is_cuda:
        return _real(residual, add, weight, bias, eps, mode, out, want_out)
    key = (T, D, residual.device)
    if key not in _cache:
        _cache[key] = _real(residual, add, weight, bias, eps, mode, None, True)
    return _cache[key] if want_out else None


ops.add_norm = fake
import bench  # noqa: E402

bench.main()
