import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def tiny_model_path(tmp_path_factory):
    """A tiny random-init Llama GGUF (exactly quantised) shared by the CPU engine tests."""
    from localai_amd.models import synth
    p = tmp_path_factory.mktemp("models") / "tiny-llama.gguf"
    synth.write_model(str(p), "tiny-llama", exact=True)
    return str(p)


def record_calls(obj, name):
    """Wrap obj.<name> so every call's (args, output) is kept: the production GPU path (graph
    capture, replays) runs unchanged and the test re-runs the same inputs elsewhere."""
    calls = []
    fn = getattr(obj, name)

    def wrapped(*args):
        out = fn(*args)
        def keep(a):
            if isinstance(a, (tuple, list)):
                return type(a)(keep(v) for v in a)
            return a.detach().clone() if hasattr(a, "detach") else a
        calls.append((tuple(keep(a) for a in args), out.detach().clone()))
        return out
    setattr(obj, name, wrapped)
    return calls


def compare_to_fp32(calls, fp32_fn, min_cos=0.999, max_rel=3e-2):
    """Every recorded (bf16 GPU) denoiser call against the same module in fp32 on the CPU, fed the
    same inputs: cosine similarity and relative L2 error of the outputs.  Returns the worst pair."""
    import torch
    worst_cos, worst_rel = 1.0, 0.0
    def to32(a):
        if isinstance(a, (tuple, list)):
            return type(a)(to32(v) for v in a)
        if hasattr(a, "is_floating_point"):
            return a.float().cpu() if a.is_floating_point() else a.cpu()
        return a
    for args, out in calls:
        a32 = tuple(to32(a) for a in args)
        with torch.inference_mode():
            ref = fp32_fn(*a32).float().flatten()
        got = out.float().cpu().flatten()
        worst_cos = min(worst_cos, float(torch.nn.functional.cosine_similarity(got, ref, dim=0)))
        worst_rel = max(worst_rel, float((got - ref).norm() / ref.norm()))
    print(f"denoiser vs fp32: {len(calls)} calls, min cosine {worst_cos:.5f}, max rel-L2 {worst_rel:.4f}")
    assert calls and worst_cos >= min_cos and worst_rel <= max_rel, (worst_cos, worst_rel)
    return worst_cos, worst_rel
