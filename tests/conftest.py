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
