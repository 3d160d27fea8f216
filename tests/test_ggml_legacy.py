"""Pre-GGUF ggjt v3 files (the reference's llama-ggml backend): the same tensors in a ggjt container
give the same model as the GGUF they came from -- vocabulary, hyper-parameters, logits, greedy text."""
import pytest
import torch

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.models import synth
from localai_amd.models.ggml_legacy import GGJTReader, is_ggjt, write_ggjt


def _engine(p):
    return LLMEngine(EngineConfig(model_path=p, device="cpu", context_size=256, max_num_seqs=2, use_graphs=False))


def test_ggjt_matches_gguf(tmp_path):
    gg = str(tmp_path / "m.gguf")
    # ggjt files carry no RoPE base or RMS epsilon: use the values llama.cpp assumed for them
    synth.write_model(gg, "tiny-llama", exact=True, tokenizer="mistral", n_vocab=2048, rope_theta=10000.0, eps=5e-6)
    gj = write_ggjt(str(tmp_path / "m.ggjt.bin"), gg)
    assert is_ggjt(gj) and not is_ggjt(gg)
    r = GGJTReader(gj)
    assert r.kv["llama.attention.head_count_kv"] == 2 and r.kv["llama.feed_forward_length"] == 512
    a, b = _engine(gg), _engine(gj)
    text = "the quick brown fox jumps over the lazy dog"
    ids = a.tokenize(text)
    assert b.tokenize(text) == ids
    la, lb = a.model.reference_logits(ids), b.model.reference_logits(ids)
    assert float((la - lb).abs().max() / la.abs().max()) < 1e-6  # same tensor bytes, same model
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    assert a.generate(text, sp)["completion_tokens"] == b.generate(text, sp)["completion_tokens"] == 6


def test_ggjt_old_versions_refused(tmp_path):
    import struct
    p = tmp_path / "old.bin"
    p.write_bytes(struct.pack("<II", 0x67676A74, 1) + b"\0" * 64)
    with pytest.raises(ValueError, match="pre-v3"):
        GGJTReader(str(p))


def test_llama_ggml_backend_through_gateway(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    mdir.mkdir()
    gg = str(tmp_path / "m.gguf")
    synth.write_model(gg, "tiny-llama", exact=True, tokenizer="mistral", n_vocab=2048)
    write_ggjt(str(mdir / "old-model.ggmlv3.q8_0.bin"), gg)
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    ac.engine_mode = "inprocess"
    st = AppState(ac)
    bc = BackendConfig({"name": "old", "backend": "llama-ggml", "context_size": 256,
                        "parameters": {"model": "old-model.ggmlv3.q8_0.bin", "temperature": 0}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/completions", json={"model": "old", "prompt": "hello", "max_tokens": 3, "ignore_eos": True})
        assert r.status_code == 200, r.text
        assert r.json()["usage"]["completion_tokens"] == 3
