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
