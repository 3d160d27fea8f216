"""GGUF container + quantisation formats (reference: llama.cpp's gguf/ggml-quants as used by
backend/cpp/llama; parity pinned by round-trip error bounds)."""
import numpy as np
import pytest

from localai_amd import gguf
from localai_amd.gguf import GGMLType


def test_writer_reader_roundtrip(tmp_path):
    p = str(tmp_path / "m.gguf")
    w = gguf.GGUFWriter(p, "llama")
    w.add_string("general.name", "t")
    w.add_uint32("llama.block_count", 2)
    w.add_float32("llama.attention.layer_norm_rms_epsilon", 1e-5)
    w.add_bool("x.flag", True)
    w.add_array("tokenizer.ggml.tokens", ["a", "b", "c"], gguf.GGUFValueType.STRING)
    a = np.arange(64 * 3, dtype=np.float32).reshape(3, 64)
    w.add_tensor("w", a.shape, GGMLType.F32, gguf.quantize(a, GGMLType.F32))
    w.write()
    r = gguf.GGUFReader(p)
    assert r.architecture == "llama"
    assert r.kv["general.name"] == "t"
    assert r.kv["llama.block_count"] == 2
    assert abs(r.kv["llama.attention.layer_norm_rms_epsilon"] - 1e-5) < 1e-9
    assert r.kv["x.flag"] is True
    assert list(r.kv["tokenizer.ggml.tokens"]) == ["a", "b", "c"]
    t = r.tensors["w"]
    assert tuple(t.shape) == (3, 64)
    np.testing.assert_array_equal(gguf.dequantize(t.data, t.ggml_type, t.shape), a)


@pytest.mark.parametrize("t,tol", [(GGMLType.Q8_0, 0.01), (GGMLType.Q6_K, 0.03), (GGMLType.Q4_K, 0.12)])
def test_quant_roundtrip(t, tol):
    rng = np.random.default_rng(0)
    w = rng.standard_normal((8, 512)).astype(np.float32)
    raw = gguf.quantize(w, t)
    assert raw.nbytes == 8 * 512 // gguf.GGML_BLOCK[t][0] * gguf.GGML_BLOCK[t][1]
    d = gguf.dequantize(raw, t, w.shape)
    rel = np.sqrt(((d - w) ** 2).mean() / (w ** 2).mean())
    assert rel < tol, rel


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0])
def test_random_blocks_have_target_std(t):
    fn = {GGMLType.Q4_K: gguf.random_q4_k_blocks, GGMLType.Q6_K: gguf.random_q6_k_blocks,
          GGMLType.Q8_0: gguf.random_q8_0_blocks}[t]
    raw = fn(np.random.default_rng(1), 64 * 1024 // gguf.GGML_BLOCK[t][0], 0.02)
    d = gguf.dequantize(raw, t, (64, 1024))
    assert np.isfinite(d).all()
    assert 0.005 < d.std() < 0.08


def test_deepseek_v3_gating_is_refused(tmp_path):
    """deepseek2 GGUFs carrying V3/R1 sigmoid gating load with a clear error, not wrong routing."""
    from localai_amd.gguf import GGUFReader
    from localai_amd.models import synth
    from localai_amd.models.hparams import HParams
    p = tmp_path / "ds.gguf"
    synth.write_model(str(p), "tiny-deepseek2")
    r = GGUFReader(str(p))
    HParams.from_gguf(r)                      # V2 softmax routing loads
    r.kv["deepseek2.expert_gating_func"] = 2  # V3 / R1: sigmoid
    with pytest.raises(ValueError, match="sigmoid"):
        HParams.from_gguf(r)
