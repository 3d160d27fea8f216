"""LoRA adapters (model-config lora_adapter / lora_base / lora_scale; grpc-server.cpp:2263-2271):
llama.cpp's GGUF adapter layout, alpha / rank scaling, merge into the base weights at load, the
engine's greedy output against the fp32 oracle of the merged model, and the gRPC option mapping."""
import types

import numpy as np
import pytest
import torch

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.gguf import GGUFReader, dequantize
from localai_amd.models import synth
from localai_amd.models.lora import LoraSet, adapter_path


@pytest.fixture(scope="module")
def model_and_lora(tmp_path_factory):
    d = tmp_path_factory.mktemp("lora")
    base = synth.write_model(str(d / "base.gguf"), "tiny-llama", exact=True)
    ad = synth.write_lora(str(d / "adapter.gguf"), base, targets=("attn_q", "ffn_down"), rank=4, alpha=8.0,
                          std=0.2)
    return base, ad


def test_adapter_parse_and_merge(model_and_lora):
    base, ad = model_and_lora
    ls = LoraSet([(ad, 0.5)])
    assert "blk.0.attn_q.weight" in ls and "blk.1.ffn_down.weight" in ls and "blk.0.attn_k.weight" not in ls
    r = GGUFReader(ad)
    t = GGUFReader(base).tensors["blk.1.ffn_down.weight"]
    w = dequantize(t.data, t.ggml_type, t.shape).reshape(t.shape)
    a = np.frombuffer(r.tensors["blk.1.ffn_down.weight.lora_a"].data, dtype=np.float32).reshape(4, -1)
    b = np.frombuffer(r.tensors["blk.1.ffn_down.weight.lora_b"].data, dtype=np.float32).reshape(-1, 4)
    want = w + 0.5 * 8.0 / 4 * (b @ a)
    assert np.abs(ls.merged("blk.1.ffn_down.weight", w) - want).max() < 1e-5


def test_engine_with_adapter_matches_merged_oracle(model_and_lora):
    base, ad = model_and_lora
    plain = LLMEngine(EngineConfig(model_path=base, device="cpu", context_size=256, max_num_seqs=4, use_graphs=False))
    eng = LLMEngine(EngineConfig(model_path=base, device="cpu", context_size=256, max_num_seqs=4, use_graphs=False,
                                 lora_adapters=((ad, 1.0),)))
    ids = eng.tokenize("adapter check")
    ref = eng.model.reference_logits(ids)[-1]
    ref0 = plain.model.reference_logits(ids)[-1]
    assert float((ref - ref0).abs().max()) > 1e-2  # the adapter changes the model
    # the merged q weight is the base weight plus the scaled delta (BF16-rounded)
    t = eng.reader.tensors["blk.0.attn_q.weight"]
    wq = dequantize(t.data, t.ggml_type, t.shape).reshape(t.shape)
    ls = LoraSet([(ad, 1.0)])
    got = eng.model.layers[0].qkv[0].dequant_f32()[: wq.shape[0]].numpy()
    assert np.abs(got - ls.merged("blk.0.attn_q.weight", wq)).max() < 2e-2
    res = eng.generate("adapter check", SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    first = eng.tokenize("adapter check" + res["text"])[len(ids)]
    top = torch.topk(ref, 2)
    assert first == int(top.indices[0]) or float(top.values[0] - ref[first]) < 0.05


def test_grpc_lora_mapping(tmp_path):
    from localai_amd.grpc.servicer import EngineServicer as BackendServicer
    mp = str(tmp_path / "m" / "model.gguf")
    req = types.SimpleNamespace(LoraAdapter="ad.gguf", LoraBase="base", LoraScale=0.0)
    assert BackendServicer._lora(req, mp) == ((str(tmp_path / "m" / "ad.gguf"), 1.0),)
    req.LoraScale = 0.25
    assert BackendServicer._lora(req, mp)[0][1] == 0.25
    req.LoraBase = ""  # the reference applies an adapter only with lora_base set
    assert BackendServicer._lora(req, mp) == ()
    assert adapter_path(mp, "/abs/x.gguf") == "/abs/x.gguf"


def test_non_adapter_gguf_rejected(model_and_lora):
    base, _ = model_and_lora
    with pytest.raises(ValueError):
        LoraSet([(base, 1.0)])
