"""HF checkpoint directories served by the engine (the reference's vllm / transformers backends load
these): logits of the engine's fp32 reference forward vs `transformers`' own forward of the same
random-init checkpoint (an independent oracle), tokenizer ids vs the library's fast tokenizer,
greedy generation through the engine, and the gateway's `use_tokenizer_template` path."""
import pytest
import torch

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.models import synth
from localai_amd.models.hf_checkpoint import HFCheckpointReader, is_hf_checkpoint

TEXT = "The quick brown fox jumps over the lazy dog, then runs 123 miles!"

CASES = {
    "llama": dict(kind="llama"),
    "llama31_rope": dict(kind="llama", rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                                     "high_freq_factor": 4.0,
                                                     "original_max_position_embeddings": 64}),
    "mistral": dict(kind="mistral"),
    "qwen2": dict(kind="qwen2"),
    "mixtral": dict(kind="mixtral", n_experts=4),
}


@pytest.fixture(scope="module", params=sorted(CASES))
def ckpt(request, tmp_path_factory):
    d = str(tmp_path_factory.mktemp("hf") / request.param)
    synth.write_hf_checkpoint(d, **CASES[request.param])
    return request.param, d


def _hf_logits(d, ids):
    import transformers as tf
    m = tf.AutoModelForCausalLM.from_pretrained(d, torch_dtype=torch.float32)
    m.eval()
    with torch.no_grad():
        return m(torch.tensor([ids])).logits[0].float()


def test_logits_match_transformers(ckpt):
    name, d = ckpt
    assert is_hf_checkpoint(d)
    e = LLMEngine(EngineConfig(model_path=d, device="cpu", context_size=256, max_num_seqs=4, use_graphs=False))
    ids = e.tokenize(TEXT)
    assert len(ids) > 10
    ours = e.model.reference_logits(ids).float()
    ref = _hf_logits(d, ids)
    assert ours.shape == ref.shape
    err = float((ours - ref).abs().max() / ref.abs().max())
    assert err < 2e-3, f"{name}: rel err {err}"
    # greedy generation through the engine continues with the oracle's argmax
    r = e.generate(TEXT, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    top = torch.topk(ref[-1], 2)
    if float(top.values[0] - top.values[1]) > 1e-3:
        assert r["text"] == e.tokenizer.decode([int(top.indices[0])])


def test_tokenizer_matches_fast_tokenizer(tmp_path):
    import transformers as tf
    d = synth.write_hf_checkpoint(str(tmp_path / "tok"), kind="llama", n_layer=1)
    fast = tf.PreTrainedTokenizerFast(tokenizer_file=f"{d}/tokenizer.json")
    r = HFCheckpointReader(d)
    from localai_amd.tokenizer import Tokenizer
    ours = Tokenizer.from_gguf(r)
    for s in (TEXT, "  leading spaces\nand\ttabs", "<|start_header_id|>user<|end_header_id|>\n\nhi<|eot_id|>",
              "naïve café — ünïcödé 😀"):
        want = fast(s, add_special_tokens=False)["input_ids"]
        assert ours.encode(s, add_bos=False) == want, s
        assert ours.decode(want) == fast.decode(want, skip_special_tokens=True)  # control tokens render empty
    assert ours.add_bos and ours.bos_id == r.kv["tokenizer.ggml.bos_token_id"]
    assert "<|eot_id|>" in ours.tokens and ours.is_eog(ours.vocab["<|eot_id|>"]) or ours.eos_id == ours.vocab["<|eot_id|>"]


def test_unsupported_architecture(tmp_path):
    import json
    (tmp_path / "config.json").write_text(json.dumps({"architectures": ["GPT2LMHeadModel"]}))
    (tmp_path / "model.safetensors").write_bytes(b"")
    with pytest.raises(ValueError, match="unsupported HF architecture"):
        HFCheckpointReader(str(tmp_path))


def test_gateway_vllm_backend_with_tokenizer_template(tmp_path):
    """A model config the way the reference's vllm gallery entries write it (backend: vllm,
    use_tokenizer_template) pointing at a checkpoint directory."""
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    synth.write_hf_checkpoint(str(mdir / "tiny-llama-hf"), kind="llama", n_layer=1)
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    ac.engine_mode = "inprocess"
    st = AppState(ac)
    bc = BackendConfig({"name": "hf-llama", "backend": "vllm", "context_size": 256,
                        "parameters": {"model": "tiny-llama-hf", "temperature": 0},
                        "template": {"use_tokenizer_template": True}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/chat/completions", json={"model": "hf-llama", "max_tokens": 4, "ignore_eos": True,
                                                 "messages": [{"role": "user", "content": "hello there"}]})
        assert r.status_code == 200, r.text
        u = r.json()["usage"]
        assert u["completion_tokens"] == 4 and u["prompt_tokens"] > 5


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["llama", "qwen2"])
def test_hf_checkpoint_on_gpu(tmp_path, kind):
    """bf16 HF checkpoint served by the HIP engine (graph decode): its greedy tokens follow the
    transformers fp32 oracle wherever the oracle's top-2 margin exceeds the bf16 noise."""
    d = synth.write_hf_checkpoint(str(tmp_path / kind), kind=kind, n_layer=2, hidden=256, heads=4, kv_heads=2,
                                  ffn=512, dtype="bfloat16")
    e = LLMEngine(EngineConfig(model_path=d, device="cuda:0", context_size=256, max_num_seqs=4,
                               max_batched_tokens=256, block_size=32))
    ids = e.tokenize(TEXT)
    res = e.generate(TEXT, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert res["completion_tokens"] == 4
    ref = _hf_logits(d, ids)[-1]
    top = torch.topk(ref, 2)
    if float(top.values[0] - top.values[1]) > 0.05 * float(ref.abs().max()):
        assert res["text"].startswith(e.tokenizer.decode([int(top.indices[0])]))


@pytest.mark.parametrize("act_order", [False, True])
def test_gptq_checkpoint(tmp_path, act_order):
    """autogptq backend: a GPTQ checkpoint (4-bit, groups of 32, optionally act-order) loads with
    the same logits as the float model holding its dequantised weights (transformers oracle)."""
    src = synth.write_hf_checkpoint(str(tmp_path / "src"), kind="llama", n_layer=2)
    q = synth.gptq_quantize_checkpoint(src, str(tmp_path / "gptq"), str(tmp_path / "oracle"), act_order=act_order)
    e = LLMEngine(EngineConfig(model_path=q, device="cpu", context_size=256, max_num_seqs=2, use_graphs=False))
    ids = e.tokenize(TEXT)
    ours = e.model.reference_logits(ids).float()
    ref = _hf_logits(str(tmp_path / "oracle"), ids)
    err = float((ours - ref).abs().max() / ref.abs().max())
    assert err < 3e-3, err  # the loader rounds dequantised weights to f16


@pytest.mark.parametrize("mode,types", [("bnb_4bit", {"attn_q": 12, "ffn_down": 14, "output": 14, "attn_v": 14}),
                                        ("bnb_8bit", {"attn_q": 8, "ffn_down": 8, "output": 8})])
def test_transformers_quantization_modes(tmp_path, mode, types):
    """`quantization: bnb_4bit / bnb_8bit` (reference transformers backend) quantise the HF
    checkpoint's linear weights at load into the GGML formats the HIP GEMMs read (Q4_K_M mix /
    Q8_0); the quantised model stays close to the float one (transformers oracle)."""
    d = str(tmp_path / "ck")
    synth.write_hf_checkpoint(d, kind="llama", hidden=256, heads=4, kv_heads=2, ffn=512)
    r = HFCheckpointReader(d, quantization=mode)
    for short, gt in types.items():
        name = "output.weight" if short == "output" else f"blk.0.{short}.weight"
        assert r.tensors[name].ggml_type == gt, (name, r.tensors[name].ggml_type)
    assert r.tensors["token_embd.weight"].ggml_type in (0, 1, 30)  # embeddings / norms stay float
    e = LLMEngine(EngineConfig(model_path=d, device="cpu", context_size=256, max_num_seqs=4, use_graphs=False,
                               quantization=mode))
    ids = e.tokenize(TEXT)
    ours = e.model.reference_logits(ids).float()
    ref = _hf_logits(d, ids)
    cos = float(torch.nn.functional.cosine_similarity(ours.flatten(), ref.flatten(), dim=0))
    # random-init gaussian weights are the worst case for 4-bit codes (no outlier structure)
    assert cos > (0.93 if mode == "bnb_4bit" else 0.999), cos
    out = e.generate(TEXT, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert out["completion_tokens"] == 4
    with pytest.raises(ValueError, match="quantization"):
        HFCheckpointReader(d, quantization="awq_3bit")
