"""RWKV-4 backend (backend/go/llm/rwkv/rwkv.go): the recurrent model vs transformers'
RwkvForCausalLM forward, BlinkDL-named state dicts, the servicer's default "\\n" stop word and
TokenizeString, and the gateway with `backend: rwkv`."""
import asyncio

import pytest
import torch

from localai_amd.models import synth
from localai_amd.models.rwkv import RwkvLM, is_rwkv_checkpoint

TEXT = "The quick brown fox jumps over the lazy dog and runs away."


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    return synth.write_hf_rwkv(str(tmp_path_factory.mktemp("rwkv") / "m"))


def _oracle(d, ids):
    import transformers as tf
    m = tf.RwkvForCausalLM.from_pretrained(d, dtype=torch.float32).eval()
    with torch.no_grad():
        return m(torch.tensor([ids])).logits[0]


def test_logits_match_transformers(ckpt):
    assert is_rwkv_checkpoint(ckpt)
    m = RwkvLM(ckpt, "cpu")
    ids = m.tokenize(TEXT)
    got = m.prefill(ids, m.new_state())
    ref = _oracle(ckpt, ids)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 1e-4, err


def test_blinkdl_state_dict(ckpt, tmp_path):
    """The original .pth naming (emb / blocks.N.att / ffn / ln0, time_mix_k/v/r) loads to the same model."""
    from safetensors.torch import load_file
    sd = load_file(f"{ckpt}/model.safetensors")
    ren = {}
    for k, v in sd.items():
        n = k.replace("rwkv.embeddings.weight", "emb.weight").replace("rwkv.ln_out.", "ln_out.")
        n = n.replace("rwkv.blocks.", "blocks.").replace(".attention.", ".att.").replace(".feed_forward.", ".ffn.")
        n = n.replace("pre_ln.", "ln0.").replace("time_mix_key", "time_mix_k").replace("time_mix_value", "time_mix_v")
        n = n.replace("time_mix_receptance", "time_mix_r")
        ren[n] = v
    pth = tmp_path / "RWKV-4-tiny.pth"
    torch.save(ren, pth)
    import shutil
    shutil.copy(f"{ckpt}/tokenizer.json", str(pth) + ".tokenizer.json")  # rwkv.go's sidecar name
    a, b = RwkvLM(ckpt, "cpu"), RwkvLM(str(pth), "cpu")
    ids = a.tokenize(TEXT)
    assert b.tokenize(TEXT) == ids
    assert torch.allclose(a.prefill(ids, a.new_state()), b.prefill(ids, b.new_state()))


def test_servicer_defaults(ckpt):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.mamba_servicer import RwkvServicer
    sv = RwkvServicer(device="cpu")

    async def go():
        assert (await sv.LoadModel(pb.ModelOptions(Model=ckpt), None)).success
        tk = await sv.TokenizeString(pb.PredictOptions(Prompt=TEXT), None)
        r = await sv.Predict(pb.PredictOptions(Prompt=TEXT, Tokens=8, Temperature=0.0), None)
        return tk, r
    tk, r = asyncio.run(go())
    assert list(tk.tokens) == sv.model.tokenize(TEXT) and tk.length == len(tk.tokens)
    assert "\n" not in r.message.decode() and r.tokens <= 8  # default stop word "\n"


def test_gateway_rwkv_backend(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    synth.write_hf_rwkv(str(mdir / "rwkv-tiny"), n_layer=2)
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    bc = BackendConfig({"name": "rwkv", "backend": "rwkv", "parameters": {"model": "rwkv-tiny", "temperature": 0}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/completions", json={"model": "rwkv", "prompt": "hello there", "max_tokens": 4})
        assert r.status_code == 200, r.text
        assert r.json()["usage"]["completion_tokens"] <= 4
