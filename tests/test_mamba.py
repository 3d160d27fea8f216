"""Mamba (selective SSM) backend: prompt scan and recurrent decode vs transformers'
MambaForCausalLM forward (independent oracle), the HIP decode-step kernels vs the PyTorch step,
and the gateway with `backend: mamba` (backend/python/mamba/backend.py)."""
import pytest
import torch

from localai_amd.models import synth
from localai_amd.models.mamba import MambaLM, is_mamba_checkpoint

TEXT = "The quick brown fox jumps over the lazy dog, then the model runs again."


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    return synth.write_hf_mamba(str(tmp_path_factory.mktemp("mamba") / "m"))


def _oracle(d, ids):
    import transformers as tf
    m = tf.MambaForCausalLM.from_pretrained(d, dtype=torch.float32).eval()
    with torch.no_grad():
        return m(torch.tensor([ids])).logits[0]


def test_prefill_and_decode_match_transformers(ckpt):
    assert is_mamba_checkpoint(ckpt)
    m = MambaLM(ckpt, "cpu")
    ids = m.tokenize(TEXT)
    ref = _oracle(ckpt, ids)
    st = m.new_state()
    got = m.prefill(ids, st)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 1e-4, err
    # the same sequence token by token through the recurrent step
    st2 = m.new_state()
    m.prefill(ids[:5], st2)
    for j in range(5, len(ids)):
        lg = m.step(torch.tensor([ids[j]]), st2)[0]
        e = float((lg - ref[j]).abs().max() / ref.abs().max())
        assert e < 1e-4, (j, e)


def test_servicer_generate_and_stop(ckpt):
    import asyncio

    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.mamba_servicer import MambaServicer
    sv = MambaServicer(device="cpu")

    async def go():
        assert (await sv.LoadModel(pb.ModelOptions(Model=ckpt), None)).success
        r = await sv.Predict(pb.PredictOptions(Prompt=TEXT, Tokens=6, Temperature=0.0, IgnoreEOS=True), None)
        parts = [x async for x in sv.PredictStream(pb.PredictOptions(Prompt=TEXT, Tokens=6, Temperature=0.0), None)]
        return r, parts
    r, parts = asyncio.run(go())
    assert r.tokens <= 6 and r.prompt_tokens == len(sv.model.tokenize(TEXT))
    assert b"".join(p.message for p in parts) == r.message and parts[-1].tokens == r.tokens
    # greedy == oracle argmax chain
    m = sv.model
    ids = m.tokenize(TEXT)
    want = []
    for _ in range(r.tokens):
        t = int(_oracle(ckpt, ids + want)[-1].argmax())
        if t == m.eos_id:
            break
        want.append(t)
    assert r.message.decode() == m.decode(want)
    if len(r.message) > 3:  # a stop string cuts the completion before it
        stop = r.message.decode()[2:4]

        async def go2():
            return await sv.Predict(pb.PredictOptions(Prompt=TEXT, Tokens=6, Temperature=0.0, StopPrompts=[stop]),
                                    None)
        r2 = asyncio.run(go2())
        assert stop not in r2.message.decode() and r.message.decode().startswith(r2.message.decode())


def test_gateway_mamba_backend(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    synth.write_hf_mamba(str(mdir / "mamba-tiny"), n_layer=1)
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    bc = BackendConfig({"name": "mamba", "backend": "mamba", "parameters": {"model": "mamba-tiny", "temperature": 0}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/completions", json={"model": "mamba", "prompt": "hello there", "max_tokens": 3})
        assert r.status_code == 200, r.text
        assert r.json()["usage"]["completion_tokens"] <= 3


@pytest.mark.gpu
def test_mamba_hip_step_matches_torch_step(ckpt):
    """The two HIP decode-step kernels (conv roll + SiLU, selective state update) vs the PyTorch
    step on the same fp32 inputs, and the GPU model vs the transformers oracle."""
    from localai_amd import ops
    torch.manual_seed(0)
    B, I, K, N, R = 3, 128, 4, 16, 8
    dev = "cuda:0"
    cs = torch.randn(B, I, K, device=dev)
    xz = torch.randn(B, 2 * I + 5, device=dev)[:, :2 * I + 5]
    w, b = torch.randn(I, K, device=dev), torch.randn(I, device=dev)
    cs_ref = torch.cat([cs[:, :, 1:], xz[:, :I].unsqueeze(-1)], -1)
    x_ref = torch.nn.functional.silu((cs_ref * w).sum(-1) + b)
    x = ops.mamba_conv_step(cs, xz, w, b, torch.empty(B, I, device=dev))
    torch.cuda.synchronize()
    assert torch.allclose(cs, cs_ref) and torch.allclose(x, x_ref, atol=1e-5, rtol=1e-5)
    ss = torch.randn(B, I, N, device=dev)
    dbc = torch.randn(B, R + 2 * N, device=dev)
    dt = torch.randn(B, I, device=dev)
    A = -torch.rand(I, N, device=dev) - 0.1
    D = torch.randn(I, device=dev)
    d = torch.nn.functional.softplus(dt)
    hs = torch.exp(d.unsqueeze(-1) * A) * ss + (d * x).unsqueeze(-1) * dbc[:, R:R + N].unsqueeze(1)
    y_ref = ((hs * dbc[:, R + N:].unsqueeze(1)).sum(-1) + x * D) * torch.nn.functional.silu(xz[:, I:2 * I])
    y = ops.mamba_ssm_step(ss, x, dt, dbc, R, R + N, A, D, xz, torch.empty(B, I, device=dev))
    torch.cuda.synchronize()
    assert torch.allclose(ss, hs, atol=1e-5, rtol=1e-4) and torch.allclose(y, y_ref, atol=1e-4, rtol=1e-4)
    # whole model on the GPU (bf16 projections) vs the fp32 oracle
    m = MambaLM(ckpt, dev)
    ids = m.tokenize(TEXT)
    ref = _oracle(ckpt, ids)
    st = m.new_state()
    m.prefill(ids[:-3], st)
    for j in range(len(ids) - 3, len(ids)):
        lg = m.step(torch.tensor([ids[j]], device=dev), st)[0].cpu()
        assert float((lg - ref[j]).abs().max() / ref.abs().max()) < 3e-2
