"""FLUX.1 (models/flux.py) on a random-init FluxPipeline-layout directory (synth.write_flux_pipeline).

Oracles: the T5 encoder (text_encoder_2) and the CLIP pooled output against transformers on the
same weights; the FlowMatch Euler sampler in closed form (the exact velocity of the linear path
lands on the clean latent) and its dynamic shift against the scheduler formula.  The transformer
has no oracle (diffusers is not installed): parity unpinned -- strict diffusers weight names,
determinism, guidance / prompt sensitivity, sizes, the diffusers backend route."""
import asyncio
import math
import os

import numpy as np
import pytest
import torch

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import synth
from localai_amd.models.flux import FluxPipeline, flow_euler, flow_sigmas, is_flux_pipeline


@pytest.fixture(scope="module")
def flux_dir(tmp_path_factory):
    return synth.write_flux_pipeline(str(tmp_path_factory.mktemp("flux") / "flux-tiny"))


def test_flux_text_encoders_match_transformers(flux_dir):
    import transformers as tf
    p = FluxPipeline(flux_dir, "cpu")
    ids = p.tok2(["a photo of a cat"], padding="max_length", max_length=32, truncation=True,
                 return_tensors="pt").input_ids
    ref = tf.T5EncoderModel.from_pretrained(os.path.join(flux_dir, "text_encoder_2")).eval()
    with torch.no_grad():
        torch.testing.assert_close(p.t5(ids), ref(ids).last_hidden_state, rtol=1e-4, atol=1e-5)
        cids = p.tok(["a photo of a cat"], padding="max_length", max_length=p.max_len, return_tensors="pt").input_ids
        clip = tf.CLIPTextModel.from_pretrained(os.path.join(flux_dir, "text_encoder")).eval()
        _, pooled = p.text.sdxl(cids, 0, pooled=True)
        torch.testing.assert_close(pooled, clip(cids).pooler_output, rtol=1e-5, atol=1e-5)


def test_flux_transformer_weight_names(flux_dir):
    p = FluxPipeline(flux_dir, "cpu")
    names = set(p.tr.state_dict())
    want = {"x_embedder.weight", "context_embedder.weight", "time_text_embed.timestep_embedder.linear_1.weight",
            "time_text_embed.guidance_embedder.linear_2.bias", "time_text_embed.text_embedder.linear_1.weight",
            "transformer_blocks.0.norm1.linear.weight", "transformer_blocks.0.norm1_context.linear.weight",
            "transformer_blocks.0.attn.to_q.weight", "transformer_blocks.0.attn.norm_q.weight",
            "transformer_blocks.0.attn.add_k_proj.bias", "transformer_blocks.0.attn.norm_added_k.weight",
            "transformer_blocks.0.attn.to_out.0.weight", "transformer_blocks.0.attn.to_add_out.weight",
            "transformer_blocks.0.ff.net.0.proj.weight", "transformer_blocks.0.ff_context.net.2.weight",
            "single_transformer_blocks.1.norm.linear.weight", "single_transformer_blocks.1.proj_mlp.weight",
            "single_transformer_blocks.1.attn.norm_k.weight", "single_transformer_blocks.1.proj_out.weight",
            "norm_out.linear.weight", "proj_out.weight"}
    assert want <= names, sorted(want - names)
    assert not any(k.startswith("single_transformer_blocks.0.attn.to_out") for k in names)


def test_flow_sampler_closed_form():
    cfg = synth.FLUX_SCHEDULER
    sig = flow_sigmas(4, 256, cfg)            # mu = base_shift 0.5 at the base sequence length
    s = np.linspace(1, 0.25, 4)
    want = math.exp(0.5) / (math.exp(0.5) + (1 / s - 1))
    assert np.allclose(sig[:-1], want) and sig[-1] == 0.0 and sig[0] == pytest.approx(1.0)
    big = flow_sigmas(4, 4096, cfg)           # longer sequences shift toward high noise (mu = 1.15)
    assert all(b >= a for a, b in zip(sig[1:-1], big[1:-1]))
    g = torch.Generator().manual_seed(0)
    x0, n = torch.randn(1, 8, 4, generator=g), torch.randn(1, 8, 4, generator=g)
    x = flow_euler(lambda xv, s_: n - x0, n.clone(), flow_sigmas(7, 1000, cfg))  # x_s = (1-s) x0 + s n
    torch.testing.assert_close(x, x0, rtol=0, atol=1e-5)


def test_flux_pipeline_determinism_and_conditioning(flux_dir):
    p = FluxPipeline(flux_dir, "cpu")
    a = p("a red fox", width=64, height=64, steps=3, seed=1, guidance_scale=3.5)
    assert a.shape == (64, 64, 3) and a.dtype == torch.uint8
    assert torch.equal(a, p("a red fox", width=64, height=64, steps=3, seed=1, guidance_scale=3.5))
    assert not torch.equal(a, p("a red fox", width=64, height=64, steps=3, seed=1, guidance_scale=7.0))
    assert not torch.equal(a, p("a blue whale", width=64, height=64, steps=3, seed=1, guidance_scale=3.5))
    assert p("a red fox", width=70, height=40, steps=1, seed=1).shape == (40, 68, 3)  # multiples of 4 (toy VAE x 2x2 packing)
    with pytest.raises(ValueError, match="text-to-image"):
        p("x", image="/nonexistent.png")


def test_flux_through_diffusers_backend(flux_dir, tmp_path):
    from PIL import Image

    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    assert is_flux_pipeline(flux_dir)
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=flux_dir, PipelineType="FluxPipeline"), None)
        assert r.success, r.message
        dst = str(tmp_path / "flux.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a castle", width=64, height=64, step=2,
                                                           seed=9, dst=dst), None)
        assert r.success, r.message
        assert Image.open(dst).size == (64, 64)
    asyncio.run(go())


def test_bfl_single_file_mapping_is_exact_inverse(flux_dir):
    """BFL layout <-> diffusers names: fused q|k|v (double blocks), fused q|k|v|mlp (single
    blocks), final adaLN halves swapped; every tensor mapped, the round trip bit-exact, and the
    config inferred from the shapes equals the pipeline's transformer config."""
    from localai_amd.models import flux_single_file as fsf
    from localai_amd.models.sd import _cfg, _load_weights
    sd = _load_weights(os.path.join(flux_dir, "transformer"))
    bfl = fsf.diffusers_to_bfl(sd)
    assert fsf.is_bfl(bfl) and "double_blocks.0.img_attn.qkv.weight" in bfl and "single_blocks.1.linear1.bias" in bfl
    assert "final_layer.adaLN_modulation.1.weight" in bfl and "guidance_in.in_layer.weight" in bfl
    d = sd["x_embedder.weight"].shape[0]
    assert bfl["single_blocks.0.linear1.weight"].shape[0] == 3 * d + sd["single_transformer_blocks.0.proj_mlp.weight"].shape[0]
    w = bfl["final_layer.adaLN_modulation.1.weight"]
    assert torch.equal(w[: w.shape[0] // 2], sd["norm_out.linear.weight"][w.shape[0] // 2:])  # (shift, scale)
    back = fsf.bfl_to_diffusers({"model.diffusion_model." + k: v for k, v in bfl.items()})
    assert set(back) == set(sd) and all(torch.equal(back[k], sd[k]) for k in sd)
    tc = _cfg(os.path.join(flux_dir, "transformer", "config.json"))
    got = fsf.infer_config(bfl, {"axes_dims_rope": tc["axes_dims_rope"]})
    for k in ("in_channels", "num_layers", "num_single_layers", "attention_head_dim", "num_attention_heads",
              "joint_attention_dim", "pooled_projection_dim", "guidance_embeds", "axes_dims_rope"):
        assert got[k] == tc[k], (k, got[k], tc[k])
    with pytest.raises(KeyError, match="unmapped|unknown"):
        fsf.bfl_to_diffusers(dict(bfl, **{"double_blocks.0.img_attn.extra.weight": w}))


def test_flux_transformer_single_file_through_backend(flux_dir, tmp_path, monkeypatch):
    """pipeline_type FluxTransformer2DModel (backend.py:255-269): the transformer from a BFL
    single file (here: the pipeline's weights with proj_out doubled, so the file is provably the
    one served), the rest of the pipeline from BFL_REPO; without BFL_REPO the load is refused."""
    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    from localai_amd.models import flux_single_file as fsf
    from localai_amd.models.sd import _cfg, _load_weights
    sd = _load_weights(os.path.join(flux_dir, "transformer"))
    sd["proj_out.weight"] = sd["proj_out.weight"] * 2
    tc = _cfg(os.path.join(flux_dir, "transformer", "config.json"))
    f = fsf.write_bfl_file(sd, str(tmp_path / "flux1-tiny.safetensors"), axes=tc["axes_dims_rope"])
    p = FluxPipeline(flux_dir, "cpu", transformer_file=f)
    assert torch.equal(p.tr.state_dict()["proj_out.weight"], sd["proj_out.weight"])
    sv = DiffusersServicer(device="cpu")

    async def go():
        monkeypatch.delenv("BFL_REPO", raising=False)
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=f, PipelineType="FluxTransformer2DModel"), None)
        assert not r.success and "BFL_REPO" in r.message
        monkeypatch.setenv("BFL_REPO", flux_dir)
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=f, PipelineType="FluxTransformer2DModel"), None)
        assert r.success, r.message
        dst = str(tmp_path / "fluxsf.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a castle", width=64, height=64, step=2,
                                                           seed=9, dst=dst), None)
        assert r.success, r.message
    asyncio.run(go())


@pytest.mark.gpu
def test_flux_on_gpu_graph_matches_eager(flux_dir):
    p = FluxPipeline(flux_dir, "cuda:0")
    a = p("graph capture", width=64, height=64, steps=3, seed=4)
    b = p("graph capture", width=64, height=64, steps=3, seed=4)
    assert p._graphs
    p.use_graphs = False
    c = p("graph capture", width=64, height=64, steps=3, seed=4)
    assert float((a.float() - b.float()).abs().max()) <= 3 and float((b.float() - c.float()).abs().max()) <= 3


@pytest.mark.gpu
def test_transformer_on_gpu_matches_fp32_forward(flux_dir):
    """Every transformer evaluation of a GPU run (bf16, graph capture and replays) against the
    same weights in fp32 PyTorch on the CPU, on the same inputs."""
    from conftest import compare_to_fp32, record_calls
    p = FluxPipeline(flux_dir, "cuda:0")
    calls = record_calls(p, "_step")
    p("numerics", width=64, height=64, steps=2, seed=4)
    cpu = FluxPipeline(flux_dir, "cpu")
    compare_to_fp32(calls, cpu.tr)
