"""Stable Diffusion 3 (models/sd3.py) on a random-init StableDiffusion3Pipeline-layout directory.

Oracles: both projected CLIP encoders and the T5 encoder against transformers; the sin-cos position
table against its closed form; the FlowMatch shift in closed form.  The transformer has no oracle
(diffusers is not installed): parity unpinned -- strict diffusers weight names, determinism,
negative-prompt CFG, the T5-less variant, the backend route."""
import asyncio
import os

import numpy as np
import pytest
import torch

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import synth
from localai_amd.models.sd3 import SD3Pipeline, _sincos_2d, is_sd3_pipeline, sd3_sigmas


@pytest.fixture(scope="module")
def sd3_dir(tmp_path_factory):
    return synth.write_sd3_pipeline(str(tmp_path_factory.mktemp("sd3") / "sd3-tiny"))


def test_sd3_text_encoders_match_transformers(sd3_dir):
    import transformers as tf
    p = SD3Pipeline(sd3_dir, "cpu")
    ctx, pooled = p.encode(["a photo of a cat"])
    ids = p.tok1(["a photo of a cat"], padding="max_length", max_length=p.max_len, return_tensors="pt").input_ids
    with torch.no_grad():
        r1 = tf.CLIPTextModelWithProjection.from_pretrained(os.path.join(sd3_dir, "text_encoder")).eval()(
            ids, output_hidden_states=True)
        r2 = tf.CLIPTextModelWithProjection.from_pretrained(os.path.join(sd3_dir, "text_encoder_2")).eval()(
            ids, output_hidden_states=True)
        t5ids = p.tok3(["a photo of a cat"], padding="max_length", max_length=p.max_seq, truncation=True,
                       return_tensors="pt").input_ids
        r3 = tf.T5EncoderModel.from_pretrained(os.path.join(sd3_dir, "text_encoder_3")).eval()(t5ids)
    clip = torch.cat([r1.hidden_states[-2], r2.hidden_states[-2]], -1)
    torch.testing.assert_close(ctx[:, :77, :clip.shape[-1]], clip, rtol=1e-5, atol=1e-5)
    assert float(ctx[:, :77, clip.shape[-1]:].abs().max()) == 0.0          # zero-padded to the T5 width
    torch.testing.assert_close(ctx[:, 77:], r3.last_hidden_state, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(pooled, torch.cat([r1.text_embeds, r2.text_embeds], -1), rtol=1e-5, atol=1e-5)


def test_sd3_position_table_and_shift():
    pe = _sincos_2d(8, 4, 4, 1.0)                                          # [16, 8]
    om = 1.0 / 10000 ** (np.arange(2) / 2.0)
    x, y = 3, 1                                                            # token (row 1, col 3)
    want = np.concatenate([np.sin(x * om), np.cos(x * om), np.sin(y * om), np.cos(y * om)])
    assert np.allclose(pe[y * 4 + x].numpy(), want, atol=1e-6)
    s = sd3_sigmas(4, {"shift": 3.0})
    base = np.linspace(1, 0.25, 4)
    assert np.allclose(s[:-1], 3 * base / (1 + 2 * base)) and s[-1] == 0.0


def test_sd3_weight_names_and_pipeline(sd3_dir, tmp_path):
    p = SD3Pipeline(sd3_dir, "cpu")
    names = set(p.tr.state_dict())
    assert {"pos_embed.proj.weight", "pos_embed.pos_embed", "time_text_embed.timestep_embedder.linear_1.weight",
            "time_text_embed.text_embedder.linear_2.bias", "context_embedder.weight",
            "transformer_blocks.0.attn.add_q_proj.weight", "transformer_blocks.0.attn.to_add_out.weight",
            "transformer_blocks.0.ff_context.net.0.proj.weight", "transformer_blocks.1.norm1_context.linear.weight",
            "norm_out.linear.weight", "proj_out.weight"} <= names
    # the last block is context_pre_only: no text output projection, no text MLP
    assert not any(k.startswith(("transformer_blocks.1.attn.to_add_out", "transformer_blocks.1.ff_context"))
                   for k in names)
    assert tuple(p.tr.norm_out.linear.weight.shape)[0] == 2 * 32
    a = p("a red fox", "", 64, 64, steps=3, seed=1)
    assert a.shape == (64, 64, 3) and torch.equal(a, p("a red fox", "", 64, 64, steps=3, seed=1))
    assert not torch.equal(a, p("a red fox", "blurry", 64, 64, steps=3, seed=1))   # CFG uses the negative
    assert not torch.equal(a, p("a red fox", "", 64, 64, steps=3, seed=1, guidance_scale=1.0))
    no_t5 = synth.write_sd3_pipeline(str(tmp_path / "no-t5"), t5=False)
    q = SD3Pipeline(no_t5, "cpu")
    ctx, _ = q.encode(["x"])
    assert float(ctx[:, 77:].abs().max()) == 0.0                           # zero T5 context without it
    assert q("x", "", 48, 32, steps=1, seed=2).shape == (32, 48, 3)


def test_sd3_through_diffusers_backend(sd3_dir, tmp_path):
    from PIL import Image

    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    assert is_sd3_pipeline(sd3_dir)
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=sd3_dir, PipelineType="StableDiffusion3Pipeline"), None)
        assert r.success, r.message
        dst = str(tmp_path / "sd3.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a lighthouse", negative_prompt="fog",
                                                           width=64, height=64, step=2, seed=5, dst=dst), None)
        assert r.success, r.message
        assert Image.open(dst).size == (64, 64)
    asyncio.run(go())


@pytest.mark.gpu
def test_sd3_on_gpu_graph_matches_eager(sd3_dir):
    p = SD3Pipeline(sd3_dir, "cuda:0")
    a = p("graph capture", "", 64, 64, steps=3, seed=4)
    b = p("graph capture", "", 64, 64, steps=3, seed=4)
    assert p._graphs
    p.use_graphs = False
    c = p("graph capture", "", 64, 64, steps=3, seed=4)
    assert float((a.float() - b.float()).abs().max()) <= 3 and float((b.float() - c.float()).abs().max()) <= 3


@pytest.mark.gpu
def test_transformer_on_gpu_matches_fp32_forward(sd3_dir):
    """Every transformer evaluation of a GPU run (bf16, graph capture and replays) against the
    same weights in fp32 PyTorch on the CPU, on the same inputs."""
    from conftest import compare_to_fp32, record_calls
    p = SD3Pipeline(sd3_dir, "cuda:0")
    calls = record_calls(p, "_step")
    p("numerics", "", 64, 64, steps=2, seed=4)
    cpu = SD3Pipeline(sd3_dir, "cpu")
    compare_to_fp32(calls, cpu.tr)
