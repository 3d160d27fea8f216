"""Single-file Stable Diffusion 3 checkpoints (models/sd3_single_file.py): the Stability MMDiT
layout maps onto the diffusers SD3Transformer2DModel names exactly (inverse pair, the fused qkv
splits and the swapped (shift, scale) halves included), a converted file renders the same image
as the directory it was written from, text encoders missing from the file come from a base
pipeline directory, and the diffusers backend loads a file path as the reference's
StableDiffusion3Pipeline.from_single_file does (backend/python/diffusers/backend.py:238-242).
Parity with diffusers' own converter is unpinned (diffusers is not installed)."""
import asyncio
import os

import pytest
import torch

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import sd3_single_file as s3f
from localai_amd.models import sd_single_file as ssf
from localai_amd.models import synth
from localai_amd.models.sd import _load_weights
from localai_amd.models.sd3 import SD3Pipeline, is_sd3_pipeline


@pytest.fixture(scope="module")
def sd3_dir(tmp_path_factory):
    return synth.write_sd3_pipeline(str(tmp_path_factory.mktemp("sd3sf") / "sd3-tiny"))


def test_mmdit_mapping_is_an_exact_inverse(sd3_dir):
    sd = _load_weights(os.path.join(sd3_dir, "transformer"))
    mm = s3f.diffusers_to_mmdit(sd)
    assert "joint_blocks.0.x_block.attn.qkv.weight" in mm and "x_embedder.proj.weight" in mm
    assert "joint_blocks.1.context_block.attn.proj.weight" not in mm   # the pre_only last block
    back = s3f.mmdit_to_diffusers(mm)
    assert set(back) == set(sd)
    for k in sd:
        assert torch.equal(back[k], sd[k]), k
    # the adaLN-continuous halves are stored (shift, scale) in the MMDiT layout
    a, b = sd["norm_out.linear.weight"].chunk(2, 0)
    assert torch.equal(mm["final_layer.adaLN_modulation.1.weight"], torch.cat([b, a], 0))
    cfg = s3f.infer_config(mm)
    assert cfg["num_layers"] == 2 and cfg["patch_size"] == 2 and cfg["in_channels"] == 16
    assert cfg["pos_embed_max_size"] == 24 and cfg["joint_attention_dim"] == 96


def test_single_file_renders_like_its_source(sd3_dir, tmp_path):
    f = s3f.to_single_file(sd3_dir, str(tmp_path / "sd3_medium_incl_clips.safetensors"))
    sd, hints = ssf.load_checkpoint(f)
    assert s3f.is_sd3_file(sd) and any(k.startswith("text_encoders.t5xxl.transformer.") for k in sd)
    d = ssf.convert(f, tokenizer_dir=sd3_dir)   # the T5 tokenizer is never in the file
    assert is_sd3_pipeline(d) and ssf.convert(f, tokenizer_dir=sd3_dir) == d
    a = SD3Pipeline(sd3_dir, "cpu")("a lighthouse", "", 64, 64, steps=2, seed=3)
    b = SD3Pipeline(d, "cpu")("a lighthouse", "", 64, 64, steps=2, seed=3)
    assert torch.equal(a, b)


def test_text_encoders_from_a_base_directory(sd3_dir, tmp_path):
    f = s3f.to_single_file(sd3_dir, str(tmp_path / "sd3_medium.safetensors"), with_text=False)
    with pytest.raises(ValueError, match="clip_model"):
        ssf.convert(f, out_dir=str(tmp_path / "x"))
    d = ssf.convert(f, tokenizer_dir=sd3_dir)
    a = SD3Pipeline(sd3_dir, "cpu")("x", "", 32, 32, steps=1, seed=1)
    assert torch.equal(a, SD3Pipeline(d, "cpu")("x", "", 32, 32, steps=1, seed=1))


def test_dual_attention_checkpoints_are_refused():
    with pytest.raises(ValueError, match="dual-attention"):
        s3f.mmdit_to_diffusers({"joint_blocks.0.x_block.attn2.qkv.weight": torch.zeros(3, 1)})


def test_single_file_through_diffusers_backend(sd3_dir, tmp_path):
    from PIL import Image

    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    f = s3f.to_single_file(sd3_dir, str(tmp_path / "sd3.safetensors"))
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=f, PipelineType="StableDiffusion3Pipeline",
                                               CLIPModel=sd3_dir), None)
        assert r.success, r.message
        dst = str(tmp_path / "out.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a lighthouse", width=64, height=64, step=2,
                                                           seed=5, dst=dst), None)
        assert r.success, r.message
        assert Image.open(dst).size == (64, 64)
    asyncio.run(go())


def test_vae_config_inferred_from_shapes(sd3_dir, tmp_path):
    """Without the file's metadata the 16-channel VAE config comes back from the LDM tensor shapes
    (all but the GroupNorm group count, which the weights do not carry: 32 for the published VAEs)."""
    import json
    f = s3f.to_single_file(sd3_dir, str(tmp_path / "m.safetensors"), with_text=False, with_hints=False)
    sd, hints = ssf.load_checkpoint(f)
    assert not hints
    cfg, vsd = s3f._vae(sd, None)
    src = json.load(open(os.path.join(sd3_dir, "vae", "config.json")))
    for k in ("block_out_channels", "layers_per_block", "latent_channels", "scaling_factor", "shift_factor"):
        assert cfg[k] == src[k], k
    ref = _load_weights(os.path.join(sd3_dir, "vae"))
    assert set(vsd) == set(ref) and all(torch.equal(vsd[k], ref[k]) for k in ref)
