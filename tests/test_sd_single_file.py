"""Single-file (LDM / SGM layout) Stable Diffusion checkpoints: conversion to the diffusers
layout (models/sd_single_file.py) is exact (same images as the directory the file was written
from), configs are inferred from tensor shapes for the published architectures, and the
diffusers backend loads a file path the way the reference's from_single_file does
(backend/python/diffusers/backend.py:184-191; aio/gpu-8g/image-gen.yaml)."""
import asyncio
import os

import pytest
import torch

from localai_amd.models import sd_single_file as ssf
from localai_amd.models import synth
from localai_amd.models.sd import StableDiffusion, UNet, VaeDecoder, VaeEncoder


@pytest.mark.parametrize("size,fam", [("tiny", "sd1"), ("tiny", "sd2"), ("tiny-xl", "sdxl")])
def test_single_file_round_trip_is_exact(tmp_path, size, fam):
    src = synth.write_sd_pipeline(str(tmp_path / "dir"), size=size, v_prediction=(fam == "sd2"))
    f = ssf.to_single_file(src, str(tmp_path / "model.safetensors"), fam)
    sd, hints = ssf.load_checkpoint(f)
    assert ssf.family(sd) == fam and hints["family"] == fam
    assert any(k.startswith("model.diffusion_model.input_blocks.") for k in sd)
    assert any(k.startswith("first_stage_model.decoder.up.") for k in sd)
    d = ssf.convert(f)
    assert os.path.isdir(d) and os.path.basename(d) == ".model.safetensors.diffusers"
    assert ssf.convert(f) == d  # cached: converted once
    a = StableDiffusion(src, "cpu")("a lighthouse", "", 32, 32, steps=2, seed=4)
    b = StableDiffusion(d, "cpu")("a lighthouse", "", 32, 32, steps=2, seed=4)
    assert torch.equal(a, b)


def _meta_state(cls, cfg):
    with torch.device("meta"):
        return cls(cfg).state_dict()


@pytest.mark.parametrize("name", ["SD15_UNET", "SDXL_UNET", "SD2"])
def test_unet_config_inferred_from_shapes(name):
    """The published UNets: config back from LDM-named tensor shapes (meta tensors, no memory)."""
    cfg = dict(getattr(synth, name)) if name != "SD2" else dict(
        synth.SD15_UNET, cross_attention_dim=1024, attention_head_dim=[5, 10, 20, 20], use_linear_projection=True)
    fam = {"SD15_UNET": "sd1", "SDXL_UNET": "sdxl", "SD2": "sd2"}[name]
    ldm = {ssf.unet_name_to_ldm(k, cfg): v for k, v in _meta_state(UNet, cfg).items()}
    got = ssf.infer_unet_config(ldm, fam)
    for k in ("block_out_channels", "layers_per_block", "cross_attention_dim", "down_block_types",
              "up_block_types", "in_channels", "out_channels"):
        assert got[k] == cfg[k], k
    assert bool(got.get("use_linear_projection")) == bool(cfg.get("use_linear_projection"))
    h = cfg["attention_head_dim"]
    assert got["attention_head_dim"] == h
    if "transformer_layers_per_block" in cfg:
        assert got["transformer_layers_per_block"][1:] == cfg["transformer_layers_per_block"][1:]
    if cfg.get("addition_embed_type"):
        assert got["projection_class_embeddings_input_dim"] == cfg["projection_class_embeddings_input_dim"]
    # the inferred config builds the same module tree
    assert set(_meta_state(UNet, got)) == set(_meta_state(UNet, cfg))


def test_vae_and_text_configs_inferred_from_shapes():
    import transformers as tf
    cfg = dict(synth.SD15_VAE)
    ldm = {}
    for cls in (VaeDecoder, VaeEncoder):
        ldm.update({ssf.vae_name_to_ldm(k, cfg): v for k, v in _meta_state(cls, cfg).items()})
    got = ssf.infer_vae_config(ldm, "sd1")
    for k in ("block_out_channels", "layers_per_block", "latent_channels", "in_channels", "out_channels"):
        assert got[k] == cfg[k], k
    with torch.device("meta"):
        te = tf.CLIPTextModelWithProjection(tf.CLIPTextConfig(**synth.SDXL_TEXT2))
    oc = ssf.hf_to_openclip(te.state_dict())
    assert "transformer.resblocks.31.attn.in_proj_weight" in oc and oc["text_projection"].shape == (1280, 1280)
    back = ssf.openclip_to_hf(oc, drop_last=False)
    tc = ssf.infer_text_config(back, "gelu", None)
    for k in ("hidden_size", "num_hidden_layers", "num_attention_heads", "intermediate_size", "projection_dim"):
        assert tc[k] == synth.SDXL_TEXT2[k], k
    sd2 = ssf.openclip_to_hf(oc, drop_last=True)
    assert ssf.infer_text_config(sd2, "gelu", None)["num_hidden_layers"] == 31


def test_ckpt_pickle_loads_weights_only(tmp_path):
    src = synth.write_sd_pipeline(str(tmp_path / "dir"))
    f = ssf.to_single_file(src, str(tmp_path / "m.safetensors"), "sd1")
    sd, hints = ssf.load_checkpoint(f)
    ck = str(tmp_path / "m.ckpt")
    torch.save({"state_dict": sd, "global_step": 1}, ck)
    sd2, _ = ssf.load_checkpoint(ck)
    assert set(sd2) == set(sd)


def test_missing_tokenizer_for_real_vocabulary_is_explained(tmp_path):
    src = synth.write_sd_pipeline(str(tmp_path / "dir"))
    f = ssf.to_single_file(src, str(tmp_path / "m.safetensors"), "sd1")
    sd, hints = ssf.load_checkpoint(f)
    k = "cond_stage_model.transformer.text_model.embeddings.token_embedding.weight"
    sd[k] = torch.zeros(49408, sd[k].shape[1])
    hints["text_encoder"]["vocab_size"] = 49408
    from safetensors.torch import save_file
    import json
    g = str(tmp_path / "big.safetensors")
    save_file(sd, g, metadata={ssf.META_KEY: json.dumps(hints)})
    with pytest.raises(ValueError, match="clip_model"):
        ssf.convert(g)
    # a tokenizer directory named by clip_model satisfies it
    d = ssf.convert(g, tokenizer_dir=src)
    assert os.path.isfile(os.path.join(d, "tokenizer", "vocab.json"))


def test_diffusers_backend_loads_single_file(tmp_path):
    """The AIO image-gen shape: a StableDiffusionPipeline model given as one .safetensors file."""
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    f = synth.write_sd_single_file(str(tmp_path / "DreamShaper_8_pruned.safetensors"))
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=f, PipelineType="StableDiffusionPipeline",
                                               SchedulerType="k_dpmpp_2m"), None)
        assert r.success, r.message
        dst = str(tmp_path / "out.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a dream", width=32, height=32, step=2,
                                                           seed=2, dst=dst), None)
        assert r.success, r.message
        assert os.path.getsize(dst) > 0
    asyncio.run(go())
