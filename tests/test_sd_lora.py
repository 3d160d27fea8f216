"""LoRA adapters for the Stable Diffusion pipeline (models/sd_lora.py; reference
backend/python/diffusers/backend.py:300-314).  The merged weights must equal
W + scale * (alpha / rank) * up @ down for linear, 1x1 and 3x3 conv targets in the UNet and the
text encoder, for the kohya, PEFT and attention-processor key layouts; unknown module names are
refused; the backend resolves a relative `LoraAdapter` against the model file's directory."""
import asyncio
import os

import pytest
import torch
from safetensors.torch import save_file

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import synth
from localai_amd.models.sd import StableDiffusion
from localai_amd.models.sd_lora import merge_sd_lora

TARGETS = ["down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q",
           "up_blocks.1.attentions.0.transformer_blocks.0.attn2.to_out.0",
           "down_blocks.0.resnets.0.conv1",                 # 3x3 conv
           "down_blocks.0.attentions.0.proj_in"]           # linear or 1x1 conv (config dependent)
TE = "text_model.encoder.layers.0.self_attn.q_proj"


@pytest.fixture(scope="module")
def pipe_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("sdl") / "sd-tiny"
    synth.write_sd_pipeline(str(d))
    return str(d)


def _lora(base, layout, rank=2, seed=0):
    g = torch.Generator().manual_seed(seed)
    sd, ref = {}, {}
    unet = dict(base.unet.named_parameters())
    te = dict(base.text.named_parameters())
    for target, name in [("unet", t) for t in TARGETS] + [("te", TE)]:
        w = (unet if target == "unet" else te)[name + ".weight"]
        out_, in_ = w.shape[0], w.shape[1]
        kern = tuple(w.shape[2:])
        down = torch.randn((rank, in_) + kern, generator=g) * 0.1
        up = torch.randn((out_, rank) + tuple(1 for _ in kern), generator=g) * 0.1
        alpha = torch.tensor(4.0)
        ref[(target, name)] = (4.0 / rank) * (up.reshape(out_, rank) @ down.reshape(rank, -1)).reshape(w.shape)
        if layout == "kohya":
            k = ("lora_unet_" if target == "unet" else "lora_te_") + name.replace(".", "_")
            sd[k + ".lora_down.weight"], sd[k + ".lora_up.weight"], sd[k + ".alpha"] = down, up, alpha
        else:
            k = ("unet." if target == "unet" else "text_encoder.") + name
            sd[k + ".lora_A.weight"], sd[k + ".lora_B.weight"], sd[k + ".alpha"] = down, up, alpha
    return sd, ref


@pytest.mark.parametrize("layout", ["kohya", "peft"])
def test_lora_merge_equals_low_rank_update(pipe_dir, tmp_path, layout):
    base = StableDiffusion(pipe_dir, "cpu")
    sd, ref = _lora(base, layout)
    f = str(tmp_path / f"{layout}.safetensors")
    save_file(sd, f)
    p = StableDiffusion(pipe_dir, "cpu", lora=f, lora_scale=0.5)
    for (target, name), delta in ref.items():
        a = dict((base.unet if target == "unet" else base.text).named_parameters())[name + ".weight"]
        b = dict((p.unet if target == "unet" else p.text).named_parameters())[name + ".weight"]
        torch.testing.assert_close(b, a + 0.5 * delta, atol=1e-6, rtol=1e-5)
    untouched = "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_k.weight"
    assert torch.equal(dict(p.unet.named_parameters())[untouched], dict(base.unet.named_parameters())[untouched])
    img_a = base("a red fox", "", 32, 32, steps=2, seed=1)
    img_b = p("a red fox", "", 32, 32, steps=2, seed=1)
    assert not torch.equal(img_a, img_b)


def test_attn_processor_layout_and_unknown_keys(pipe_dir, tmp_path):
    base = StableDiffusion(pipe_dir, "cpu")
    name = "down_blocks.0.attentions.0.transformer_blocks.0.attn1"
    w = dict(base.unet.named_parameters())[name + ".to_v.weight"].detach().clone()
    down, up = torch.randn(2, w.shape[1]) * 0.1, torch.randn(w.shape[0], 2) * 0.1
    d = tmp_path / "procs"
    os.makedirs(d)
    save_file({f"{name}.processor.to_v_lora.down.weight": down, f"{name}.processor.to_v_lora.up.weight": up},
              str(d / "pytorch_lora_weights.safetensors"))
    assert merge_sd_lora(str(d), base.unet) == 1
    torch.testing.assert_close(dict(base.unet.named_parameters())[name + ".to_v.weight"], w + up @ down)
    bad = str(tmp_path / "bad.safetensors")
    save_file({"lora_unet_input_blocks_9_1_proj_in.lora_down.weight": down,
               "lora_unet_input_blocks_9_1_proj_in.lora_up.weight": up}, bad)
    with pytest.raises(ValueError, match="match no pipeline weight"):
        merge_sd_lora(bad, base.unet)


# the tiny UNet: layers_per_block 1; down blocks (CrossAttn + downsampler, plain); up blocks
# (plain + upsampler, CrossAttn) -- the LDM input / middle / output block numbering of that layout
LDM_NAMES = {
    "input_blocks_1_1_transformer_blocks_0_attn1_to_q": "down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q",
    "input_blocks_1_0_in_layers_2": "down_blocks.0.resnets.0.conv1",
    "input_blocks_2_0_op": "down_blocks.0.downsamplers.0.conv",
    "input_blocks_3_0_emb_layers_1": "down_blocks.1.resnets.0.time_emb_proj",
    "middle_block_1_proj_in": "mid_block.attentions.0.proj_in",
    "middle_block_2_out_layers_3": "mid_block.resnets.1.conv2",
    "output_blocks_0_0_skip_connection": "up_blocks.0.resnets.0.conv_shortcut",
    "output_blocks_1_1_conv": "up_blocks.0.upsamplers.0.conv",
    "output_blocks_3_1_transformer_blocks_0_attn2_to_out_0":
        "up_blocks.1.attentions.1.transformer_blocks.0.attn2.to_out.0",
    "time_embed_2": "time_embedding.linear_2",
    "out_2": "conv_out",
}


def test_ldm_named_kohya_lora(pipe_dir, tmp_path):
    """kohya files in the original LDM / SGM UNet naming land on the same modules as their
    diffusers-named twins."""
    from localai_amd.models.sd_lora import ldm_unet_path
    base = StableDiffusion(pipe_dir, "cpu")
    params = dict(base.unet.named_parameters())
    g = torch.Generator().manual_seed(7)
    ldm, diff = {}, {}
    for k, name in LDM_NAMES.items():
        assert ldm_unet_path(k, base.unet) == name.replace(".", "_"), k
        w = params[name + ".weight"]
        down = torch.randn((2,) + tuple(w.shape[1:]), generator=g) * 0.1
        up = torch.randn((w.shape[0], 2) + tuple(1 for _ in w.shape[2:]), generator=g) * 0.1
        for sd, key in ((ldm, "lora_unet_" + k), (diff, "lora_unet_" + name.replace(".", "_"))):
            sd[key + ".lora_down.weight"], sd[key + ".lora_up.weight"] = down, up
    fa, fb = str(tmp_path / "ldm.safetensors"), str(tmp_path / "diffusers.safetensors")
    save_file(ldm, fa)
    save_file(diff, fb)
    a = StableDiffusion(pipe_dir, "cpu", lora=fa)
    b = StableDiffusion(pipe_dir, "cpu", lora=fb)
    for (n1, p1), (n2, p2) in zip(a.unet.named_parameters(), b.unet.named_parameters()):
        assert n1 == n2 and torch.equal(p1, p2), n1


def test_backend_lora_adapter_relative_to_model_dir(pipe_dir, tmp_path):
    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    base = StableDiffusion(pipe_dir, "cpu")
    sd, _ = _lora(base, "kohya")
    models = os.path.dirname(pipe_dir)
    save_file(sd, os.path.join(models, "style.safetensors"))
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=pipe_dir, LoraAdapter="style.safetensors"))
        assert r.success, r.message
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=pipe_dir, LoraAdapter="missing.safetensors"))
        assert not r.success and "not found" in r.message
    asyncio.run(go())
