"""Stable Diffusion 1.x / 2.x / XL text-to-image, served by the `diffusers` / `stablediffusion`
backends (reference: `backend/python/diffusers/backend.py:147-471` -- LoadModel keeps
`CFGScale` (default 7), `CLIPSkip`, `SchedulerType`; GenerateImage takes `step` (default 1),
width / height, `negative_prompt`, `seed` and `EnableParameters`, runs the pipeline and saves a
PNG to `dst`).

Reads the diffusers directory layout (`model_index.json`, `unet/`, `vae/`, `text_encoder/`,
`tokenizer/`, `scheduler/`, each with `config.json` + safetensors).  The modules below are named
like the checkpoint's tensors so `load_state_dict(strict=True)` checks every weight:

* CLIP text encoder (pre-LN transformer, causal mask, quick-GELU / GELU, optional clip-skip);
* UNet2DConditionModel: sinusoidal timestep embedding, ResNet blocks with time conditioning,
  Transformer2D blocks (self-attention, cross-attention to the prompt, GEGLU feed-forward),
  stride-2 downsamplers, nearest-2x upsamplers, skip concatenation;
* AutoencoderKL decoder (post-quant conv, ResNet / single-head attention mid block, upsampling
  ResNet stacks).

GroupNorm (+ the SiLU that follows it in every ResNet block) runs as one hand-written HIP kernel
pair on NHWC bf16 activations (ops/csrc/groupnorm.hip); it was the largest kernel-time item of the
PyTorch path (profiles/r2c_sd15.md).

Classifier-free guidance runs conditional and unconditional branches as one batch of 2.  On
the GPU everything is bf16 (convolutions through MIOpen, attention through PyTorch's fused SDPA,
the GEMMs through hipBLASLt); the schedulers keep latents in fp32.  Schedulers: every
`SchedulerType` of backend.py:74-143 (models/schedulers.py: DDIM, PNDM/PLMS, and the sigma-space
samplers euler, euler_a, heun, lms, dpm_2, dpm_2_a, dpmpp_2m, dpmpp_sde, dpmpp_2m_sde, unipc, with
`k_` Karras variants); an unknown name is refused, as the reference's get_scheduler does.
img2img: the KL-VAE encoder half samples the source image's latents, noised to `strength`.
"""
from __future__ import annotations

import json
import math
from collections import OrderedDict
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def _cfg(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def _load_weights(d: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    for n in ("diffusion_pytorch_model.safetensors", "model.safetensors"):
        p = os.path.join(d, n)
        if os.path.isfile(p):
            return load_file(p)
    for n in ("diffusion_pytorch_model.bin", "pytorch_model.bin"):
        p = os.path.join(d, n)
        if os.path.isfile(p):
            return torch.load(p, map_location="cpu", weights_only=True)
    raise FileNotFoundError(f"no weights in {d}")


def is_sd_pipeline(path: str) -> bool:
    return os.path.isdir(path) and os.path.isfile(os.path.join(path, "unet", "config.json")) and \
        os.path.isfile(os.path.join(path, "vae", "config.json"))


# ------------------------------------------------------------------ CLIP text encoder
class _ClipLayer(nn.Module):
    def __init__(self, d: int, heads: int, inter: int, act: str):
        super().__init__()
        self.heads, self.act = heads, act
        self.layer_norm1, self.layer_norm2 = nn.LayerNorm(d), nn.LayerNorm(d)
        self.self_attn = nn.Module()
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            setattr(self.self_attn, n, nn.Linear(d, d))
        self.mlp = nn.Module()
        self.mlp.fc1, self.mlp.fc2 = nn.Linear(d, inter), nn.Linear(inter, d)

    def forward(self, x):
        B, L, D = x.shape
        h = self.layer_norm1(x)
        a = self.self_attn
        q, k, v = (p(h).view(B, L, self.heads, -1).transpose(1, 2) for p in (a.q_proj, a.k_proj, a.v_proj))
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, L, D)
        x = x + a.out_proj(o)
        h = self.mlp.fc1(self.layer_norm2(x))
        h = h * torch.sigmoid(1.702 * h) if self.act == "quick_gelu" else F.gelu(h)
        return x + self.mlp.fc2(h)


class ClipTextEncoder(nn.Module):
    def __init__(self, c: dict):
        super().__init__()
        d = c["hidden_size"]
        self.eps = float(c.get("layer_norm_eps", 1e-5))
        self.text_model = nn.Module()
        tm = self.text_model
        tm.embeddings = nn.Module()
        tm.embeddings.token_embedding = nn.Embedding(c["vocab_size"], d)
        tm.embeddings.position_embedding = nn.Embedding(c["max_position_embeddings"], d)
        tm.encoder = nn.Module()
        tm.encoder.layers = nn.ModuleList(_ClipLayer(d, c["num_attention_heads"], c["intermediate_size"],
                                                     c.get("hidden_act", "quick_gelu"))
                                          for _ in range(c["num_hidden_layers"]))
        tm.final_layer_norm = nn.LayerNorm(d)
        self.eos_id = int(c.get("eos_token_id", 2))
        if c.get("projection_dim") and "CLIPTextModelWithProjection" in (c.get("architectures") or []):
            # SDXL's second encoder: the pooled (EOS) state through text_projection
            self.text_projection = nn.Linear(d, int(c["projection_dim"]), bias=False)
        for m in self.modules():
            if isinstance(m, nn.LayerNorm):
                m.eps = self.eps

    def _run(self, ids: torch.Tensor, n_layers: int) -> torch.Tensor:
        tm = self.text_model
        x = tm.embeddings.token_embedding(ids) + tm.embeddings.position_embedding.weight[: ids.shape[1]]
        for ly in tm.encoder.layers[:n_layers]:
            x = ly(x)
        return x

    def forward(self, ids: torch.Tensor, clip_skip: int = 0) -> torch.Tensor:
        # diffusers' clip_skip: the hidden state `clip_skip` layers before the last, then final LN
        return self.text_model.final_layer_norm(self._run(ids, len(self.text_model.encoder.layers) - clip_skip))

    def sdxl(self, ids: torch.Tensor, clip_skip: int = 0, pooled: bool = False):
        """SDXL conditioning: hidden_states[-(clip_skip + 2)] (no final LN) and, for the
        projection encoder, the final-LN state at the first EOS token through text_projection
        (transformers CLIPTextModelWithProjection.text_embeds)."""
        n = len(self.text_model.encoder.layers)
        h = self._run(ids, n - 1)
        pen = self._run(ids, n - 1 - clip_skip) if clip_skip else h
        if not pooled:
            return pen, None
        fin = self.text_model.final_layer_norm(self.text_model.encoder.layers[n - 1](h))
        eos = (ids == self.eos_id).int().argmax(-1)
        pool = fin[torch.arange(ids.shape[0], device=ids.device), eos]
        if hasattr(self, "text_projection"):
            pool = self.text_projection(pool)
        return pen, pool


# ------------------------------------------------------------------ UNet / VAE building blocks
def _gn(norm: nn.GroupNorm, x: torch.Tensor, silu: bool = False) -> torch.Tensor:
    """GroupNorm (+ SiLU): the fused HIP kernel (ops/csrc/groupnorm.hip) on bf16 NHWC activations,
    PyTorch elsewhere (CPU, NCHW)."""
    if x.is_cuda:
        from .. import ops
        if ops.groupnorm_supported(x, norm.num_groups):
            return ops.groupnorm_nhwc(x, norm.num_groups, norm.weight, norm.bias, norm.eps, silu)
    y = F.group_norm(x, norm.num_groups, norm.weight, norm.bias, norm.eps)
    return F.silu(y) if silu else y


class _Resnet(nn.Module):
    def __init__(self, cin: int, cout: int, groups: int, eps: float, temb: Optional[int]):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, cin, eps=eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        if temb:
            self.time_emb_proj = nn.Linear(temb, cout)
        self.norm2 = nn.GroupNorm(groups, cout, eps=eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        if cin != cout:
            self.conv_shortcut = nn.Conv2d(cin, cout, 1)

    def forward(self, x, temb=None):
        h = _gn(self.norm1, x, True)
        if temb is not None:
            # conv1's bias rides on the time-embedding add (one elementwise pass instead of two)
            tb = self.conv1.bias + self.time_emb_proj(F.silu(temb))
            h = F.conv2d(h, self.conv1.weight, None, padding=1) + tb[:, :, None, None]
        else:
            h = self.conv1(h)
        h = self.conv2(_gn(self.norm2, h, True))
        return (self.conv_shortcut(x) if hasattr(self, "conv_shortcut") else x) + h


class _Attn(nn.Module):
    def __init__(self, d: int, heads: int, ctx: Optional[int] = None, bias: bool = False):
        super().__init__()
        self.heads = heads
        self.to_q = nn.Linear(d, d, bias=bias)
        self.to_k = nn.Linear(ctx or d, d, bias=bias)
        self.to_v = nn.Linear(ctx or d, d, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(d, d)])

    def forward(self, x, ctx=None):
        B, L, D = x.shape
        c = x if ctx is None else ctx
        q = self.to_q(x).view(B, L, self.heads, -1).transpose(1, 2)
        k = self.to_k(c).view(B, c.shape[1], self.heads, -1).transpose(1, 2)
        v = self.to_v(c).view(B, c.shape[1], self.heads, -1).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, L, D)
        return self.to_out[0](o)


class _GEGLU(nn.Module):
    def __init__(self, d: int, inner: int):
        super().__init__()
        self.proj = nn.Linear(d, 2 * inner)

    def forward(self, x):
        h, g = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(g)


class _TBlock(nn.Module):
    def __init__(self, d: int, heads: int, ctx: int):
        super().__init__()
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn1, self.attn2 = _Attn(d, heads), _Attn(d, heads, ctx)
        self.ff = nn.Module()
        self.ff.net = nn.ModuleList([_GEGLU(d, 4 * d), nn.Identity(), nn.Linear(4 * d, d)])

    def forward(self, x, ctx):
        x = x + self.attn1(self.norm1(x))
        x = x + self.attn2(self.norm2(x), ctx)
        h = self.ff.net[0](self.norm3(x))
        return x + self.ff.net[2](h)


class _Transformer2D(nn.Module):
    def __init__(self, c: int, heads: int, ctx: int, groups: int, linear_proj: bool, depth: int = 1):
        super().__init__()
        self.linear = linear_proj
        self.norm = nn.GroupNorm(groups, c, eps=1e-6)
        self.proj_in = nn.Linear(c, c) if linear_proj else nn.Conv2d(c, c, 1)
        self.transformer_blocks = nn.ModuleList([_TBlock(c, heads, ctx) for _ in range(depth)])
        self.proj_out = nn.Linear(c, c) if linear_proj else nn.Conv2d(c, c, 1)

    def forward(self, x, ctx):
        B, C, H, W = x.shape
        h = _gn(self.norm, x)
        if not self.linear:
            h = self.proj_in(h)
        h = h.permute(0, 2, 3, 1).reshape(B, H * W, C)
        if self.linear:
            h = self.proj_in(h)
        for b in self.transformer_blocks:
            h = b(h, ctx)
        if self.linear:
            h = self.proj_out(h)
        h = h.reshape(B, H, W, C).permute(0, 3, 1, 2)
        if not self.linear:
            h = self.proj_out(h)
        return x + h


class _Down(nn.Module):
    def __init__(self, c: int, pad: int = 1):
        super().__init__()
        self.pad = pad
        self.conv = nn.Conv2d(c, c, 3, stride=2, padding=pad)

    def forward(self, x):
        if self.pad == 0:  # the VAE encoder pads right / bottom only
            x = F.pad(x, (0, 1, 0, 1))
        return self.conv(x)


class _Up(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)

    def forward(self, x, size=None):
        # diffusers' forward_upsample_size: when the latent side is not a multiple of 2^(levels-1)
        # the down path rounded up (stride-2 conv, padding 1), so the up path must land on the skip's
        # size exactly, not on 2x (e.g. 520 px -> latent 65 -> 33 -> 17 -> 9; 9 -> 17, not 18)
        if size is not None and (x.shape[-2] * 2 != size[0] or x.shape[-1] * 2 != size[1]):
            return self.conv(F.interpolate(x, size=tuple(size), mode="nearest"))
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


def _per_block(v, n: int) -> List[int]:
    return list(v) if isinstance(v, (list, tuple)) else [v] * n


class UNet(nn.Module):
    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        n = len(ch)
        lpb = int(c.get("layers_per_block", 2))
        g, eps = int(c.get("norm_num_groups", 32)), float(c.get("norm_eps", 1e-5))
        ctx = int(c["cross_attention_dim"])
        # diffusers: `attention_head_dim` holds the number of heads when num_attention_heads is unset
        heads = _per_block(c.get("num_attention_heads") or c.get("attention_head_dim", 8), n)
        lin = bool(c.get("use_linear_projection", False))
        # SDXL: several transformer blocks per attention (transformer_layers_per_block, e.g. 1/2/10)
        depth = _per_block(c.get("transformer_layers_per_block", 1), n)
        rdepth = c.get("reverse_transformer_layers_per_block")
        self.flip = bool(c.get("flip_sin_to_cos", True))
        self.shift = float(c.get("freq_shift", 0))
        temb = ch[0] * 4
        self.conv_in = nn.Conv2d(c.get("in_channels", 4), ch[0], 3, padding=1)
        self.time_embedding = nn.Module()
        self.time_embedding.linear_1 = nn.Linear(ch[0], temb)
        self.time_embedding.linear_2 = nn.Linear(temb, temb)
        # SDXL micro-conditioning (addition_embed_type "text_time"): sinusoidal embeddings of the 6
        # size / crop time ids, concatenated with the pooled text embedding, through add_embedding
        self.text_time = c.get("addition_embed_type") == "text_time"
        if self.text_time:
            self.add_time_dim = int(c["addition_time_embed_dim"])
            self.add_embedding = nn.Module()
            self.add_embedding.linear_1 = nn.Linear(int(c["projection_class_embeddings_input_dim"]), temb)
            self.add_embedding.linear_2 = nn.Linear(temb, temb)
        elif c.get("addition_embed_type"):
            raise ValueError(f"unsupported UNet addition_embed_type {c.get('addition_embed_type')!r}")
        downs, prev = [], ch[0]
        for i, t in enumerate(c["down_block_types"]):
            b = nn.Module()
            b.resnets = nn.ModuleList(_Resnet(prev if j == 0 else ch[i], ch[i], g, eps, temb) for j in range(lpb))
            if "CrossAttn" in t:
                b.attentions = nn.ModuleList(_Transformer2D(ch[i], heads[i], ctx, g, lin, depth[i]) for _ in range(lpb))
            if i < n - 1:
                b.downsamplers = nn.ModuleList([_Down(ch[i])])
            downs.append(b)
            prev = ch[i]
        self.down_blocks = nn.ModuleList(downs)
        self.mid_block = nn.Module()
        self.mid_block.resnets = nn.ModuleList([_Resnet(ch[-1], ch[-1], g, eps, temb) for _ in range(2)])
        self.mid_block.attentions = nn.ModuleList([_Transformer2D(ch[-1], heads[-1], ctx, g, lin, depth[-1])])
        rch, rheads = ch[::-1], heads[::-1]
        rdep = _per_block(rdepth, n) if rdepth is not None else depth[::-1]
        ups, prev = [], ch[-1]
        for i, t in enumerate(c["up_block_types"]):
            out, skip_in = rch[i], rch[min(i + 1, n - 1)]
            b = nn.Module()
            b.resnets = nn.ModuleList(
                _Resnet((prev if j == 0 else out) + (skip_in if j == lpb else out), out, g, eps, temb)
                for j in range(lpb + 1))
            if "CrossAttn" in t:
                b.attentions = nn.ModuleList(_Transformer2D(out, rheads[i], ctx, g, lin, rdep[i]) for _ in range(lpb + 1))
            if i < n - 1:
                b.upsamplers = nn.ModuleList([_Up(out)])
            ups.append(b)
            prev = out
        self.up_blocks = nn.ModuleList(ups)
        self.conv_norm_out = nn.GroupNorm(g, ch[0], eps=eps)
        self.conv_out = nn.Conv2d(ch[0], c.get("out_channels", 4), 3, padding=1)
        self.ch0 = ch[0]

    def _tproj(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        half = (dim or self.ch0) // 2
        f = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - self.shift))
        e = t.float()[:, None] * f[None]
        e = torch.cat([torch.cos(e), torch.sin(e)] if self.flip else [torch.sin(e), torch.cos(e)], dim=-1)
        return e

    def _temb(self, x, t, text_embeds=None, time_ids=None):
        temb = self._tproj(t).to(x.dtype)
        temb = self.time_embedding.linear_2(F.silu(self.time_embedding.linear_1(temb)))
        if self.text_time:
            if text_embeds is None or time_ids is None:
                raise ValueError("this UNet (SDXL) needs text_embeds and time_ids")
            B = x.shape[0]
            tid = self._tproj(time_ids.reshape(-1), self.add_time_dim).reshape(B, -1)
            a = torch.cat([text_embeds.to(x.dtype), tid.to(x.dtype)], dim=-1)
            temb = temb + self.add_embedding.linear_2(F.silu(self.add_embedding.linear_1(a)))
        return temb

    def _down_mid(self, h, temb, ctx):
        """conv_in output -> (mid-block output, skip tensors of the down path)."""
        skips = [h]
        for b in self.down_blocks:
            for j, r in enumerate(b.resnets):
                h = r(h, temb)
                if hasattr(b, "attentions"):
                    h = b.attentions[j](h, ctx)
                skips.append(h)
            if hasattr(b, "downsamplers"):
                h = b.downsamplers[0](h)
                skips.append(h)
        m = self.mid_block
        h = m.attentions[0](m.resnets[0](h, temb), ctx)
        return m.resnets[1](h, temb), skips

    def forward(self, x, t, ctx, text_embeds=None, time_ids=None, down_res=None, mid_res=None):
        """down_res / mid_res: ControlNet residuals added to the skips / the mid-block output
        (diffusers' down_block_additional_residuals / mid_block_additional_residual)."""
        temb = self._temb(x, t, text_embeds, time_ids)
        h, skips = self._down_mid(self.conv_in(x), temb, ctx)
        if down_res is not None:
            skips = [s_ + r_ for s_, r_ in zip(skips, down_res)]
        if mid_res is not None:
            h = h + mid_res
        for b in self.up_blocks:
            for j, r in enumerate(b.resnets):
                h = r(torch.cat([h, skips.pop()], dim=1), temb)
                if hasattr(b, "attentions"):
                    h = b.attentions[j](h, ctx)
            if hasattr(b, "upsamplers"):
                h = b.upsamplers[0](h, skips[-1].shape[-2:] if skips else None)
        return self.conv_out(_gn(self.conv_norm_out, h, True))


class ControlNet(UNet):
    """diffusers ControlNetModel: the UNet's encoder half (conv_in, time embedding, down blocks,
    mid block -- named like the UNet's) plus a conditioning-image embedding added after conv_in
    and zero-initialised 1x1 convolutions that turn every skip and the mid output into residuals
    for the UNet (reference: `backend/python/diffusers/backend.py:292-296`, ControlNetModel with
    the control image as `image`)."""

    def __init__(self, c: dict):
        n = len(c["block_out_channels"])
        super().__init__(dict(c, up_block_types=c.get("up_block_types") or ["UpBlock2D"] * n))
        del self.up_blocks, self.conv_norm_out, self.conv_out
        ch = list(c["block_out_channels"])
        lpb = int(c.get("layers_per_block", 2))
        emb = list(c.get("conditioning_embedding_out_channels") or [16, 32, 96, 256])
        self.bgr = str(c.get("controlnet_conditioning_channel_order", "rgb")) == "bgr"
        ce = nn.Module()
        ce.conv_in = nn.Conv2d(int(c.get("conditioning_channels", 3)), emb[0], 3, padding=1)
        ce.blocks = nn.ModuleList()
        for i in range(len(emb) - 1):
            ce.blocks.append(nn.Conv2d(emb[i], emb[i], 3, padding=1))
            ce.blocks.append(nn.Conv2d(emb[i], emb[i + 1], 3, padding=1, stride=2))
        ce.conv_out = nn.Conv2d(emb[-1], ch[0], 3, padding=1)
        self.controlnet_cond_embedding = ce
        skip_ch = [ch[0]]
        for i in range(n):
            skip_ch += [ch[i]] * lpb + ([ch[i]] if i < n - 1 else [])
        self.controlnet_down_blocks = nn.ModuleList(nn.Conv2d(k, k, 1) for k in skip_ch)
        self.controlnet_mid_block = nn.Conv2d(ch[-1], ch[-1], 1)

    def forward(self, x, t, ctx, cond, scale: float = 1.0, text_embeds=None, time_ids=None):
        """cond: the control image in [0, 1], [B, 3, 8h, 8w] -> (skip residuals, mid residual)."""
        temb = self._temb(x, t, text_embeds, time_ids)
        ce = self.controlnet_cond_embedding
        if self.bgr:
            cond = cond.flip(1)
        e = F.silu(ce.conv_in(cond))
        for blk in ce.blocks:
            e = F.silu(blk(e))
        h = self.conv_in(x) + ce.conv_out(e)
        h, skips = self._down_mid(h, temb, ctx)
        down = [conv(s_) * scale for conv, s_ in zip(self.controlnet_down_blocks, skips)]
        return down, self.controlnet_mid_block(h) * scale


class _VaeAttn(nn.Module):
    def __init__(self, c: int, groups: int, eps: float):
        super().__init__()
        self.group_norm = nn.GroupNorm(groups, c, eps=eps)
        self.to_q, self.to_k, self.to_v = nn.Linear(c, c), nn.Linear(c, c), nn.Linear(c, c)
        self.to_out = nn.ModuleList([nn.Linear(c, c)])

    def forward(self, x):
        B, C, H, W = x.shape
        h = _gn(self.group_norm, x).reshape(B, C, H * W).transpose(1, 2)
        q, k, v = (p(h)[:, None] for p in (self.to_q, self.to_k, self.to_v))
        o = F.scaled_dot_product_attention(q, k, v)[:, 0]
        return x + self.to_out[0](o).transpose(1, 2).reshape(B, C, H, W)


class VaeDecoder(nn.Module):
    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        lpb = int(c.get("layers_per_block", 2))
        g = int(c.get("norm_num_groups", 32))
        lat = int(c.get("latent_channels", 4))
        self.scaling = float(c.get("scaling_factor", 0.18215))
        self.shift = float(c.get("shift_factor") or 0.0)   # FLUX / SD3 VAEs: z / scaling + shift
        # FLUX / SD3 VAEs have no post-quant convolution (use_post_quant_conv: false)
        self.post_quant_conv = nn.Conv2d(lat, lat, 1) if c.get("use_post_quant_conv", True) else nn.Identity()
        d = nn.Module()
        d.conv_in = nn.Conv2d(lat, ch[-1], 3, padding=1)
        d.mid_block = nn.Module()
        d.mid_block.resnets = nn.ModuleList([_Resnet(ch[-1], ch[-1], g, 1e-6, None) for _ in range(2)])
        d.mid_block.attentions = nn.ModuleList([_VaeAttn(ch[-1], g, 1e-6)])
        rch, ups, prev = ch[::-1], [], ch[-1]
        for i in range(len(ch)):
            b = nn.Module()
            b.resnets = nn.ModuleList(_Resnet(prev if j == 0 else rch[i], rch[i], g, 1e-6, None) for j in range(lpb + 1))
            if i < len(ch) - 1:
                b.upsamplers = nn.ModuleList([_Up(rch[i])])
            ups.append(b)
            prev = rch[i]
        d.up_blocks = nn.ModuleList(ups)
        d.conv_norm_out = nn.GroupNorm(g, ch[0], eps=1e-6)
        d.conv_out = nn.Conv2d(ch[0], c.get("out_channels", 3), 3, padding=1)
        self.decoder = d

    def forward(self, z):
        d = self.decoder
        h = d.conv_in(self.post_quant_conv(z / self.scaling + self.shift))
        h = d.mid_block.resnets[1](d.mid_block.attentions[0](d.mid_block.resnets[0](h)))
        for b in d.up_blocks:
            for r in b.resnets:
                h = r(h)
            if hasattr(b, "upsamplers"):
                h = b.upsamplers[0](h)
        return d.conv_out(_gn(d.conv_norm_out, h, True))


class VaeEncoder(nn.Module):
    """KL-VAE encoder (img2img): conv stem, DownEncoderBlock2D stages (right/bottom-padded stride-2
    convs), mid block, then the latent distribution's mean / log-variance through quant_conv."""

    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        lpb = int(c.get("layers_per_block", 2))
        g = int(c.get("norm_num_groups", 32))
        lat = int(c.get("latent_channels", 4))
        self.scaling = float(c.get("scaling_factor", 0.18215))
        e = nn.Module()
        e.conv_in = nn.Conv2d(c.get("in_channels", 3), ch[0], 3, padding=1)
        downs, prev = [], ch[0]
        for i in range(len(ch)):
            b = nn.Module()
            b.resnets = nn.ModuleList(_Resnet(prev if j == 0 else ch[i], ch[i], g, 1e-6, None) for j in range(lpb))
            if i < len(ch) - 1:
                b.downsamplers = nn.ModuleList([_Down(ch[i], pad=0)])
            downs.append(b)
            prev = ch[i]
        e.down_blocks = nn.ModuleList(downs)
        e.mid_block = nn.Module()
        e.mid_block.resnets = nn.ModuleList([_Resnet(ch[-1], ch[-1], g, 1e-6, None) for _ in range(2)])
        e.mid_block.attentions = nn.ModuleList([_VaeAttn(ch[-1], g, 1e-6)])
        e.conv_norm_out = nn.GroupNorm(g, ch[-1], eps=1e-6)
        e.conv_out = nn.Conv2d(ch[-1], 2 * lat, 3, padding=1)
        self.encoder = e
        self.quant_conv = nn.Conv2d(2 * lat, 2 * lat, 1) if c.get("use_quant_conv", True) else nn.Identity()
        self.shift = float(c.get("shift_factor") or 0.0)

    def forward(self, img: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        """img [B, 3, H, W] in [-1, 1] -> scaled latents (a sample of the latent distribution)."""
        e = self.encoder
        h = e.conv_in(img)
        for b in e.down_blocks:
            for r in b.resnets:
                h = r(h)
            if hasattr(b, "downsamplers"):
                h = b.downsamplers[0](h)
        h = e.mid_block.resnets[1](e.mid_block.attentions[0](e.mid_block.resnets[0](h)))
        m = self.quant_conv(e.conv_out(_gn(e.conv_norm_out, h, True))).float()
        mean, logvar = m.chunk(2, dim=1)
        std = torch.exp(0.5 * logvar.clamp(-30.0, 20.0))
        eps = torch.randn(mean.shape, generator=gen).to(mean.device)
        return (mean + std * eps - self.shift) * self.scaling


def _vae_enc_names(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    ren = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}
    out = {}
    for k, v in sd.items():
        if not (k.startswith("encoder.") or k.startswith("quant_conv.")):
            continue
        for a, b in ren.items():
            k = k.replace(a, b)
        if ".attentions." in k and k.endswith(".weight") and v.dim() == 4:
            v = v[:, :, 0, 0]
        out[k] = v
    return out


def _vae_names(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Decoder tensors only; older VAE checkpoints name the attention `query/key/value/proj_attn`
    and store them as 1x1 convolutions."""
    ren = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}
    out = {}
    for k, v in sd.items():
        if not (k.startswith("decoder.") or k.startswith("post_quant_conv.")):
            continue
        for a, b in ren.items():
            k = k.replace(a, b)
        if ".attentions." in k and k.endswith(".weight") and v.dim() == 4:
            v = v[:, :, 0, 0]
        out[k] = v
    return out


# ------------------------------------------------------------------ schedulers
class Scheduler:
    """DDIM (eta 0) or Euler-discrete over the scaled-linear beta schedule, "leading" spacing."""

    def __init__(self, c: dict, kind: str = "ddim"):
        n = int(c.get("num_train_timesteps", 1000))
        b0, b1 = float(c.get("beta_start", 0.00085)), float(c.get("beta_end", 0.012))
        if c.get("beta_schedule", "scaled_linear") == "linear":
            betas = torch.linspace(b0, b1, n, dtype=torch.float64)
        else:
            betas = torch.linspace(b0 ** 0.5, b1 ** 0.5, n, dtype=torch.float64) ** 2
        self.ac = torch.cumprod(1.0 - betas, 0)
        self.n_train = n
        self.offset = int(c.get("steps_offset", 1))
        self.final_ac = 1.0 if c.get("set_alpha_to_one", False) else float(self.ac[0])
        self.pred = c.get("prediction_type", "epsilon")
        self.kind = kind if kind in ("ddim", "euler") else "ddim"

    def timesteps(self, steps: int) -> List[int]:
        r = self.n_train // steps
        return [i * r + self.offset for i in range(steps)][::-1]

    def init_sigma(self, ts: Sequence[int]) -> float:
        if self.kind == "euler":
            a = float(self.ac[ts[0]])
            return math.sqrt((1 - a) / a + 1)  # x_T = x0 + sigma * eps has variance sigma^2 + 1
        return 1.0

    def scale_input(self, x: torch.Tensor, t: int) -> torch.Tensor:
        if self.kind == "euler":
            a = float(self.ac[t])
            return x / math.sqrt((1 - a) / a + 1)
        return x

    def _x0_eps(self, out, x, a):
        if self.pred == "v_prediction":
            x0 = math.sqrt(a) * x - math.sqrt(1 - a) * out
            return x0, math.sqrt(a) * out + math.sqrt(1 - a) * x
        return (x - math.sqrt(1 - a) * out) / math.sqrt(a), out

    def step(self, out: torch.Tensor, t: int, t_prev: Optional[int], x: torch.Tensor) -> torch.Tensor:
        a = float(self.ac[t])
        a_prev = float(self.ac[t_prev]) if t_prev is not None else self.final_ac
        if self.kind == "euler":
            # latents carry sigma scaling: x = x0 + sigma * eps, with x0 / eps from the model
            s, s_prev = math.sqrt((1 - a) / a), (math.sqrt((1 - a_prev) / a_prev) if t_prev is not None else 0.0)
            x0, eps = self._x0_eps(out, x / math.sqrt(s * s + 1), a)
            return x0 + s_prev * eps if t_prev is not None else x0
        x0, eps = self._x0_eps(out, x, a)
        return math.sqrt(a_prev) * x0 + math.sqrt(1 - a_prev) * eps


# ------------------------------------------------------------------ pipeline
class StableDiffusion:
    def __init__(self, path: str, device: str = "cpu", scheduler: str = "", clip_skip: int = 0,
                 channels_last: Optional[bool] = None, controlnet: str = "", controlnet_scale: float = 1.0,
                 lora: str = "", lora_scale: float = 1.0, deterministic: Optional[bool] = None):
        self.device = torch.device(device)
        # MIOpen's default convolution solvers are not bitwise reproducible run to run (a 1-ulp
        # difference in a bf16 conv output, scripts/determinism_probe.py); deterministic=True (or
        # LOCALAI_AMD_SD_DETERMINISTIC=1) restricts the convolutions -- eager and captured -- to
        # deterministic solvers: identical images for identical requests, ~1.8x the UNet time on
        # the toy shapes measured
        if deterministic is None:
            deterministic = os.environ.get("LOCALAI_AMD_SD_DETERMINISTIC", "0") == "1"
        self.deterministic = bool(deterministic)
        # NHWC activations for the MIOpen convolutions (LOCALAI_AMD_SD_NHWC=0 keeps NCHW)
        if channels_last is None:
            channels_last = os.environ.get("LOCALAI_AMD_SD_NHWC", "1") != "0"
        self.channels_last = channels_last and self.device.type == "cuda"
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.clip_skip = clip_skip
        self.text = self._load_text(os.path.join(path, "text_encoder"))
        # SDXL: a second (OpenCLIP bigG, projected) text encoder; prompt embeddings are the two
        # encoders' penultimate states side by side, the pooled projection conditions add_embedding
        self.xl = os.path.isdir(os.path.join(path, "text_encoder_2"))
        self.text2 = self._load_text(os.path.join(path, "text_encoder_2")) if self.xl else None
        mi = os.path.join(path, "model_index.json")
        self.zero_neg = bool((_cfg(mi) if os.path.isfile(mi) else {}).get("force_zeros_for_empty_prompt", True))
        ucfg = _cfg(os.path.join(path, "unet", "config.json"))
        self.unet_sample_size = int(ucfg.get("sample_size", 64))
        self.unet = UNet(ucfg)
        self.unet.load_state_dict(_load_weights(os.path.join(path, "unet")), strict=True)
        vcfg = _cfg(os.path.join(path, "vae", "config.json"))
        vae_sd = _load_weights(os.path.join(path, "vae"))
        self.vae = VaeDecoder(vcfg)
        self.vae.load_state_dict(_vae_names(vae_sd), strict=True)
        enc = _vae_enc_names(vae_sd)
        self.vae_enc = None
        if enc:  # img2img needs the encoder half (decoder-only VAE checkpoints stay txt2img)
            self.vae_enc = VaeEncoder(vcfg)
            self.vae_enc.load_state_dict(enc, strict=True)
            self.vae_enc.to(self.device, self.dtype).eval().requires_grad_(False)
        # ControlNet (diffusers ControlNetModel directory: config.json + weights)
        self.controlnet = None
        self.cn_scale = float(controlnet_scale)
        if controlnet:
            self.controlnet = ControlNet(_cfg(os.path.join(controlnet, "config.json")))
            self.controlnet.load_state_dict(_load_weights(controlnet), strict=True)
        if lora:  # LoraAdapter: merged in fp32 before the cast (models/sd_lora.py)
            from .sd_lora import merge_sd_lora
            merge_sd_lora(lora, self.unet, self.text, self.text2, lora_scale)
        for m in (self.text, self.text2, self.unet, self.vae, self.controlnet):
            if m is not None:
                m.to(self.device, self.dtype).eval().requires_grad_(False)
        if self.xl and not self.unet.text_time:
            raise ValueError("SDXL pipeline (text_encoder_2) with a UNet lacking text_time conditioning")
        if self.channels_last:
            self.unet.to(memory_format=torch.channels_last)
            self.vae.to(memory_format=torch.channels_last)
            if self.controlnet is not None:
                self.controlnet.to(memory_format=torch.channels_last)
        sc = os.path.join(path, "scheduler", "scheduler_config.json")
        self.sched_cfg = _cfg(sc) if os.path.isfile(sc) else {}
        from .schedulers import PLMS, KSampler, parse_name
        self.sched_name, karras = parse_name(scheduler or "ddim")
        self.sched = Scheduler(self.sched_cfg, "ddim")
        self.ksampler = KSampler(self.sched_cfg, scheduler) if self.sched_name not in ("ddim", "pndm") else None
        self.plms = PLMS(self.sched_cfg) if self.sched_name == "pndm" else None
        self.pred = self.sched_cfg.get("prediction_type", "epsilon")
        from transformers import CLIPTokenizer
        self.tok = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer"))
        self.tok2 = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer_2")) if self.xl else None
        self.max_len = self.text.text_model.embeddings.position_embedding.weight.shape[0]
        # latent channels come from the VAE; a depth2img UNet takes one more (the depth map)
        self.latent_ch = int(vcfg.get("latent_channels", self.unet.conv_in.in_channels))
        self.extra_ch = self.unet.conv_in.in_channels - self.latent_ch
        # StableDiffusionDepth2ImgPipeline (backend.py:196-198): a DPT depth estimator and its
        # image processor beside the UNet; the estimated depth of the source image, resized to the
        # latent grid and scaled to [-1, 1], is concatenated to every UNet input
        self.depth = self.depth_fe = None
        de = os.path.join(path, "depth_estimator")
        if os.path.isdir(de):
            import transformers as tf
            self.depth = tf.DPTForDepthEstimation.from_pretrained(de).to(self.device, self.dtype).eval()
            fe = os.path.join(path, "feature_extractor")
            self.depth_fe = (tf.DPTImageProcessor.from_pretrained(fe) if os.path.isdir(fe) else
                             tf.DPTImageProcessor(size={"height": 384, "width": 384}, keep_aspect_ratio=False))
        if self.extra_ch != (1 if self.depth is not None else 0):
            raise ValueError(f"UNet takes {self.unet.conv_in.in_channels} input channels for {self.latent_ch} latent "
                             "channels: only depth2img (one extra channel, with a depth_estimator) is supported")
        # one hipGraph per (batch, latent size) replays the whole UNet step (~1300 launches)
        self.use_graphs = self.device.type == "cuda" and os.environ.get("LOCALAI_AMD_SD_GRAPH", "1") != "0"
        # bounded LRU: every captured graph owns its activation pool, so a stream of distinct image
        # sizes must not grow device memory without limit
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.graph_cache = max(0, int(os.environ.get("LOCALAI_AMD_SD_GRAPH_CACHE", "4")))
        self.vae_scale = 2 ** (len(self.vae.decoder.up_blocks) - 1)

    @staticmethod
    def _load_text(d: str) -> ClipTextEncoder:
        te = ClipTextEncoder(_cfg(os.path.join(d, "config.json")))
        # transformers 4 keeps the `text_model.` prefix, transformers 5 drops it
        te.load_state_dict({(k if k.startswith(("text_model.", "text_projection")) else "text_model." + k): v
                            for k, v in _load_weights(d).items() if "position_ids" not in k}, strict=True)
        return te

    def _model(self, x, t, ctx, te=None, ti=None, cond=None):
        """One denoiser evaluation: ControlNet residuals (when a control image is given) + UNet."""
        dr = mr = None
        if cond is not None:
            dr, mr = self.controlnet(x, t, ctx, cond, self.cn_scale, te, ti)
        return self.unet(x, t, ctx, te, ti, dr, mr)

    def _unet(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, add=None, cond=None) -> torch.Tensor:
        """add: SDXL (text_embeds, time_ids) or None; cond: ControlNet image or None.  On the GPU
        the whole step (ControlNet + UNet, ~1300 launches) replays from one hipGraph per input
        shape set, kept in a bounded LRU (each graph owns its activation pool)."""
        te, ti = add if add is not None else (None, None)
        ins = (x, t, ctx, te, ti, cond)
        if not self.use_graphs:
            return self._model(*ins)
        key = tuple(None if v is None else tuple(v.shape) for v in ins)
        g = self._graphs.get(key)
        if g is None:
            out = self._model(*ins)  # eager first call: kernel selection / workspaces happen outside capture
            if self.graph_cache == 0:
                return out
            while len(self._graphs) >= self.graph_cache:
                _, old = self._graphs.popitem(last=False)   # least recently used shape set
                del old
                torch.cuda.empty_cache()
            try:
                st = tuple(None if v is None else v.clone() for v in ins)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    so = self._model(*st)
                self._graphs[key] = (graph, st, so)
            except Exception as e:  # noqa: BLE001 - capture is an optimisation; eager stays correct
                import logging
                logging.getLogger(__name__).warning("sd: UNet graph capture failed (%r); running eager", e)
                self.use_graphs = False
            return out
        self._graphs.move_to_end(key)
        graph, st, so = g
        for dst, src in zip(st, ins):
            if dst is not None:
                dst.copy_(src)
        graph.replay()
        return so.clone()

    def _encode(self, prompts: List[str]) -> torch.Tensor:
        ids = self.tok(prompts, padding="max_length", max_length=self.max_len, truncation=True,
                       return_tensors="pt").input_ids.to(self.device)
        return self.text(ids, self.clip_skip)

    def _encode_xl(self, prompts: List[str]):
        """SDXL: (prompt embeds [B, 77, d1 + d2], pooled projection [B, p]); an empty prompt is all
        zeros when the pipeline sets force_zeros_for_empty_prompt (diffusers encode_prompt)."""
        outs = []
        for tok, te, pooled in ((self.tok, self.text, False), (self.tok2, self.text2, True)):
            ids = tok(prompts, padding="max_length", max_length=self.max_len, truncation=True,
                      return_tensors="pt").input_ids.to(self.device)
            outs.append(te.sdxl(ids, self.clip_skip, pooled))
        ctx = torch.cat([outs[0][0], outs[1][0]], dim=-1)
        pool = outs[1][1]
        if self.zero_neg:
            for i, p in enumerate(prompts):
                if p == "" and len(prompts) > 1 and i == 0:  # the negative branch of CFG
                    ctx[i] = 0
                    pool[i] = 0
        return ctx, pool

    def _eps(self, x: torch.Tensor, t: float, ctx: torch.Tensor, cfg: bool, guidance_scale: float,
             add=None, cond=None) -> torch.Tensor:
        """Model output (eps or v) at timestep t with classifier-free guidance as one batch of 2."""
        xin = torch.cat([x, x]) if cfg else x
        tt = torch.full((xin.shape[0],), float(t), device=self.device)
        xin = xin.to(self.dtype)
        if self._depth_map is not None:
            xin = torch.cat([xin, self._depth_map.expand(xin.shape[0], -1, -1, -1)], dim=1)
        if self.channels_last:
            xin = xin.contiguous(memory_format=torch.channels_last)
        out = self._unet(xin, tt, ctx, add, cond).float()
        if cfg:
            u, c = out.chunk(2)
            out = u + guidance_scale * (c - u)
        return out

    _depth_map = None

    @torch.no_grad()
    def _estimate_depth(self, image, w: int, h: int) -> torch.Tensor:
        """diffusers StableDiffusionDepth2ImgPipeline.prepare_depth_map: DPT depth of the source,
        bicubic to the latent grid, min/max-scaled to [-1, 1] -> [1, 1, h, w]."""
        from PIL import Image
        im = image if isinstance(image, Image.Image) else Image.open(image)
        px = self.depth_fe(images=im.convert("RGB"), return_tensors="pt").pixel_values.to(self.device, self.dtype)
        d = self.depth(pixel_values=px).predicted_depth.float()
        d = F.interpolate(d.unsqueeze(1), size=(h, w), mode="bicubic", align_corners=False)
        lo, hi = d.amin(dim=[1, 2, 3], keepdim=True), d.amax(dim=[1, 2, 3], keepdim=True)
        d = 2.0 * (d - lo) / (hi - lo).clamp_min(1e-12) - 1.0
        return d.to(self.dtype)

    def _init_latents(self, image, w: int, h: int, g: torch.Generator) -> torch.Tensor:
        """img2img source -> scaled latents of the requested size."""
        from PIL import Image
        if self.vae_enc is None:
            raise ValueError("this VAE checkpoint has no encoder: img2img is unavailable")
        im = image if isinstance(image, Image.Image) else Image.open(image)
        im = im.convert("RGB").resize((w * self.vae_scale, h * self.vae_scale), Image.BICUBIC)
        a = torch.from_numpy(np.asarray(im, dtype=np.float32)).permute(2, 0, 1)[None] / 127.5 - 1.0
        a = a.to(self.device, self.dtype)
        if self.channels_last:
            a = a.contiguous(memory_format=torch.channels_last)
        return self.vae_enc(a, g).float()

    def _control_image(self, image, W: int, H: int, batch: int) -> torch.Tensor:
        """ControlNet conditioning image -> [batch, 3, H, W] in [0, 1] (diffusers'
        control_image_processor: RGB, resized to the output size, not normalised)."""
        from PIL import Image
        im = image if isinstance(image, Image.Image) else Image.open(image)
        im = im.convert("RGB").resize((W, H), Image.LANCZOS)
        a = torch.from_numpy(np.asarray(im, dtype=np.float32) / 255.0).permute(2, 0, 1)[None]
        a = a.expand(batch, -1, -1, -1).to(self.device, self.dtype)
        return a.contiguous(memory_format=torch.channels_last) if self.channels_last else a.contiguous()

    def __call__(self, *args, **kw) -> torch.Tensor:
        if not self.deterministic:
            return self._call(*args, **kw)
        with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
            return self._call(*args, **kw)

    @torch.no_grad()
    def _call(self, prompt: str, negative_prompt: str = "", width: int = 512, height: int = 512,
              steps: int = 1, guidance_scale: float = 7.0, seed: Optional[int] = None,
              image=None, strength: float = 0.8, control_image=None) -> torch.Tensor:
        """-> uint8 image [H, W, 3] on the CPU.  `image` (a path or PIL image) turns the call into
        img2img: its latents are noised to `strength` of the schedule and denoised from there.
        `control_image` conditions every step through the ControlNet (pipelines loaded with one)."""
        if control_image is not None and self.controlnet is None:
            raise ValueError("control_image given but no ControlNet is loaded")
        g = torch.Generator().manual_seed(seed if seed is not None else int.from_bytes(os.urandom(4), "little"))
        if image is not None and not (width and height):
            from PIL import Image
            im = image if isinstance(image, Image.Image) else Image.open(image)
            width, height = im.size
        h, w = max(1, height // self.vae_scale), max(1, width // self.vae_scale)
        cfg = guidance_scale > 1.0
        prompts = [negative_prompt, prompt] if cfg else [prompt]
        add = None
        if self.xl:
            ctx, pool = self._encode_xl(prompts)
            H, W = h * self.vae_scale, w * self.vae_scale   # original = target size, no crop
            tid = torch.tensor([[H, W, 0, 0, H, W]] * len(prompts), dtype=torch.float32, device=self.device)
            add = (pool, tid)
        else:
            ctx = self._encode(prompts)
        cond = None
        if control_image is not None:
            cond = self._control_image(control_image, w * self.vae_scale, h * self.vae_scale, len(prompts))
        steps = max(1, steps)
        if self.depth is not None:
            if image is None:
                raise ValueError("a depth2img pipeline needs a source image (src)")
            self._depth_map = self._estimate_depth(image, w, h)
        x0 = self._init_latents(image, w, h, g) if image is not None else None
        # img2img: skip the first (1 - strength) of the schedule (diffusers get_timesteps)
        skip = max(steps - min(int(steps * strength), steps), 0) if x0 is not None else 0
        noise = torch.randn(1, self.latent_ch, h, w, generator=g).to(self.device)
        if x0 is not None and skip >= steps:
            x = x0                                 # strength 0: nothing to denoise
        elif self.ksampler is not None:
            ks = self.ksampler
            sig = ks.sigmas(steps)[skip:]
            x = noise * sig[0] if x0 is None else x0 + noise * sig[0]

            def denoise(xv, sigma):
                c_in = 1.0 / math.sqrt(sigma * sigma + 1.0)
                out = self._eps(xv * c_in, ks.sched.sigma_to_t(sigma), ctx, cfg, guidance_scale, add, cond)
                if self.pred == "v_prediction":
                    return xv / (sigma * sigma + 1.0) - out * (sigma * c_in)
                return xv - sigma * out
            x = ks.sample(denoise, x, sig, g)
        elif self.plms is not None:
            ts = self.plms.timesteps(steps)
            self.plms.reset(steps)
            ts = ts[skip:] if skip else ts
            x = noise if x0 is None else self._add_noise(x0, noise, ts[0])
            for t in ts:
                x = self.plms.step(self._eps(x, t, ctx, cfg, guidance_scale, add, cond), t, x)
        else:
            ts = self.sched.timesteps(steps)[skip:]
            x = noise if x0 is None else self._add_noise(x0, noise, ts[0])
            for i, t in enumerate(ts):
                out = self._eps(x, t, ctx, cfg, guidance_scale, add, cond)
                x = self.sched.step(out, t, ts[i + 1] if i + 1 < len(ts) else None, x)
        self._depth_map = None
        img = self.vae(x.to(self.dtype)).float()
        img = ((img[0] / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)
        return img.permute(1, 2, 0).cpu()

    def _add_noise(self, x0: torch.Tensor, noise: torch.Tensor, t: int) -> torch.Tensor:
        a = float(self.sched.ac[t])
        return math.sqrt(a) * x0 + math.sqrt(1 - a) * noise

    def save(self, img: torch.Tensor, dst: str):
        from PIL import Image
        Image.fromarray(img.numpy()).save(dst)
