"""Image-to-video diffusion (Stable Video Diffusion), served by the `diffusers` backend for
`pipeline_type: StableVideoDiffusionPipeline` (reference: `backend/python/diffusers/backend.py:199-205`
loads the pipeline; `:435-443` resizes `src` to 1024 x 576, calls it with `guidance_scale`
(max guidance), `decode_chunk_size = CHUNK_SIZE` (8) and a seeded generator, and writes the frames
with export_to_video at `FPS` (7)).

Reads the diffusers directory layout (`model_index.json` with `_class_name:
StableVideoDiffusionPipeline`, `unet/` UNetSpatioTemporalConditionModel, `vae/`
AutoencoderKLTemporalDecoder, `image_encoder/` CLIPVisionModelWithProjection, `scheduler/`
EulerDiscreteScheduler).  Modules are named like the checkpoint's tensors (strict loads):

* SpatioTemporalResBlock: the 2-D ResNet block per frame, then a temporal ResNet block ((3, 1, 1)
  Conv3d, time embedding per frame), mixed by a learned AlphaBlender (sigmoid(mix_factor));
* TransformerSpatioTemporalModel: the spatial transformer block per frame (cross-attention to the
  CLIP image embedding), then per pixel a temporal transformer block over the frames (GEGLU
  ff_in, self-attention, cross-attention to the first frame's context, GEGLU ff) on the frame-
  index position embedding, mixed by another AlphaBlender;
* conditioning: the CLIP image embedding (encoder_hidden_states), the noise-augmented image's VAE
  latent concatenated to every frame's noisy latent (8 input channels), and the added time ids
  (fps - 1, motion_bucket_id, noise_aug_strength) through add_embedding;
* EulerDiscrete sampling on Karras sigmas with v-prediction and continuous timesteps
  (t = log(sigma) / 4), classifier-free guidance ramped linearly over the frames
  (min_guidance_scale 1 -> max_guidance_scale);
* the temporal VAE decoder (spatio-temporal ResNets in the mid / up blocks, a (3, 1, 1) Conv3d on
  the output) decoding `decode_chunk_size` frames at a time.

The CLIP vision tower runs through transformers (CLIPVisionModelWithProjection).  Parity with
diffusers is unpinned (diffusers is not installed).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .sd import _Attn, _cfg, _Down, _GEGLU, _load_weights, _per_block, _Up, _VaeAttn, _vae_enc_names, VaeEncoder


def is_svd_pipeline(path: str) -> bool:
    mi = os.path.join(path, "model_index.json")
    if not os.path.isfile(mi):
        return False
    try:
        return _cfg(mi).get("_class_name") == "StableVideoDiffusionPipeline"
    except (OSError, ValueError):
        return False


def _tproj(t: torch.Tensor, dim: int) -> torch.Tensor:
    """diffusers Timesteps(dim, flip_sin_to_cos=True, downscale_freq_shift=0)."""
    half = dim // 2
    f = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / half)
    e = t.float()[:, None] * f[None]
    return torch.cat([torch.cos(e), torch.sin(e)], dim=-1)


class _TEmb(nn.Module):
    """diffusers TimestepEmbedding: linear_1, SiLU, linear_2."""

    def __init__(self, cin: int, dim: int, out: Optional[int] = None):
        super().__init__()
        self.linear_1, self.linear_2 = nn.Linear(cin, dim), nn.Linear(dim, out or dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class _Blend(nn.Module):
    """AlphaBlender, learned strategies (no image-only frames at inference):
    alpha = sigmoid(mix_factor), 1 - alpha when switch_spatial_to_temporal_mix."""

    def __init__(self, alpha: float, switch: bool):
        super().__init__()
        self.mix_factor = nn.Parameter(torch.tensor([alpha]))
        self.switch = switch

    def forward(self, spatial, temporal):
        a = torch.sigmoid(self.mix_factor.float()).to(spatial.dtype)
        if self.switch:
            a = 1.0 - a
        return a * spatial + (1.0 - a) * temporal


class _Res2D(nn.Module):
    """ResnetBlock2D (time embedding optional); PyTorch GroupNorm (the SVD blocks mix layouts)."""

    def __init__(self, cin: int, cout: int, temb: Optional[int], eps: float, groups: int = 32):
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
        h = self.conv1(F.silu(self.norm1(x)))
        if temb is not None and hasattr(self, "time_emb_proj"):
            h = h + self.time_emb_proj(F.silu(temb))[:, :, None, None]
        h = self.conv2(F.silu(self.norm2(h)))
        return (self.conv_shortcut(x) if hasattr(self, "conv_shortcut") else x) + h


class _ResT(nn.Module):
    """TemporalResnetBlock: (3, 1, 1) convolutions over [B, C, F, H, W]."""

    def __init__(self, c: int, temb: Optional[int], eps: float, groups: int = 32):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, c, eps=eps)
        self.conv1 = nn.Conv3d(c, c, (3, 1, 1), padding=(1, 0, 0))
        if temb:
            self.time_emb_proj = nn.Linear(temb, c)
        self.norm2 = nn.GroupNorm(groups, c, eps=eps)
        self.conv2 = nn.Conv3d(c, c, (3, 1, 1), padding=(1, 0, 0))

    def forward(self, x, temb=None):
        h = self.conv1(F.silu(self.norm1(x)))
        if temb is not None and hasattr(self, "time_emb_proj"):
            h = h + self.time_emb_proj(F.silu(temb)).permute(0, 2, 1)[:, :, :, None, None]   # [B, C, F, 1, 1]
        h = self.conv2(F.silu(self.norm2(h)))
        return x + h


class _STRes(nn.Module):
    """SpatioTemporalResBlock."""

    def __init__(self, cin: int, cout: int, temb: Optional[int], eps: float, temporal_eps: Optional[float] = None,
                 merge: float = 0.5, switch: bool = True, groups: int = 32):
        super().__init__()
        self.spatial_res_block = _Res2D(cin, cout, temb, eps, groups)
        self.temporal_res_block = _ResT(cout, temb, temporal_eps if temporal_eps is not None else eps, groups)
        self.time_mixer = _Blend(merge, switch)

    def forward(self, x, temb, frames: int):
        h = self.spatial_res_block(x, temb)
        BF, C, H, W = h.shape
        B = BF // frames
        hs = h.reshape(B, frames, C, H, W).permute(0, 2, 1, 3, 4)
        tb = temb.reshape(B, frames, -1) if temb is not None else None
        ht = self.temporal_res_block(hs, tb)
        h = self.time_mixer(hs, ht)
        return h.permute(0, 2, 1, 3, 4).reshape(BF, C, H, W)


class _SBlock(nn.Module):
    """BasicTransformerBlock (self-attention, cross-attention, GEGLU)."""

    def __init__(self, d: int, heads: int, ctx: int):
        super().__init__()
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn1, self.attn2 = _Attn(d, heads), _Attn(d, heads, ctx)
        self.ff = nn.Module()
        self.ff.net = nn.ModuleList([_GEGLU(d, 4 * d), nn.Identity(), nn.Linear(4 * d, d)])

    def forward(self, x, ctx):
        x = x + self.attn1(self.norm1(x))
        x = x + self.attn2(self.norm2(x), ctx)
        return x + self.ff.net[2](self.ff.net[0](self.norm3(x)))


class _TBlock(nn.Module):
    """TemporalBasicTransformerBlock (dim == time_mix_inner_dim: residual ff_in and ff)."""

    def __init__(self, d: int, heads: int, ctx: int):
        super().__init__()
        self.norm_in = nn.LayerNorm(d)
        self.ff_in = nn.Module()
        self.ff_in.net = nn.ModuleList([_GEGLU(d, 4 * d), nn.Identity(), nn.Linear(4 * d, d)])
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn1, self.attn2 = _Attn(d, heads), _Attn(d, heads, ctx)
        self.ff = nn.Module()
        self.ff.net = nn.ModuleList([_GEGLU(d, 4 * d), nn.Identity(), nn.Linear(4 * d, d)])

    def forward(self, x, frames: int, ctx):
        BF, S, C = x.shape
        B = BF // frames
        h = x.reshape(B, frames, S, C).permute(0, 2, 1, 3).reshape(B * S, frames, C)
        h = h + self.ff_in.net[2](self.ff_in.net[0](self.norm_in(h)))
        h = h + self.attn1(self.norm1(h))
        h = h + self.attn2(self.norm2(h), ctx)
        h = h + self.ff.net[2](self.ff.net[0](self.norm3(h)))
        return h.reshape(B, S, frames, C).permute(0, 2, 1, 3).reshape(BF, S, C)


class _STTransformer(nn.Module):
    """TransformerSpatioTemporalModel (one layer of each)."""

    def __init__(self, c: int, heads: int, head_dim: int, ctx: int, depth: int = 1, groups: int = 32):
        super().__init__()
        inner = heads * head_dim
        self.norm = nn.GroupNorm(groups, c, eps=1e-6)
        self.proj_in = nn.Linear(c, inner)
        self.transformer_blocks = nn.ModuleList(_SBlock(inner, heads, ctx) for _ in range(depth))
        self.temporal_transformer_blocks = nn.ModuleList(_TBlock(inner, heads, ctx) for _ in range(depth))
        self.time_pos_embed = _TEmb(c, 4 * c, c)
        self.time_mixer = _Blend(0.5, False)
        self.proj_out = nn.Linear(inner, c)
        self.c = c

    def forward(self, x, ctx, frames: int):
        BF, C, H, W = x.shape
        B = BF // frames
        # the temporal blocks attend to the first frame's context, broadcast over the pixels
        tc = ctx.reshape(B, frames, -1, ctx.shape[-1])[:, 0]
        tc = tc[:, None].expand(B, H * W, tc.shape[1], tc.shape[2]).reshape(B * H * W, tc.shape[1], tc.shape[2])
        h = self.norm(x).permute(0, 2, 3, 1).reshape(BF, H * W, C)
        h = self.proj_in(h)
        fid = torch.arange(frames, device=x.device).repeat(B)
        emb = self.time_pos_embed(_tproj(fid, self.c).to(h.dtype))[:, None, :]
        for sb, tb in zip(self.transformer_blocks, self.temporal_transformer_blocks):
            h = sb(h, ctx)
            hm = tb(h + emb, frames, tc)
            h = self.time_mixer(h, hm)
        h = self.proj_out(h).reshape(BF, H, W, C).permute(0, 3, 1, 2)
        return x + h


class UNetSTC(nn.Module):
    """UNetSpatioTemporalConditionModel."""

    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        n = len(ch)
        lpb = int(c.get("layers_per_block", 2))
        ctx = int(c["cross_attention_dim"])
        heads = _per_block(c.get("num_attention_heads", 8), n)
        depth = _per_block(c.get("transformer_layers_per_block", 1), n)
        g = int(c.get("norm_num_groups", 32))
        temb = ch[0] * 4
        self.ch0 = ch[0]
        self.add_dim = int(c.get("addition_time_embed_dim", 256))
        self.conv_in = nn.Conv2d(c.get("in_channels", 8), ch[0], 3, padding=1)
        self.time_embedding = _TEmb(ch[0], temb)
        self.add_embedding = _TEmb(int(c.get("projection_class_embeddings_input_dim", 768)), temb)
        downs, prev = [], ch[0]
        for i, t in enumerate(c["down_block_types"]):
            b = nn.Module()
            cross = "CrossAttn" in t
            b.resnets = nn.ModuleList(_STRes(prev if j == 0 else ch[i], ch[i], temb, 1e-6 if cross else 1e-5, groups=g)
                                      for j in range(lpb))
            if cross:
                b.attentions = nn.ModuleList(_STTransformer(ch[i], heads[i], ch[i] // heads[i], ctx, depth[i], g)
                                             for _ in range(lpb))
            if i < n - 1:
                b.downsamplers = nn.ModuleList([_Down(ch[i])])
            downs.append(b)
            prev = ch[i]
        self.down_blocks = nn.ModuleList(downs)
        m = nn.Module()
        m.resnets = nn.ModuleList(_STRes(ch[-1], ch[-1], temb, 1e-5, groups=g) for _ in range(2))
        m.attentions = nn.ModuleList([_STTransformer(ch[-1], heads[-1], ch[-1] // heads[-1], ctx, depth[-1], g)])
        self.mid_block = m
        rch, rheads, rdepth = ch[::-1], heads[::-1], depth[::-1]
        ups, prev = [], ch[-1]
        for i, t in enumerate(c["up_block_types"]):
            out, skip_in = rch[i], rch[min(i + 1, n - 1)]
            cross = "CrossAttn" in t
            b = nn.Module()
            b.resnets = nn.ModuleList(   # the up blocks get resnet_eps 1e-5 whatever their kind
                _STRes((prev if j == 0 else out) + (skip_in if j == lpb else out), out, temb, 1e-5, groups=g)
                for j in range(lpb + 1))
            if cross:
                b.attentions = nn.ModuleList(_STTransformer(out, rheads[i], out // rheads[i], ctx, rdepth[i], g)
                                             for _ in range(lpb + 1))
            if i < n - 1:
                b.upsamplers = nn.ModuleList([_Up(out)])
            ups.append(b)
            prev = out
        self.up_blocks = nn.ModuleList(ups)
        self.conv_norm_out = nn.GroupNorm(g, ch[0], eps=1e-5)
        self.conv_out = nn.Conv2d(ch[0], c.get("out_channels", 4), 3, padding=1)

    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor, time_ids: torch.Tensor) -> torch.Tensor:
        """x [B, F, C, H, W], t [B], ctx [B, 1, D], time_ids [B, 3] -> [B, F, C_out, H, W]."""
        B, Fr = x.shape[:2]
        emb = self.time_embedding(_tproj(t, self.ch0).to(x.dtype))
        te = _tproj(time_ids.reshape(-1), self.add_dim).reshape(B, -1).to(x.dtype)
        emb = (emb + self.add_embedding(te)).repeat_interleave(Fr, 0)
        ctx = ctx.repeat_interleave(Fr, 0)
        h = self.conv_in(x.flatten(0, 1))
        skips = [h]
        for b in self.down_blocks:
            for j, r in enumerate(b.resnets):
                h = r(h, emb, Fr)
                if hasattr(b, "attentions"):
                    h = b.attentions[j](h, ctx, Fr)
                skips.append(h)
            if hasattr(b, "downsamplers"):
                h = b.downsamplers[0](h)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[1](m.attentions[0](m.resnets[0](h, emb, Fr), ctx, Fr), emb, Fr)
        for b in self.up_blocks:
            for j, r in enumerate(b.resnets):
                h = r(torch.cat([h, skips.pop()], dim=1), emb, Fr)
                if hasattr(b, "attentions"):
                    h = b.attentions[j](h, ctx, Fr)
            if hasattr(b, "upsamplers"):
                h = b.upsamplers[0](h, skips[-1].shape[-2:] if skips else None)
        h = self.conv_out(F.silu(self.conv_norm_out(h)))
        return h.reshape(B, Fr, *h.shape[1:])


class TemporalVaeDecoder(nn.Module):
    """AutoencoderKLTemporalDecoder's decoder (no post-quant convolution)."""

    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        lpb = int(c.get("layers_per_block", 2))
        lat = int(c.get("latent_channels", 4))
        g = int(c.get("norm_num_groups", 32))
        self.scaling = float(c.get("scaling_factor", 0.18215))

        def st(cin, cout):
            return _STRes(cin, cout, None, 1e-6, 1e-5, merge=0.0, switch=True, groups=g)
        d = nn.Module()
        d.conv_in = nn.Conv2d(lat, ch[-1], 3, padding=1)
        d.mid_block = nn.Module()
        d.mid_block.resnets = nn.ModuleList(st(ch[-1], ch[-1]) for _ in range(lpb))
        d.mid_block.attentions = nn.ModuleList([_VaeAttn(ch[-1], g, 1e-6)])
        rch, ups, prev = ch[::-1], [], ch[-1]
        for i in range(len(ch)):
            b = nn.Module()
            b.resnets = nn.ModuleList(st(prev if j == 0 else rch[i], rch[i]) for j in range(lpb + 1))
            if i < len(ch) - 1:
                b.upsamplers = nn.ModuleList([_Up(rch[i])])
            ups.append(b)
            prev = rch[i]
        d.up_blocks = nn.ModuleList(ups)
        d.conv_norm_out = nn.GroupNorm(g, ch[0], eps=1e-6)
        d.conv_out = nn.Conv2d(ch[0], c.get("out_channels", 3), 3, padding=1)
        d.time_conv_out = nn.Conv3d(c.get("out_channels", 3), c.get("out_channels", 3), (3, 1, 1), padding=(1, 0, 0))
        self.decoder = d

    def forward(self, z: torch.Tensor, frames: int) -> torch.Tensor:
        """z [frames, lat, h, w] (already divided by the scaling factor) -> [frames, 3, H, W]."""
        d = self.decoder
        h = d.conv_in(z)
        m = d.mid_block
        h = m.resnets[0](h, None, frames)
        for r, a in zip(m.resnets[1:], m.attentions):
            h = r(a(h), None, frames)
        for b in d.up_blocks:
            for r in b.resnets:
                h = r(h, None, frames)
            if hasattr(b, "upsamplers"):
                h = b.upsamplers[0](h)
        h = d.conv_out(F.silu(d.conv_norm_out(h)))
        BF, C, H, W = h.shape
        h = d.time_conv_out(h.reshape(BF // frames, frames, C, H, W).permute(0, 2, 1, 3, 4))
        return h.permute(0, 2, 1, 3, 4).reshape(BF, C, H, W)


def _temporal_vae_names(sd):
    out = {}
    for k, v in sd.items():
        if k.startswith("decoder."):
            out[k] = v
    return out


class KarrasEuler:
    """EulerDiscreteScheduler as SVD configures it: Karras sigmas between sigma_min and
    sigma_max (rho 7), v-prediction, continuous timesteps t = log(sigma) / 4."""

    def __init__(self, c: dict):
        self.smin = float(c.get("sigma_min", 0.002))
        self.smax = float(c.get("sigma_max", 700.0))
        self.pred = c.get("prediction_type", "v_prediction")
        self.spacing = c.get("timestep_spacing", "leading")

    def sigmas(self, steps: int) -> torch.Tensor:
        rho = 7.0
        ramp = torch.linspace(0, 1, steps, dtype=torch.float64)
        a, b = self.smax ** (1 / rho), self.smin ** (1 / rho)
        s = (a + ramp * (b - a)) ** rho
        return torch.cat([s, torch.zeros(1, dtype=torch.float64)])

    def init_sigma(self, sig: torch.Tensor) -> float:
        m = float(sig.max())
        return m if self.spacing in ("linspace", "trailing") else math.sqrt(m * m + 1.0)

    def denoised(self, out: torch.Tensor, x: torch.Tensor, sigma: float) -> torch.Tensor:
        if self.pred == "v_prediction":
            return out * (-sigma / math.sqrt(sigma * sigma + 1)) + x / (sigma * sigma + 1)
        return x - sigma * out


class StableVideoDiffusion:
    def __init__(self, path: str, device: str = "cpu"):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.unet_cfg = _cfg(os.path.join(path, "unet", "config.json"))
        self.unet = UNetSTC(self.unet_cfg)
        self.unet.load_state_dict(_load_weights(os.path.join(path, "unet")), strict=True)
        vcfg = _cfg(os.path.join(path, "vae", "config.json"))
        vsd = _load_weights(os.path.join(path, "vae"))
        self.vae = TemporalVaeDecoder(vcfg)
        self.vae.load_state_dict(_temporal_vae_names(vsd), strict=True)
        self.vae_enc = VaeEncoder(vcfg)
        self.vae_enc.load_state_dict(_vae_enc_names(vsd), strict=True)
        import transformers as tf
        self.image_encoder = tf.CLIPVisionModelWithProjection.from_pretrained(os.path.join(path, "image_encoder"))
        fe = os.path.join(path, "feature_extractor", "preprocessor_config.json")
        pcfg = _cfg(fe) if os.path.isfile(fe) else {}
        self.clip_mean = torch.tensor(pcfg.get("image_mean", [0.48145466, 0.4578275, 0.40821073])).view(1, 3, 1, 1)
        self.clip_std = torch.tensor(pcfg.get("image_std", [0.26862954, 0.26130258, 0.27577711])).view(1, 3, 1, 1)
        self.clip_px = int(self.image_encoder.config.image_size)
        for mod in (self.unet, self.vae, self.vae_enc, self.image_encoder):
            mod.to(self.device, self.dtype).eval().requires_grad_(False)
        sc = os.path.join(path, "scheduler", "scheduler_config.json")
        self.sched = KarrasEuler(_cfg(sc) if os.path.isfile(sc) else {})
        self.vae_scale = 2 ** (len(self.vae.decoder.up_blocks) - 1)
        self.num_frames = int(self.unet_cfg.get("num_frames", 14))

    def _image_embed(self, img: torch.Tensor) -> torch.Tensor:
        """img [1, 3, H, W] in [-1, 1] -> CLIP image embedding [1, 1, D] (antialiased bicubic to the
        tower's size, CLIP normalisation)."""
        x = F.interpolate(img.float(), size=(self.clip_px, self.clip_px), mode="bicubic", align_corners=True,
                          antialias=True)
        x = ((x + 1.0) / 2.0 - self.clip_mean.to(x.device)) / self.clip_std.to(x.device)
        e = self.image_encoder(pixel_values=x.to(self.dtype)).image_embeds
        return e[:, None, :]

    @torch.no_grad()
    def __call__(self, image, width: int = 1024, height: int = 576, num_frames: Optional[int] = None,
                 steps: int = 25, min_guidance_scale: float = 1.0, max_guidance_scale: float = 3.0, fps: int = 7,
                 motion_bucket_id: int = 127, noise_aug_strength: float = 0.02, decode_chunk_size: int = 8,
                 seed: Optional[int] = None) -> torch.Tensor:
        """-> uint8 frames [F, H, W, 3]; `image` a path or PIL image."""
        from PIL import Image
        g = torch.Generator().manual_seed(seed if seed is not None else int.from_bytes(os.urandom(4), "little"))
        Fr = int(num_frames or self.num_frames)
        h, w = max(1, height // self.vae_scale), max(1, width // self.vae_scale)
        im = image if isinstance(image, Image.Image) else Image.open(image)
        im = im.convert("RGB").resize((w * self.vae_scale, h * self.vae_scale), Image.BICUBIC)
        img = torch.from_numpy(np.asarray(im, dtype=np.float32)).permute(2, 0, 1)[None] / 127.5 - 1.0
        img = img.to(self.device)
        emb = self._image_embed(img)
        cfg = max_guidance_scale > 1.0
        ctx = torch.cat([torch.zeros_like(emb), emb]) if cfg else emb
        noisy = img + noise_aug_strength * torch.randn(img.shape, generator=g).to(self.device)
        # the latent distribution's mean (diffusers: latent_dist.mode()), unscaled
        ev = self.vae_enc
        e = ev.encoder
        hh = e.conv_in(noisy.to(self.dtype))
        for b in e.down_blocks:
            for r in b.resnets:
                hh = r(hh)
            if hasattr(b, "downsamplers"):
                hh = b.downsamplers[0](hh)
        hh = e.mid_block.resnets[1](e.mid_block.attentions[0](e.mid_block.resnets[0](hh)))
        from .sd import _gn
        mom = ev.quant_conv(e.conv_out(_gn(e.conv_norm_out, hh, True))).float()
        lat = mom.chunk(2, dim=1)[0]
        cond_lat = torch.cat([torch.zeros_like(lat), lat]) if cfg else lat
        cond_lat = cond_lat[:, None].expand(-1, Fr, -1, -1, -1)
        ids = torch.tensor([[fps - 1, motion_bucket_id, noise_aug_strength]], dtype=torch.float32, device=self.device)
        ids = torch.cat([ids, ids]) if cfg else ids
        sig = self.sched.sigmas(max(1, steps))
        x = torch.randn(1, Fr, lat.shape[1], h, w, generator=g).to(self.device) * self.sched.init_sigma(sig)
        gs = torch.linspace(min_guidance_scale, max_guidance_scale, Fr, device=self.device)[None, :, None, None, None]
        for i in range(len(sig) - 1):
            s, s_next = float(sig[i]), float(sig[i + 1])
            xin = x / math.sqrt(s * s + 1.0)
            xin = torch.cat([xin, xin]) if cfg else xin
            xin = torch.cat([xin, cond_lat.to(xin.dtype)], dim=2).to(self.dtype)
            t = torch.full((xin.shape[0],), 0.25 * math.log(s), device=self.device)
            out = self.unet(xin, t, ctx.to(self.dtype), ids).float()
            if cfg:
                u, c = out.chunk(2)
                out = u + gs * (c - u)
            den = self.sched.denoised(out, x, s)
            x = x + (x - den) / s * (s_next - s)
        z = (x[0] / self.vae.scaling).to(self.dtype)
        frames = []
        for i in range(0, Fr, max(1, decode_chunk_size)):
            chunk = z[i:i + decode_chunk_size]
            frames.append(self.vae(chunk, chunk.shape[0]).float())
        v = torch.cat(frames)
        return ((v / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8).permute(0, 2, 3, 1).cpu()
