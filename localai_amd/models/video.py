"""Text-to-video diffusion, served by the `diffusers` backend for `pipeline_type:
VideoDiffusionPipeline` (reference: `backend/python/diffusers/backend.py:223-226` loads a
DiffusionPipeline -- a TextToVideoSDPipeline such as ModelScope text-to-video-ms-1.7b -- and
`:445-448` renders `num_frames` frames at `step` steps, guidance `cfg_scale`, and writes them with
export_to_video).

Reads the diffusers directory layout (`model_index.json` with `_class_name:
TextToVideoSDPipeline`, `unet/` UNet3DConditionModel, `vae/`, `text_encoder/`, `tokenizer/`,
`scheduler/`).  The UNet3DConditionModel is the 2-D UNet of models/sd.py interleaved with the
temporal layers, named like the checkpoint's tensors (strict state-dict load):

* TemporalConvLayer after every ResNet: four GroupNorm / SiLU / (3, 1, 1) Conv3d stages over the
  frame axis, the last zero-initialised, added to its input;
* TransformerTemporalModel after every spatial transformer (and `transformer_in` after conv_in):
  GroupNorm over (C/groups, frames, H, W), then per pixel a transformer block over the frames
  (self-attention twice -- `double_self_attention` -- and a GEGLU feed-forward);
* diffusers' head-count quirk: `attention_head_dim` is passed as the NUMBER of heads, so the
  spatial and temporal attentions of a C-channel block run C / attention_head_dim heads of
  attention_head_dim dims, and transformer_in runs 8 heads of attention_head_dim.

Frames are decoded one latent at a time by the SD VAE decoder.  Video files: `.gif` (animated
GIF), `.webp` (animated WebP), `.png` (APNG), anything else -- `.mp4` included -- an MJPEG AVI
written here (no video codec library is available in this image; export_to_video's mp4v mp4
needs OpenCV).  Parity with diffusers is unpinned (diffusers is not installed).
"""
from __future__ import annotations

import math
import os
import struct
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .sd import (ClipTextEncoder, Scheduler, VaeDecoder, _Attn, _cfg, _Down, _gn, _GEGLU, _load_weights, _per_block,
                 _Resnet, _Transformer2D, _Up, _vae_names)


def is_video_pipeline(path: str) -> bool:
    mi = os.path.join(path, "model_index.json")
    if not os.path.isfile(mi):
        return False
    try:
        return _cfg(mi).get("_class_name") in ("TextToVideoSDPipeline", "VideoToVideoSDPipeline")
    except (OSError, ValueError):
        return False


# ------------------------------------------------------------------ temporal layers
class _TemporalConv(nn.Module):
    """diffusers TemporalConvLayer: conv1 = (GroupNorm, SiLU, Conv3d), conv2..4 = (GroupNorm, SiLU,
    Dropout, Conv3d) with (3, 1, 1) kernels over the frame axis; residual."""

    def __init__(self, c: int, groups: int):
        super().__init__()
        self.conv1 = nn.Sequential(nn.GroupNorm(groups, c), nn.SiLU(), nn.Conv3d(c, c, (3, 1, 1), padding=(1, 0, 0)))
        for n in ("conv2", "conv3", "conv4"):
            setattr(self, n, nn.Sequential(nn.GroupNorm(groups, c), nn.SiLU(), nn.Identity(),
                                           nn.Conv3d(c, c, (3, 1, 1), padding=(1, 0, 0))))

    def forward(self, x: torch.Tensor, frames: int) -> torch.Tensor:
        BF, C, H, W = x.shape
        h = x.reshape(BF // frames, frames, C, H, W).permute(0, 2, 1, 3, 4)          # B C F H W
        r = h
        for seq in (self.conv1, self.conv2, self.conv3, self.conv4):
            gn, conv = seq[0], seq[-1]
            h = conv(F.silu(F.group_norm(h, gn.num_groups, gn.weight, gn.bias, gn.eps)))
        h = r + h
        return h.permute(0, 2, 1, 3, 4).reshape(BF, C, H, W)


class _TTBlock(nn.Module):
    """BasicTransformerBlock of the temporal transformer: self-attention, self-attention again
    (double_self_attention), GEGLU feed-forward; pre-LayerNorm."""

    def __init__(self, d: int, heads: int):
        super().__init__()
        self.norm1, self.norm2, self.norm3 = nn.LayerNorm(d), nn.LayerNorm(d), nn.LayerNorm(d)
        self.attn1, self.attn2 = _Attn(d, heads), _Attn(d, heads)
        self.ff = nn.Module()
        self.ff.net = nn.ModuleList([_GEGLU(d, 4 * d), nn.Identity(), nn.Linear(4 * d, d)])

    def forward(self, x):
        x = x + self.attn1(self.norm1(x))
        x = x + self.attn2(self.norm2(x))
        return x + self.ff.net[2](self.ff.net[0](self.norm3(x)))


class _TransformerTemporal(nn.Module):
    """diffusers TransformerTemporalModel: every pixel attends over the frames."""

    def __init__(self, c: int, heads: int, head_dim: int, groups: int):
        super().__init__()
        inner = heads * head_dim
        self.norm = nn.GroupNorm(groups, c, eps=1e-6)
        self.proj_in = nn.Linear(c, inner)
        self.transformer_blocks = nn.ModuleList([_TTBlock(inner, heads)])
        self.proj_out = nn.Linear(inner, c)

    def forward(self, x: torch.Tensor, frames: int) -> torch.Tensor:
        BF, C, H, W = x.shape
        B = BF // frames
        h = x.reshape(B, frames, C, H, W).permute(0, 2, 1, 3, 4)                      # B C F H W
        h = F.group_norm(h, self.norm.num_groups, self.norm.weight, self.norm.bias, self.norm.eps)
        h = h.permute(0, 3, 4, 2, 1).reshape(B * H * W, frames, C)
        h = self.proj_in(h)
        for b in self.transformer_blocks:
            h = b(h)
        h = self.proj_out(h)
        h = h.reshape(B, H, W, frames, C).permute(0, 3, 4, 1, 2).reshape(BF, C, H, W)
        return x + h


# ------------------------------------------------------------------ UNet3DConditionModel
class UNet3D(nn.Module):
    def __init__(self, c: dict):
        super().__init__()
        ch = list(c["block_out_channels"])
        n = len(ch)
        lpb = int(c.get("layers_per_block", 2))
        g, eps = int(c.get("norm_num_groups", 32)), float(c.get("norm_eps", 1e-5))
        ctx = int(c["cross_attention_dim"])
        hd = _per_block(c.get("num_attention_heads") or c.get("attention_head_dim", 64), n)
        self.flip = bool(c.get("flip_sin_to_cos", True))
        self.shift = float(c.get("freq_shift", 0))
        temb = ch[0] * 4
        self.conv_in = nn.Conv2d(c.get("in_channels", 4), ch[0], 3, padding=1)
        self.time_embedding = nn.Module()
        self.time_embedding.linear_1 = nn.Linear(ch[0], temb)
        self.time_embedding.linear_2 = nn.Linear(temb, temb)
        # transformer_in: 8 heads of attention_head_dim (the config value, not the per-block heads)
        ahd = c.get("attention_head_dim", 64)
        self.transformer_in = _TransformerTemporal(ch[0], 8, int(ahd[0] if isinstance(ahd, (list, tuple)) else ahd), g)

        def attn2d(cc, i):
            return _Transformer2D(cc, cc // hd[i], ctx, g, bool(c.get("use_linear_projection", False)))

        def attn_t(cc, i):
            return _TransformerTemporal(cc, cc // hd[i], hd[i], g)
        downs, prev = [], ch[0]
        for i, t in enumerate(c["down_block_types"]):
            b = nn.Module()
            b.resnets = nn.ModuleList(_Resnet(prev if j == 0 else ch[i], ch[i], g, eps, temb) for j in range(lpb))
            b.temp_convs = nn.ModuleList(_TemporalConv(ch[i], g) for _ in range(lpb))
            if "CrossAttn" in t:
                b.attentions = nn.ModuleList(attn2d(ch[i], i) for _ in range(lpb))
                b.temp_attentions = nn.ModuleList(attn_t(ch[i], i) for _ in range(lpb))
            if i < n - 1:
                b.downsamplers = nn.ModuleList([_Down(ch[i])])
            downs.append(b)
            prev = ch[i]
        self.down_blocks = nn.ModuleList(downs)
        m = nn.Module()
        m.resnets = nn.ModuleList([_Resnet(ch[-1], ch[-1], g, eps, temb) for _ in range(2)])
        m.temp_convs = nn.ModuleList([_TemporalConv(ch[-1], g) for _ in range(2)])
        m.attentions = nn.ModuleList([attn2d(ch[-1], n - 1)])
        m.temp_attentions = nn.ModuleList([attn_t(ch[-1], n - 1)])
        self.mid_block = m
        rch, rhd = ch[::-1], hd[::-1]
        ups, prev = [], ch[-1]
        for i, t in enumerate(c["up_block_types"]):
            out, skip_in = rch[i], rch[min(i + 1, n - 1)]
            b = nn.Module()
            b.resnets = nn.ModuleList(
                _Resnet((prev if j == 0 else out) + (skip_in if j == lpb else out), out, g, eps, temb)
                for j in range(lpb + 1))
            b.temp_convs = nn.ModuleList(_TemporalConv(out, g) for _ in range(lpb + 1))
            if "CrossAttn" in t:
                b.attentions = nn.ModuleList(
                    _Transformer2D(out, out // rhd[i], ctx, g, bool(c.get("use_linear_projection", False)))
                    for _ in range(lpb + 1))
                b.temp_attentions = nn.ModuleList(_TransformerTemporal(out, out // rhd[i], rhd[i], g)
                                                  for _ in range(lpb + 1))
            if i < n - 1:
                b.upsamplers = nn.ModuleList([_Up(out)])
            ups.append(b)
            prev = out
        self.up_blocks = nn.ModuleList(ups)
        self.conv_norm_out = nn.GroupNorm(g, ch[0], eps=eps)
        self.conv_out = nn.Conv2d(ch[0], c.get("out_channels", 4), 3, padding=1)
        self.ch0 = ch[0]

    def _temb(self, t: torch.Tensor, dtype) -> torch.Tensor:
        half = self.ch0 // 2
        f = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / (half - self.shift))
        e = t.float()[:, None] * f[None]
        e = torch.cat([torch.cos(e), torch.sin(e)] if self.flip else [torch.sin(e), torch.cos(e)], dim=-1).to(dtype)
        return self.time_embedding.linear_2(F.silu(self.time_embedding.linear_1(e)))

    def forward(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        """x [B, C, F, H, W], t [B], ctx [B, L, D] -> [B, C_out, F, H, W]."""
        B, C, Fr, H, W = x.shape
        temb = self._temb(t, x.dtype).repeat_interleave(Fr, 0)
        ctx = ctx.repeat_interleave(Fr, 0)
        h = x.permute(0, 2, 1, 3, 4).reshape(B * Fr, C, H, W)
        h = self.transformer_in(self.conv_in(h), Fr)
        skips = [h]
        for b in self.down_blocks:
            for j, r in enumerate(b.resnets):
                h = b.temp_convs[j](r(h, temb), Fr)
                if hasattr(b, "attentions"):
                    h = b.temp_attentions[j](b.attentions[j](h, ctx), Fr)
                skips.append(h)
            if hasattr(b, "downsamplers"):
                h = b.downsamplers[0](h)
                skips.append(h)
        m = self.mid_block
        h = m.temp_convs[0](m.resnets[0](h, temb), Fr)
        h = m.temp_attentions[0](m.attentions[0](h, ctx), Fr)
        h = m.temp_convs[1](m.resnets[1](h, temb), Fr)
        for b in self.up_blocks:
            for j, r in enumerate(b.resnets):
                h = b.temp_convs[j](r(torch.cat([h, skips.pop()], dim=1), temb), Fr)
                if hasattr(b, "attentions"):
                    h = b.temp_attentions[j](b.attentions[j](h, ctx), Fr)
            if hasattr(b, "upsamplers"):
                h = b.upsamplers[0](h, skips[-1].shape[-2:] if skips else None)
        h = self.conv_out(_gn(self.conv_norm_out, h, True))
        return h.reshape(B, Fr, -1, H, W).permute(0, 2, 1, 3, 4)


# ------------------------------------------------------------------ pipeline
class TextToVideo:
    """TextToVideoSDPipeline: CLIP prompt embeddings, DDIM over [1, 4, F, h, w] latents with
    classifier-free guidance as one batch of 2, per-frame VAE decode -> uint8 [F, H, W, 3]."""

    def __init__(self, path: str, device: str = "cpu"):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.text = ClipTextEncoder(_cfg(os.path.join(path, "text_encoder", "config.json")))
        self.text.load_state_dict({(k if k.startswith("text_model.") else "text_model." + k): v
                                   for k, v in _load_weights(os.path.join(path, "text_encoder")).items()
                                   if "position_ids" not in k}, strict=True)
        self.unet = UNet3D(_cfg(os.path.join(path, "unet", "config.json")))
        self.unet.load_state_dict(_load_weights(os.path.join(path, "unet")), strict=True)
        vcfg = _cfg(os.path.join(path, "vae", "config.json"))
        self.vae = VaeDecoder(vcfg)
        self.vae.load_state_dict(_vae_names(_load_weights(os.path.join(path, "vae"))), strict=True)
        for mod in (self.text, self.unet, self.vae):
            mod.to(self.device, self.dtype).eval().requires_grad_(False)
        sc = os.path.join(path, "scheduler", "scheduler_config.json")
        self.sched = Scheduler(_cfg(sc) if os.path.isfile(sc) else {}, "ddim")
        from transformers import CLIPTokenizer
        self.tok = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer"))
        self.max_len = self.text.text_model.embeddings.position_embedding.weight.shape[0]
        self.latent_ch = int(vcfg.get("latent_channels", 4))
        self.vae_scale = 2 ** (len(self.vae.decoder.up_blocks) - 1)

    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: str = "", width: int = 256, height: int = 256,
                 num_frames: int = 16, steps: int = 25, guidance_scale: float = 9.0,
                 seed: Optional[int] = None) -> torch.Tensor:
        g = torch.Generator().manual_seed(seed if seed is not None else int.from_bytes(os.urandom(4), "little"))
        h, w = max(1, height // self.vae_scale), max(1, width // self.vae_scale)
        cfg = guidance_scale > 1.0
        prompts = [negative_prompt, prompt] if cfg else [prompt]
        ids = self.tok(prompts, padding="max_length", max_length=self.max_len, truncation=True,
                       return_tensors="pt").input_ids.to(self.device)
        ctx = self.text(ids)
        x = torch.randn(1, self.latent_ch, num_frames, h, w, generator=g).to(self.device)
        ts = self.sched.timesteps(max(1, steps))
        for i, t in enumerate(ts):
            xin = (torch.cat([x, x]) if cfg else x).to(self.dtype)
            tt = torch.full((xin.shape[0],), float(t), device=self.device)
            out = self.unet(xin, tt, ctx).float()
            if cfg:
                u, c = out.chunk(2)
                out = u + guidance_scale * (c - u)
            x = self.sched.step(out, t, ts[i + 1] if i + 1 < len(ts) else None, x)
        frames = []
        for f in range(num_frames):
            img = self.vae(x[:, :, f].to(self.dtype)).float()[0]
            frames.append(((img / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8).permute(1, 2, 0).cpu())
        return torch.stack(frames)


# ------------------------------------------------------------------ video files
def _mjpeg_avi(frames: Sequence[np.ndarray], fps: int) -> bytes:
    """A minimal RIFF AVI with one MJPEG video stream (JPEG frames from PIL) and an idx1 index."""
    import io
    from PIL import Image
    jpgs = []
    for fr in frames:
        b = io.BytesIO()
        Image.fromarray(fr).save(b, format="JPEG", quality=90)
        jpgs.append(b.getvalue())
    H, W = frames[0].shape[:2]
    n = len(jpgs)

    def chunk(fourcc: bytes, data: bytes) -> bytes:
        pad = b"\0" if len(data) % 2 else b""
        return fourcc + struct.pack("<I", len(data)) + data + pad

    def lst(kind: bytes, data: bytes) -> bytes:
        return b"LIST" + struct.pack("<I", len(data) + 4) + kind + data
    us = int(round(1e6 / max(1, fps)))
    avih = struct.pack("<IIIIIIIIIIIIII", us, max(len(j) for j in jpgs) * fps, 0, 0x10, n, 0, 1,
                       max(len(j) for j in jpgs), W, H, 0, 0, 0, 0)
    strh = struct.pack("<4s4sIHHIIIIIIIIhhhh", b"vids", b"MJPG", 0, 0, 0, 0, 1, max(1, fps), 0, n,
                       max(len(j) for j in jpgs), 0xFFFFFFFF, 0, 0, 0, W, H)
    strf = struct.pack("<IiiHH4sIiiII", 40, W, H, 1, 24, b"MJPG", W * H * 3, 0, 0, 0, 0)
    hdrl = lst(b"hdrl", chunk(b"avih", avih) + lst(b"strl", chunk(b"strh", strh) + chunk(b"strf", strf)))
    movi_data, idx, off = b"", b"", 4
    for j in jpgs:
        c = chunk(b"00dc", j)
        idx += b"00dc" + struct.pack("<III", 0x10, off, len(j))
        movi_data += c
        off += len(c)
    body = b"AVI " + hdrl + lst(b"movi", movi_data) + chunk(b"idx1", idx)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def export_video(frames: torch.Tensor, dst: str, fps: int = 8) -> str:
    """Write uint8 frames [F, H, W, 3] to dst (format by extension, see the module docstring)."""
    from PIL import Image
    arr = [f.numpy() if isinstance(f, torch.Tensor) else np.asarray(f) for f in frames]
    ext = os.path.splitext(dst)[1].lower()
    ims = [Image.fromarray(a) for a in arr]
    dur = int(round(1000 / max(1, fps)))
    if ext == ".gif":
        ims[0].save(dst, save_all=True, append_images=ims[1:], duration=dur, loop=0)
    elif ext == ".webp":
        ims[0].save(dst, save_all=True, append_images=ims[1:], duration=dur, loop=0, lossless=False)
    elif ext == ".png":
        ims[0].save(dst, save_all=True, append_images=ims[1:], duration=dur, loop=0)
    else:
        with open(dst, "wb") as f:
            f.write(_mjpeg_avi(arr, fps))
    return dst


def read_avi_frames(path: str) -> List[bytes]:
    """The JPEG payloads of an MJPEG AVI written by export_video (tests / tooling): the `00dc`
    chunks of the `movi` list."""
    data = open(path, "rb").read()
    i = data.index(b"movi") + 4
    end = data.index(b"idx1", i)
    out = []
    while i < end and data[i:i + 4] == b"00dc":
        n = struct.unpack("<I", data[i + 4:i + 8])[0]
        out.append(data[i + 8:i + 8 + n])
        i += 8 + n + (n % 2)
    return out
