"""Stable Diffusion 3 / 3.5 text-to-image (diffusers StableDiffusion3Pipeline layout), served by the
`diffusers` backend with `pipeline_type: StableDiffusion3Pipeline` (reference:
`backend/python/diffusers/backend.py:235-246`; GenerateImage passes `guidance_scale = CFGScale`,
`negative_prompt`, width / height, `num_inference_steps`).

* text: CLIP-L and OpenCLIP-bigG (both CLIPTextModelWithProjection: penultimate hidden states,
  projected pooled embeddings) and, when present, T5 (`text_encoder_3`, up to 256 tokens; an
  all-zero T5 context otherwise, as diffusers does without it): context = [CLIP-L | CLIP-G padded to
  the T5 width ; T5] along the sequence, pooled = [CLIP-L pooled | CLIP-G pooled];
* SD3Transformer2DModel: 2x2 conv patch embedding plus the centre-cropped 2-D sin-cos position
  table (`pos_embed.pos_embed`, pos_embed_max_size), timestep + pooled-text conditioning,
  `num_layers` joint (MMDiT) blocks over [image | text] tokens with AdaLN-Zero modulation (the last
  block `context_pre_only`: AdaLN-continuous text input, no text output), optional RMS q/k norm
  (SD3.5), AdaLN-continuous output norm, projection and unpatchify;
* classifier-free guidance as one batch of 2; FlowMatch Euler with the scheduler's static shift;
  the 16-channel VAE (shift_factor, no quant convs) of models/sd.py.

Parity unpinned for the transformer (diffusers is not installed); the text encoders are checked
against transformers and the sampler in closed form (models/flux.py:flow_euler).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from typing import List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .flux import _FF, _RMS, _TEmb, _ln, _mod, _timestep_embedding, flow_euler
from .sd import StableDiffusion, VaeDecoder, _cfg, _load_weights, _vae_names


def _sincos_2d(embed_dim: int, grid: int, base_size: int, interp: float) -> torch.Tensor:
    """diffusers get_2d_sincos_pos_embed(embed_dim, grid, base_size, interpolation_scale): [grid^2, D]."""
    gh = np.arange(grid, dtype=np.float64) / (grid / base_size) / interp
    gw = np.arange(grid, dtype=np.float64) / (grid / base_size) / interp
    gx, gy = np.meshgrid(gw, gh)  # w first, as diffusers
    def one(d, pos):
        om = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float64) / (d / 2.0))
        out = pos.reshape(-1)[:, None] * om[None]
        return np.concatenate([np.sin(out), np.cos(out)], 1)
    emb = np.concatenate([one(embed_dim // 2, gx), one(embed_dim // 2, gy)], 1)
    return torch.from_numpy(emb).float()


class _JointAttn(nn.Module):
    def __init__(self, d: int, heads: int, pre_only: bool, qk_norm: bool):
        super().__init__()
        self.heads, self.pre_only, self.qk = heads, pre_only, qk_norm
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        self.to_out = nn.ModuleList([nn.Linear(d, d)])
        if not pre_only:
            self.to_add_out = nn.Linear(d, d)
        if qk_norm:
            hd = d // heads
            self.norm_q, self.norm_k = _RMS(hd), _RMS(hd)
            self.norm_added_q, self.norm_added_k = _RMS(hd), _RMS(hd)

    def _heads(self, t):
        B, L, _ = t.shape
        return t.view(B, L, self.heads, -1).transpose(1, 2)

    def forward(self, x, ctx):
        q, k, v = (self._heads(p(x)) for p in (self.to_q, self.to_k, self.to_v))
        cq, ck, cv = (self._heads(p(ctx)) for p in (self.add_q_proj, self.add_k_proj, self.add_v_proj))
        if self.qk:
            q, k, cq, ck = self.norm_q(q), self.norm_k(k), self.norm_added_q(cq), self.norm_added_k(ck)
        # JointAttnProcessor2_0: image tokens first, then text
        o = F.scaled_dot_product_attention(torch.cat([q, cq], 2), torch.cat([k, ck], 2),
                                           torch.cat([v, cv], 2)).transpose(1, 2).flatten(2)
        N = x.shape[1]
        return self.to_out[0](o[:, :N]), (None if self.pre_only else self.to_add_out(o[:, N:]))


class _JointBlock(nn.Module):
    def __init__(self, d: int, heads: int, pre_only: bool, qk_norm: bool):
        super().__init__()
        self.pre_only = pre_only
        self.norm1, self.norm1_context = nn.Module(), nn.Module()
        self.norm1.linear = nn.Linear(d, 6 * d)
        self.norm1_context.linear = nn.Linear(d, (2 if pre_only else 6) * d)
        self.attn = _JointAttn(d, heads, pre_only, qk_norm)
        self.ff = _FF(d)
        if not pre_only:
            self.ff_context = _FF(d)

    def forward(self, x, ctx, temb):
        e = self.norm1.linear(F.silu(temb)).chunk(6, -1)
        cm = self.norm1_context.linear(F.silu(temb))
        if self.pre_only:  # AdaLayerNormContinuous: (scale, shift)
            sc, sh = cm.chunk(2, -1)
            cn = _mod(_ln(ctx), sh, sc)
        else:
            c = cm.chunk(6, -1)
            cn = _mod(_ln(ctx), c[0], c[1])
        a, ca = self.attn(_mod(_ln(x), e[0], e[1]), cn)
        x = x + e[2][:, None] * a
        x = x + e[5][:, None] * self.ff(_mod(_ln(x), e[3], e[4]))
        if self.pre_only:
            return x, None
        ctx = ctx + c[2][:, None] * ca
        ctx = ctx + c[5][:, None] * self.ff_context(_mod(_ln(ctx), c[3], c[4]))
        return x, ctx


class SD3Transformer(nn.Module):
    """diffusers SD3Transformer2DModel (no dual-attention layers)."""

    def __init__(self, c: dict):
        super().__init__()
        heads, hd = int(c.get("num_attention_heads", 24)), int(c.get("attention_head_dim", 64))
        d = heads * hd
        if c.get("dual_attention_layers"):
            raise ValueError("SD3.5 dual-attention layers are not supported")
        self.p = int(c.get("patch_size", 2))
        self.cin = int(c.get("in_channels", 16))
        self.cout = int(c.get("out_channels") or self.cin)
        self.max_pos = int(c.get("pos_embed_max_size") or 0)
        sample = int(c.get("sample_size", 128))
        self.pos_embed = nn.Module()
        self.pos_embed.proj = nn.Conv2d(self.cin, d, self.p, stride=self.p)
        grid = self.max_pos or sample // self.p
        self.pos_embed.register_buffer("pos_embed", _sincos_2d(d, grid, sample // self.p, 1.0)[None], persistent=True)
        te = nn.Module()
        te.timestep_embedder = _TEmb(256, d)
        te.text_embedder = _TEmb(int(c.get("pooled_projection_dim", 2048)), d)
        self.time_text_embed = te
        self.context_embedder = nn.Linear(int(c.get("joint_attention_dim", 4096)), d)
        L = int(c.get("num_layers", 24))
        qk = c.get("qk_norm") == "rms_norm"
        self.transformer_blocks = nn.ModuleList(_JointBlock(d, heads, i == L - 1, qk) for i in range(L))
        self.norm_out = nn.Module()
        self.norm_out.linear = nn.Linear(d, 2 * d)
        self.proj_out = nn.Linear(d, self.p * self.p * self.cout)

    def _pos(self, h: int, w: int) -> torch.Tensor:
        pe = self.pos_embed.pos_embed
        if not self.max_pos:
            return pe
        g = self.max_pos
        if h > g or w > g:
            raise ValueError(f"latent {h}x{w} patches exceeds pos_embed_max_size {g}")
        top, left = (g - h) // 2, (g - w) // 2
        return pe.view(1, g, g, -1)[:, top:top + h, left:left + w].reshape(1, h * w, -1)

    def forward(self, x, ctx, pooled, t):
        """x [B, C, H, W] latents; ctx [B, T, 4096]; pooled [B, 2048]; t [B] timesteps (0..1000)."""
        B, _, H, W = x.shape
        h, w = H // self.p, W // self.p
        tok = self.pos_embed.proj(x).flatten(2).transpose(1, 2) + self._pos(h, w).to(x.dtype)
        te = self.time_text_embed
        temb = te.timestep_embedder(_timestep_embedding(t).to(x.dtype)) + te.text_embedder(pooled.to(x.dtype))
        c = self.context_embedder(ctx)
        for b in self.transformer_blocks:
            tok, c = b(tok, c, temb)
        scale, shift = self.norm_out.linear(F.silu(temb)).chunk(2, -1)
        o = self.proj_out(_mod(_ln(tok), shift, scale))
        o = o.view(B, h, w, self.p, self.p, self.cout).permute(0, 5, 1, 3, 2, 4)
        return o.reshape(B, self.cout, h * self.p, w * self.p)


def is_sd3_pipeline(path: str) -> bool:
    mi = os.path.join(path, "model_index.json")
    try:
        return os.path.isfile(mi) and str(_cfg(mi).get("_class_name", "")).startswith("StableDiffusion3")
    except (OSError, ValueError):
        return False


def sd3_sigmas(steps: int, cfg: dict) -> List[float]:
    """FlowMatchEulerDiscreteScheduler with a static shift (SD3: 3.0): linspace(1, 1/steps), shifted."""
    sh = float(cfg.get("shift", 3.0))
    s = np.linspace(1.0, 1.0 / steps, steps)
    s = sh * s / (1 + (sh - 1) * s)
    return [float(v) for v in s] + [0.0]


class SD3Pipeline:
    def __init__(self, path: str, device: str = "cpu", max_sequence_length: int = 256, clip_skip: int = 0):
        from transformers import CLIPTokenizer, PreTrainedTokenizerFast

        from .musicgen import T5Encoder
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.clip_skip = clip_skip
        self.te1 = StableDiffusion._load_text(os.path.join(path, "text_encoder"))
        self.te2 = StableDiffusion._load_text(os.path.join(path, "text_encoder_2"))
        self.tok1 = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer"))
        self.tok2 = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer_2"))
        self.t5 = self.tok3 = None
        t3 = os.path.join(path, "text_encoder_3")
        if os.path.isdir(t3):
            t5c = _cfg(os.path.join(t3, "config.json"))
            hp = {k: t5c[k] for k in ("num_heads", "d_kv", "num_layers", "relative_attention_num_buckets",
                                     "relative_attention_max_distance", "feed_forward_proj", "layer_norm_epsilon")}
            self.t5 = T5Encoder({k: v.to(self.device, self.dtype) for k, v in _load_weights(t3).items()}, hp, prefix="")
            self.tok3 = PreTrainedTokenizerFast.from_pretrained(os.path.join(path, "tokenizer_3"))
        tc = _cfg(os.path.join(path, "transformer", "config.json"))
        self.tr = SD3Transformer(tc)
        sd = _load_weights(os.path.join(path, "transformer"))
        if "pos_embed.pos_embed" not in sd:  # non-persistent table (no pos_embed_max_size): computed
            sd["pos_embed.pos_embed"] = self.tr.pos_embed.pos_embed
        self.tr.load_state_dict(sd, strict=True)
        self.t5_dim = int(tc.get("joint_attention_dim", 4096))
        vc = _cfg(os.path.join(path, "vae", "config.json"))
        self.vae = VaeDecoder(vc)
        self.vae.load_state_dict(_vae_names(_load_weights(os.path.join(path, "vae"))), strict=True)
        for m in (self.te1, self.te2, self.tr, self.vae):
            m.to(self.device, self.dtype).eval().requires_grad_(False)
        sc = os.path.join(path, "scheduler", "scheduler_config.json")
        self.sched_cfg = _cfg(sc) if os.path.isfile(sc) else {}
        self.max_len = self.te1.text_model.embeddings.position_embedding.weight.shape[0]
        self.max_seq = max_sequence_length
        self.vae_scale = 2 ** (len(self.vae.decoder.up_blocks) - 1)
        self.lat_ch = int(vc.get("latent_channels", 16))
        self.unet_sample_size = int(tc.get("sample_size", 128))
        self.controlnet = None
        self.use_graphs = self.device.type == "cuda" and os.environ.get("LOCALAI_AMD_SD_GRAPH", "1") != "0"
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.graph_cache = max(0, int(os.environ.get("LOCALAI_AMD_SD_GRAPH_CACHE", "4")))

    def encode(self, prompts: List[str]):
        """-> (context [B, 77 + T5 len, 4096], pooled [B, 2048]) (StableDiffusion3Pipeline.encode_prompt)."""
        hs, pools = [], []
        for tok, te in ((self.tok1, self.te1), (self.tok2, self.te2)):
            ids = tok(prompts, padding="max_length", max_length=self.max_len, truncation=True,
                      return_tensors="pt").input_ids.to(self.device)
            h, p = te.sdxl(ids, self.clip_skip, pooled=True)
            hs.append(h)
            pools.append(p)
        clip = torch.cat(hs, -1)
        clip = F.pad(clip, (0, self.t5_dim - clip.shape[-1]))
        if self.t5 is not None:
            ids = self.tok3(prompts, padding="max_length", max_length=self.max_seq, truncation=True,
                            return_tensors="pt").input_ids.to(self.device)
            t5 = self.t5(ids).to(clip.dtype)
        else:
            t5 = torch.zeros(len(prompts), self.max_seq, self.t5_dim, dtype=clip.dtype, device=self.device)
        return torch.cat([clip, t5], 1), torch.cat(pools, -1)

    def _step(self, *ins):
        if not self.use_graphs:
            return self.tr(*ins)
        key = tuple(tuple(v.shape) for v in ins)
        gr = self._graphs.get(key)
        if gr is None:
            out = self.tr(*ins)
            if self.graph_cache == 0:
                return out
            while len(self._graphs) >= self.graph_cache:
                self._graphs.popitem(last=False)
                torch.cuda.empty_cache()
            try:
                st = tuple(v.clone() for v in ins)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    so = self.tr(*st)
                self._graphs[key] = (graph, st, so)
            except Exception as e:  # noqa: BLE001
                import logging
                logging.getLogger(__name__).warning("sd3: transformer graph capture failed (%r); eager", e)
                self.use_graphs = False
            return out
        self._graphs.move_to_end(key)
        graph, st, so = gr
        for d, s in zip(st, ins):
            d.copy_(s)
        graph.replay()
        return so.clone()

    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: str = "", width: int = 1024, height: int = 1024,
                 steps: int = 28, guidance_scale: float = 7.0, seed: Optional[int] = None, image=None,
                 control_image=None) -> torch.Tensor:
        if image is not None or control_image is not None:
            raise ValueError("StableDiffusion3Pipeline here is text-to-image only (no src image)")
        g = torch.Generator().manual_seed(seed if seed is not None else int.from_bytes(os.urandom(4), "little"))
        q = self.vae_scale * self.tr.p
        H, W = max(q, height // q * q), max(q, width // q * q)
        cfg = guidance_scale > 1.0
        ctx, pooled = self.encode([negative_prompt, prompt] if cfg else [prompt])
        x = torch.randn(1, self.lat_ch, H // self.vae_scale, W // self.vae_scale, generator=g).to(self.device)

        def velocity(xv, s):
            xin = torch.cat([xv, xv]) if cfg else xv
            t = torch.full((xin.shape[0],), s * 1000.0, device=self.device)
            v = self._step(xin.to(self.dtype), ctx.to(self.dtype), pooled.to(self.dtype), t).float()
            if cfg:
                u, c = v.chunk(2)
                v = u + guidance_scale * (c - u)
            return v
        x = flow_euler(velocity, x.float(), sd3_sigmas(max(1, steps), self.sched_cfg))
        img = self.vae(x.to(self.dtype)).float()
        img = ((img[0] / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)
        return img.permute(1, 2, 0).cpu()

    def save(self, img: torch.Tensor, dst: str):
        from PIL import Image
        Image.fromarray(img.numpy()).save(dst)
