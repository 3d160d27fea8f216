"""FLUX.1 text-to-image (diffusers FluxPipeline layout), served by the `diffusers` backend with
`pipeline_type: FluxPipeline` (reference: `backend/python/diffusers/backend.py:247-251` loads
FluxPipeline in bf16; GenerateImage passes `guidance_scale = CFGScale` (7 when unset),
`num_inference_steps`, width / height and `max_sequence_length = 256`, backend.py:424-466).

* text: CLIP-L pooled output (final-LN state at the first EOS token) and T5 encoder states
  (`text_encoder_2`, max 256 tokens) -- the T5 stack is models/musicgen.py's;
* FluxTransformer2DModel: 2x2-patch-packed 16-channel latents, timestep / distilled-guidance /
  pooled-text conditioning, 3-axis RoPE over (0, row, col) image ids and zero text ids,
  `num_layers` double-stream MMDiT blocks (separate AdaLN-Zero modulation, QKV with RMS-normed
  q/k, MLPs for image and text tokens; joint attention over [text | image]) then
  `num_single_layers` single-stream blocks (fused attention + MLP over the concatenation), then
  AdaLN-continuous output norm and projection; module names follow diffusers so
  `load_state_dict(strict=True)` checks every weight;
* FlowMatch Euler sampler with resolution-dependent shift (use_dynamic_shifting: mu from the image
  token count, the scheduler config's base/max shift);
* the 16-channel KL-VAE decoder (shift_factor, no post-quant conv) from models/sd.py.

On the GPU everything runs in bf16 (PyTorch SDPA attention, hipBLASLt GEMMs) and the transformer
step replays from a hipGraph per shape.  Parity unpinned: diffusers is not installed here; the
text encoders are checked against transformers, the sampler in closed form.
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .sd import ClipTextEncoder, VaeDecoder, _cfg, _load_weights, _vae_names


def _timestep_embedding(t: torch.Tensor, dim: int = 256) -> torch.Tensor:
    """diffusers Timesteps(dim, flip_sin_to_cos=True, downscale_freq_shift=0)."""
    half = dim // 2
    f = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / half)
    e = t.float()[:, None] * f[None]
    return torch.cat([torch.cos(e), torch.sin(e)], -1)


class _TEmb(nn.Module):
    """TimestepEmbedding / PixArtAlphaTextProjection: linear_1 -> SiLU -> linear_2."""

    def __init__(self, cin: int, d: int):
        super().__init__()
        self.linear_1, self.linear_2 = nn.Linear(cin, d), nn.Linear(d, d)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class _RMS(nn.Module):
    def __init__(self, d: int, eps: float = 1e-6):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        v = x.float().pow(2).mean(-1, keepdim=True)
        return (x.float() * torch.rsqrt(v + self.eps)).to(x.dtype) * self.weight


def _rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """diffusers apply_rotary_emb(use_real, repeat_interleave_real): adjacent pairs rotate."""
    xr = x.float().unflatten(-1, (-1, 2))
    x0, x1 = xr[..., 0], xr[..., 1]
    rot = torch.stack([-x1, x0], -1).flatten(-2)
    return (x.float() * cos + rot * sin).to(x.dtype)


def _ln(x):
    return F.layer_norm(x, (x.shape[-1],), eps=1e-6)


def _mod(x, shift, scale):
    return x * (1 + scale[:, None]) + shift[:, None]


class _Attn(nn.Module):
    def __init__(self, d: int, heads: int, added: bool, out: bool):
        super().__init__()
        self.heads = heads
        self.to_q, self.to_k, self.to_v = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
        hd = d // heads
        self.norm_q, self.norm_k = _RMS(hd), _RMS(hd)
        if added:
            self.add_q_proj, self.add_k_proj, self.add_v_proj = nn.Linear(d, d), nn.Linear(d, d), nn.Linear(d, d)
            self.norm_added_q, self.norm_added_k = _RMS(hd), _RMS(hd)
            self.to_add_out = nn.Linear(d, d)
        if out:
            self.to_out = nn.ModuleList([nn.Linear(d, d)])

    def _qkv(self, x, q, k, v, nq, nk):
        B, L, D = x.shape
        sh = lambda t: t.view(B, L, self.heads, -1).transpose(1, 2)  # noqa: E731
        return nq(sh(q(x))), nk(sh(k(x))), sh(v(x))

    def forward(self, x, cos, sin, ctx=None):
        q, k, v = self._qkv(x, self.to_q, self.to_k, self.to_v, self.norm_q, self.norm_k)
        if ctx is not None:  # joint attention: [text | image] tokens
            cq, ck, cv = self._qkv(ctx, self.add_q_proj, self.add_k_proj, self.add_v_proj,
                                   self.norm_added_q, self.norm_added_k)
            q, k, v = torch.cat([cq, q], 2), torch.cat([ck, k], 2), torch.cat([cv, v], 2)
        q, k = _rope(q, cos, sin), _rope(k, cos, sin)
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).flatten(2)
        if ctx is None:
            return o
        T = ctx.shape[1]
        return self.to_out[0](o[:, T:]), self.to_add_out(o[:, :T])


class _FF(nn.Module):
    def __init__(self, d: int):
        super().__init__()
        self.net = nn.ModuleList([nn.Module(), nn.Identity(), nn.Linear(4 * d, d)])
        self.net[0].proj = nn.Linear(d, 4 * d)

    def forward(self, x):
        return self.net[2](F.gelu(self.net[0].proj(x), approximate="tanh"))


class _DoubleBlock(nn.Module):
    def __init__(self, d: int, heads: int):
        super().__init__()
        self.norm1, self.norm1_context = nn.Module(), nn.Module()
        self.norm1.linear, self.norm1_context.linear = nn.Linear(d, 6 * d), nn.Linear(d, 6 * d)
        self.attn = _Attn(d, heads, added=True, out=True)
        self.ff, self.ff_context = _FF(d), _FF(d)

    def forward(self, x, ctx, temb, cos, sin):
        e = self.norm1.linear(F.silu(temb)).chunk(6, -1)
        c = self.norm1_context.linear(F.silu(temb)).chunk(6, -1)
        a, ca = self.attn(_mod(_ln(x), e[0], e[1]), cos, sin, _mod(_ln(ctx), c[0], c[1]))
        x = x + e[2][:, None] * a
        x = x + e[5][:, None] * self.ff(_mod(_ln(x), e[3], e[4]))
        ctx = ctx + c[2][:, None] * ca
        ctx = ctx + c[5][:, None] * self.ff_context(_mod(_ln(ctx), c[3], c[4]))
        return x, ctx


class _SingleBlock(nn.Module):
    def __init__(self, d: int, heads: int):
        super().__init__()
        self.norm = nn.Module()
        self.norm.linear = nn.Linear(d, 3 * d)
        self.proj_mlp = nn.Linear(d, 4 * d)
        self.attn = _Attn(d, heads, added=False, out=False)
        self.proj_out = nn.Linear(5 * d, d)

    def forward(self, x, temb, cos, sin):
        shift, scale, gate = self.norm.linear(F.silu(temb)).chunk(3, -1)
        h = _mod(_ln(x), shift, scale)
        o = torch.cat([self.attn(h, cos, sin), F.gelu(self.proj_mlp(h), approximate="tanh")], -1)
        return x + gate[:, None] * self.proj_out(o)


class FluxTransformer(nn.Module):
    """diffusers FluxTransformer2DModel (patch_size 1 over 2x2-packed latents)."""

    def __init__(self, c: dict):
        super().__init__()
        heads, hd = int(c.get("num_attention_heads", 24)), int(c.get("attention_head_dim", 128))
        d = heads * hd
        self.axes = list(c.get("axes_dims_rope", [16, 56, 56]))
        if sum(self.axes) != hd:
            raise ValueError("axes_dims_rope must sum to attention_head_dim")
        self.guidance = bool(c.get("guidance_embeds", False))
        cin = int(c.get("in_channels", 64))
        self.x_embedder = nn.Linear(cin, d)
        self.context_embedder = nn.Linear(int(c.get("joint_attention_dim", 4096)), d)
        te = nn.Module()
        te.timestep_embedder = _TEmb(256, d)
        if self.guidance:
            te.guidance_embedder = _TEmb(256, d)
        te.text_embedder = _TEmb(int(c.get("pooled_projection_dim", 768)), d)
        self.time_text_embed = te
        self.transformer_blocks = nn.ModuleList(_DoubleBlock(d, heads) for _ in range(int(c.get("num_layers", 19))))
        self.single_transformer_blocks = nn.ModuleList(
            _SingleBlock(d, heads) for _ in range(int(c.get("num_single_layers", 38))))
        self.norm_out = nn.Module()
        self.norm_out.linear = nn.Linear(d, 2 * d)
        self.proj_out = nn.Linear(d, int(c.get("out_channels") or cin))

    def rope(self, ids: torch.Tensor):
        """ids [L, 3] -> (cos, sin) [L, head_dim] (theta 10000, one band per axis, pairs repeated)."""
        cs, sn = [], []
        for i, dim in enumerate(self.axes):
            f = 1.0 / (10000 ** (torch.arange(0, dim, 2, dtype=torch.float64, device=ids.device) / dim))
            ang = ids[:, i].double()[:, None] * f[None]
            cs.append(ang.cos().repeat_interleave(2, -1))
            sn.append(ang.sin().repeat_interleave(2, -1))
        return torch.cat(cs, -1).float(), torch.cat(sn, -1).float()

    def forward(self, x, ctx, pooled, t, guidance, cos, sin):
        """x [B, N, 64] packed latents; ctx [B, T, 4096]; pooled [B, 768]; t / guidance [B] in
        [0, 1] (x1000 inside, as diffusers does); cos / sin [T + N, head_dim]."""
        te = self.time_text_embed
        temb = te.timestep_embedder(_timestep_embedding(t * 1000).to(x.dtype))
        if self.guidance:
            temb = temb + te.guidance_embedder(_timestep_embedding(guidance * 1000).to(x.dtype))
        temb = temb + te.text_embedder(pooled.to(x.dtype))
        h, c = self.x_embedder(x), self.context_embedder(ctx)
        for b in self.transformer_blocks:
            h, c = b(h, c, temb, cos, sin)
        h = torch.cat([c, h], 1)
        for b in self.single_transformer_blocks:
            h = b(h, temb, cos, sin)
        h = h[:, c.shape[1]:]
        scale, shift = self.norm_out.linear(F.silu(temb)).chunk(2, -1)
        return self.proj_out(_mod(_ln(h), shift, scale))


# ------------------------------------------------------------------ sampler
def flow_sigmas(steps: int, image_seq_len: int, cfg: dict) -> List[float]:
    """FlowMatchEulerDiscreteScheduler.set_timesteps as FluxPipeline drives it: sigmas
    linspace(1, 1/steps), time-shifted by mu (dynamic: linear in the image token count between
    base/max_image_seq_len) or by `shift`; a final 0."""
    s = np.linspace(1.0, 1.0 / steps, steps)
    if cfg.get("use_dynamic_shifting", False):
        b0, b1 = int(cfg.get("base_image_seq_len", 256)), int(cfg.get("max_image_seq_len", 4096))
        s0, s1 = float(cfg.get("base_shift", 0.5)), float(cfg.get("max_shift", 1.15))
        mu = image_seq_len * (s1 - s0) / (b1 - b0) + (s0 - (s1 - s0) / (b1 - b0) * b0)
        s = math.exp(mu) / (math.exp(mu) + (1.0 / s - 1.0))
    else:
        sh = float(cfg.get("shift", 1.0))
        s = sh * s / (1 + (sh - 1) * s)
    return [float(v) for v in s] + [0.0]


def flow_euler(velocity, x: torch.Tensor, sigmas: Sequence[float]) -> torch.Tensor:
    """x_{i+1} = x_i + (sigma_{i+1} - sigma_i) * v(x_i, sigma_i) (flow matching: x_s = (1-s) x0 + s n)."""
    for s0, s1 in zip(sigmas[:-1], sigmas[1:]):
        x = x + (s1 - s0) * velocity(x, s0)
    return x


def is_flux_pipeline(path: str) -> bool:
    mi = os.path.join(path, "model_index.json")
    if not os.path.isfile(mi):
        return False
    try:
        return str(_cfg(mi).get("_class_name", "")).startswith("Flux")
    except (OSError, ValueError):
        return False


class FluxPipeline:
    def __init__(self, path: str, device: str = "cpu", max_sequence_length: int = 256,
                 transformer_file: Optional[str] = None):
        """path: a diffusers FLUX directory; transformer_file: a single-file transformer (BFL
        layout, models/flux_single_file.py) replacing path/transformer (pipeline_type
        FluxTransformer2DModel, reference backend.py:255-269)."""
        from transformers import CLIPTokenizer, PreTrainedTokenizerFast

        from .musicgen import T5Encoder
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.text = StableDiffusionTextLoader.load(os.path.join(path, "text_encoder"))
        t5c = _cfg(os.path.join(path, "text_encoder_2", "config.json"))
        self.t5_hp = {k: t5c[k] for k in ("num_heads", "d_kv", "num_layers", "relative_attention_num_buckets",
                                         "relative_attention_max_distance", "feed_forward_proj",
                                         "layer_norm_epsilon")}
        w2 = {k: v.to(self.device, self.dtype) for k, v in _load_weights(os.path.join(path, "text_encoder_2")).items()}
        self.t5 = T5Encoder(w2, self.t5_hp, prefix="")
        if transformer_file:
            from .flux_single_file import load_transformer_file
            tc, tw = load_transformer_file(transformer_file, path)
        else:
            tc = _cfg(os.path.join(path, "transformer", "config.json"))
            tw = _load_weights(os.path.join(path, "transformer"))
        self.tr = FluxTransformer(tc)
        self.tr.load_state_dict(tw, strict=True)
        vc = _cfg(os.path.join(path, "vae", "config.json"))
        self.vae = VaeDecoder(vc)
        self.vae.load_state_dict(_vae_names(_load_weights(os.path.join(path, "vae"))), strict=True)
        for m in (self.text, self.tr, self.vae):
            m.to(self.device, self.dtype).eval().requires_grad_(False)
        sc = os.path.join(path, "scheduler", "scheduler_config.json")
        self.sched_cfg = _cfg(sc) if os.path.isfile(sc) else {}
        self.tok = CLIPTokenizer.from_pretrained(os.path.join(path, "tokenizer"))
        self.tok2 = PreTrainedTokenizerFast.from_pretrained(os.path.join(path, "tokenizer_2"))
        self.max_len = self.text.text_model.embeddings.position_embedding.weight.shape[0]
        self.max_seq = max_sequence_length
        self.vae_scale = 2 ** (len(self.vae.decoder.up_blocks) - 1)
        self.lat_ch = int(vc.get("latent_channels", 16))
        self.unet_sample_size = int(tc.get("sample_size", 128))
        self.use_graphs = self.device.type == "cuda" and os.environ.get("LOCALAI_AMD_SD_GRAPH", "1") != "0"
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self.graph_cache = max(0, int(os.environ.get("LOCALAI_AMD_SD_GRAPH_CACHE", "4")))

    def encode(self, prompt: str):
        """-> (T5 states [1, max_seq, 4096], CLIP pooled [1, 768]) (FluxPipeline.encode_prompt)."""
        ids = self.tok([prompt], padding="max_length", max_length=self.max_len, truncation=True,
                       return_tensors="pt").input_ids.to(self.device)
        _, pooled = self.text.sdxl(ids, 0, pooled=True)
        t = self.tok2([prompt], padding="max_length", max_length=self.max_seq, truncation=True,
                      return_tensors="pt").input_ids.to(self.device)
        return self.t5(t).to(self.dtype), pooled

    def _step(self, x, ctx, pooled, t, g, cos, sin):
        ins = (x, ctx, pooled, t, g, cos, sin)
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
                logging.getLogger(__name__).warning("flux: transformer graph capture failed (%r); eager", e)
                self.use_graphs = False
            return out
        self._graphs.move_to_end(key)
        graph, st, so = gr
        for d, s in zip(st, ins):
            d.copy_(s)
        graph.replay()
        return so.clone()

    # no_grad, not inference_mode, around every pipeline that captures hipGraphs: a capture under
    # inference_mode creates the CUDA generator's graph-state tensors as inference tensors, and
    # every later capture outside it (the LLM engine's decode graphs) then fails
    @torch.no_grad()
    def __call__(self, prompt: str, negative_prompt: str = "", width: int = 1024, height: int = 1024,
                 steps: int = 28, guidance_scale: float = 3.5, seed: Optional[int] = None, image=None,
                 control_image=None) -> torch.Tensor:
        """-> uint8 [H, W, 3] (FluxPipeline.__call__ with distilled guidance; no negative prompt)."""
        if image is not None or control_image is not None:
            raise ValueError("FluxPipeline is text-to-image only (no src image)")
        g = torch.Generator().manual_seed(seed if seed is not None else int.from_bytes(os.urandom(4), "little"))
        pack = self.vae_scale * 2
        H, W = max(pack, height // pack * pack), max(pack, width // pack * pack)
        h2, w2 = H // pack, W // pack        # packed token grid
        ctx, pooled = self.encode(prompt)
        noise = torch.randn(1, self.lat_ch, 2 * h2, 2 * w2, generator=g)
        x = noise.view(1, self.lat_ch, h2, 2, w2, 2).permute(0, 2, 4, 1, 3, 5).reshape(1, h2 * w2, self.lat_ch * 4)
        x = x.to(self.device)
        img_ids = torch.zeros(h2, w2, 3)
        img_ids[..., 1] = torch.arange(h2)[:, None]
        img_ids[..., 2] = torch.arange(w2)[None, :]
        ids = torch.cat([torch.zeros(ctx.shape[1], 3), img_ids.view(-1, 3)], 0).to(self.device)
        cos, sin = (v.to(self.dtype) for v in self.tr.rope(ids))
        gt = torch.full((1,), float(guidance_scale), device=self.device)
        sig = flow_sigmas(max(1, steps), h2 * w2, self.sched_cfg)

        def velocity(xv, s):
            t = torch.full((1,), s, device=self.device)
            return self._step(xv.to(self.dtype), ctx, pooled.to(self.dtype), t, gt, cos, sin).float()
        x = flow_euler(velocity, x.float(), sig)
        lat = x.view(1, h2, w2, self.lat_ch, 2, 2).permute(0, 3, 1, 4, 2, 5).reshape(1, self.lat_ch, 2 * h2, 2 * w2)
        img = self.vae(lat.to(self.dtype)).float()
        img = ((img[0] / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)
        return img.permute(1, 2, 0).cpu()

    def save(self, img: torch.Tensor, dst: str):
        from PIL import Image
        Image.fromarray(img.numpy()).save(dst)


class StableDiffusionTextLoader:
    @staticmethod
    def load(d: str) -> ClipTextEncoder:
        from .sd import StableDiffusion
        return StableDiffusion._load_text(d)
