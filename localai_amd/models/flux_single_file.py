"""Single-file FLUX transformers: the Black Forest Labs checkpoint layout (`flux1-dev.safetensors`,
`double_blocks.*` / `single_blocks.*`) mapped onto models/flux.py's FluxTransformer (diffusers
FluxTransformer2DModel names), for the diffusers backend's `pipeline_type: FluxTransformer2DModel`.

Reference: `backend/python/diffusers/backend.py:255-269` loads the transformer with
`FluxTransformer2DModel.from_single_file(modelFile)` and takes the rest of the pipeline (CLIP, T5,
VAE, scheduler, tokenizers) from `BFL_REPO` (default `ChuckMcSneed/FLUX.1-dev`); it then
quantises the transformer and T5 to float8 (optimum.quanto) to fit small GPUs.  Here BFL_REPO
names a local diffusers FLUX directory (no network) and both run in bf16: a 288 GB MI355X holds
the 12 B transformer (24 GB) without weight quantisation.

Layout facts the mapping relies on (the public BFL `flux/model.py` modules):
* fused projections are split: a double block's `img_attn.qkv` / `txt_attn.qkv` into
  to_q|to_k|to_v and add_q|add_k|add_v; a single block's `linear1` into q|k|v|proj_mlp;
* per-head RMS norms are `*.norm.query_norm.scale` / `key_norm.scale`;
* `final_layer.adaLN_modulation.1` emits (shift, scale) where AdaLayerNormContinuous reads
  (scale, shift): its two halves are swapped; the block modulations keep their order
  (shift, scale, gate [x2]).
Parity unpinned: diffusers is not installed here and no real FLUX file is available, so the
tests check the mapping as an exact inverse pair and the forward on a synthetic checkpoint.
"""
from __future__ import annotations

import json
import os
import re
from typing import Dict, Optional

import torch

_TOP = {
    "img_in": "x_embedder",
    "txt_in": "context_embedder",
    "time_in.in_layer": "time_text_embed.timestep_embedder.linear_1",
    "time_in.out_layer": "time_text_embed.timestep_embedder.linear_2",
    "vector_in.in_layer": "time_text_embed.text_embedder.linear_1",
    "vector_in.out_layer": "time_text_embed.text_embedder.linear_2",
    "guidance_in.in_layer": "time_text_embed.guidance_embedder.linear_1",
    "guidance_in.out_layer": "time_text_embed.guidance_embedder.linear_2",
    "final_layer.linear": "proj_out",
}
_DOUBLE = {
    "img_mod.lin": "norm1.linear",
    "txt_mod.lin": "norm1_context.linear",
    "img_attn.proj": "attn.to_out.0",
    "txt_attn.proj": "attn.to_add_out",
    "img_mlp.0": "ff.net.0.proj",
    "img_mlp.2": "ff.net.2",
    "txt_mlp.0": "ff_context.net.0.proj",
    "txt_mlp.2": "ff_context.net.2",
}
_DOUBLE_NORMS = {
    "img_attn.norm.query_norm.scale": "attn.norm_q.weight",
    "img_attn.norm.key_norm.scale": "attn.norm_k.weight",
    "txt_attn.norm.query_norm.scale": "attn.norm_added_q.weight",
    "txt_attn.norm.key_norm.scale": "attn.norm_added_k.weight",
}
_SINGLE = {"linear2": "proj_out", "modulation.lin": "norm.linear"}
_SINGLE_NORMS = {"norm.query_norm.scale": "attn.norm_q.weight", "norm.key_norm.scale": "attn.norm_k.weight"}


def is_bfl(sd: Dict[str, torch.Tensor]) -> bool:
    return any(k.startswith("double_blocks.") for k in sd) and "img_in.weight" in sd


def _strip(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Checkpoints saved from a wrapper carry a `model.diffusion_model.` prefix."""
    p = "model.diffusion_model."
    if any(k.startswith(p) for k in sd):
        return {k[len(p):]: v for k, v in sd.items() if k.startswith(p)}
    return sd


def _swap_halves(t: torch.Tensor) -> torch.Tensor:
    a, b = t.chunk(2, 0)
    return torch.cat([b, a], 0)


def bfl_to_diffusers(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """BFL FLUX transformer state dict -> FluxTransformer (diffusers) names; every key is consumed."""
    sd = _strip(sd)
    out: Dict[str, torch.Tensor] = {}
    used = set()
    d = sd["img_in.weight"].shape[0]
    for k, v in sd.items():
        for src, dst in _TOP.items():
            if k.startswith(src + "."):
                out[dst + k[len(src):]] = v
                used.add(k)
        if k.startswith("final_layer.adaLN_modulation.1."):
            out["norm_out.linear." + k.rsplit(".", 1)[1]] = _swap_halves(v)
            used.add(k)
    for k, v in sd.items():
        m = re.match(r"double_blocks\.(\d+)\.(.+)$", k)
        if m:
            i, rest = m.group(1), m.group(2)
            pre = f"transformer_blocks.{i}."
            if rest in _DOUBLE_NORMS:
                out[pre + _DOUBLE_NORMS[rest]] = v
            elif rest.startswith(("img_attn.qkv.", "txt_attn.qkv.")):
                names = ("to_q", "to_k", "to_v") if rest.startswith("img") else ("add_q_proj", "add_k_proj",
                                                                                  "add_v_proj")
                for n, part in zip(names, v.chunk(3, 0)):
                    out[pre + "attn." + n + "." + rest.rsplit(".", 1)[1]] = part
            else:
                base, leaf = rest.rsplit(".", 1)
                if base not in _DOUBLE:
                    raise KeyError(f"unknown FLUX double-block tensor {k}")
                out[pre + _DOUBLE[base] + "." + leaf] = v
            used.add(k)
            continue
        m = re.match(r"single_blocks\.(\d+)\.(.+)$", k)
        if m:
            i, rest = m.group(1), m.group(2)
            pre = f"single_transformer_blocks.{i}."
            if rest in _SINGLE_NORMS:
                out[pre + _SINGLE_NORMS[rest]] = v
            elif rest.startswith("linear1."):
                leaf = rest.rsplit(".", 1)[1]
                q, kk, vv, mlp = torch.split(v, [d, d, d, v.shape[0] - 3 * d], 0)
                out[pre + "attn.to_q." + leaf], out[pre + "attn.to_k." + leaf] = q, kk
                out[pre + "attn.to_v." + leaf], out[pre + "proj_mlp." + leaf] = vv, mlp
            else:
                base, leaf = rest.rsplit(".", 1)
                if base not in _SINGLE:
                    raise KeyError(f"unknown FLUX single-block tensor {k}")
                out[pre + _SINGLE[base] + "." + leaf] = v
            used.add(k)
    left = sorted(set(sd) - used)
    if left:
        raise KeyError(f"unmapped FLUX tensors: {left[:8]}")
    return out


def diffusers_to_bfl(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """The inverse mapping (synthetic single files for the tests, export)."""
    inv_top = {v: k for k, v in _TOP.items()}
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        for dst, src in inv_top.items():
            if k.startswith(dst + "."):
                out[src + k[len(dst):]] = v
        if k.startswith("norm_out.linear."):
            out["final_layer.adaLN_modulation.1." + k.rsplit(".", 1)[1]] = _swap_halves(v)
    n_double = 1 + max([int(m.group(1)) for k in sd for m in [re.match(r"transformer_blocks\.(\d+)\.", k)] if m],
                       default=-1)
    n_single = 1 + max([int(m.group(1)) for k in sd
                        for m in [re.match(r"single_transformer_blocks\.(\d+)\.", k)] if m], default=-1)
    for i in range(n_double):
        pre = f"transformer_blocks.{i}."
        for src, dst in _DOUBLE.items():
            for leaf in ("weight", "bias"):
                if pre + dst + "." + leaf in sd:
                    out[f"double_blocks.{i}.{src}.{leaf}"] = sd[pre + dst + "." + leaf]
        for src, dst in _DOUBLE_NORMS.items():
            out[f"double_blocks.{i}.{src}"] = sd[pre + dst]
        for side, names in (("img", ("to_q", "to_k", "to_v")), ("txt", ("add_q_proj", "add_k_proj", "add_v_proj"))):
            for leaf in ("weight", "bias"):
                out[f"double_blocks.{i}.{side}_attn.qkv.{leaf}"] = torch.cat(
                    [sd[pre + "attn." + n + "." + leaf] for n in names], 0)
    for i in range(n_single):
        pre = f"single_transformer_blocks.{i}."
        for src, dst in _SINGLE.items():
            for leaf in ("weight", "bias"):
                out[f"single_blocks.{i}.{src}.{leaf}"] = sd[pre + dst + "." + leaf]
        for src, dst in _SINGLE_NORMS.items():
            out[f"single_blocks.{i}.{src}"] = sd[pre + dst]
        for leaf in ("weight", "bias"):
            out[f"single_blocks.{i}.linear1.{leaf}"] = torch.cat(
                [sd[pre + f"attn.to_{n}.{leaf}"] for n in ("q", "k", "v")] + [sd[pre + f"proj_mlp.{leaf}"]], 0)
    return out


def infer_config(sd: Dict[str, torch.Tensor], base: Optional[dict] = None) -> dict:
    """FluxTransformer2DModel config from the tensor shapes (the base pipeline's transformer
    config supplies what shapes cannot: axes_dims_rope)."""
    sd = _strip(sd)
    d, cin = sd["img_in.weight"].shape
    hd = int(sd["double_blocks.0.img_attn.norm.query_norm.scale"].shape[0])
    c = dict(base or {})
    c.update({
        "_class_name": "FluxTransformer2DModel",
        "in_channels": int(cin),
        "out_channels": int(sd["final_layer.linear.weight"].shape[0]),
        "num_layers": len({k.split(".")[1] for k in sd if k.startswith("double_blocks.")}),
        "num_single_layers": len({k.split(".")[1] for k in sd if k.startswith("single_blocks.")}),
        "attention_head_dim": hd,
        "num_attention_heads": int(d) // hd,
        "joint_attention_dim": int(sd["txt_in.weight"].shape[1]),
        "pooled_projection_dim": int(sd["vector_in.in_layer.weight"].shape[1]),
        "guidance_embeds": "guidance_in.in_layer.weight" in sd,
    })
    axes = c.get("axes_dims_rope")
    if not axes or sum(axes) != hd:
        # FLUX.1: (16, 56, 56) for 128-wide heads; other widths keep the same proportions (even sizes)
        a0 = max(2, (hd // 8) // 2 * 2)
        a1 = (hd - a0) // 2 // 2 * 2
        c["axes_dims_rope"] = [a0, a1, hd - a0 - a1]
    return c


def load_transformer_file(path: str, base_dir: Optional[str] = None):
    """(config, diffusers-named state dict) of a single-file FLUX transformer (BFL layout, or a
    diffusers-named single file).  Safetensors only: pickled checkpoints are loaded weights-only."""
    from .sd_single_file import load_checkpoint
    sd, hints = load_checkpoint(path)
    base = None
    if base_dir and os.path.isfile(os.path.join(base_dir, "transformer", "config.json")):
        with open(os.path.join(base_dir, "transformer", "config.json")) as f:
            base = json.load(f)
    hint = (hints or {}).get("flux_config")
    if hint:
        base = dict(base or {}, **hint)
    if is_bfl(_strip(sd)):
        return infer_config(sd, base), bfl_to_diffusers(sd)
    if base is None:
        raise ValueError(f"{path}: diffusers-named FLUX transformer without a base transformer config")
    return base, sd


def write_bfl_file(transformer_sd: Dict[str, torch.Tensor], dst: str, axes=None) -> str:
    """Save a diffusers-named FluxTransformer state dict as a BFL-layout single file."""
    from safetensors.torch import save_file

    from .sd_single_file import META_KEY
    meta = {META_KEY: json.dumps({"flux_config": {"axes_dims_rope": list(axes)}})} if axes else None
    save_file({k: v.contiguous() for k, v in diffusers_to_bfl(transformer_sd).items()}, dst, metadata=meta)
    return dst
