"""Single-file Stable Diffusion 3 / 3.5 checkpoints (Stability's `sd3_medium*.safetensors` layout:
MMDiT under `model.diffusion_model.` with its original names, the 16-channel VAE under
`first_stage_model.`, and -- in the `*_incl_clips*` files -- the text encoders under
`text_encoders.{clip_l,clip_g,t5xxl}.transformer.` in transformers layout) -> the diffusers
StableDiffusion3Pipeline directory models/sd3.py loads.

Reference: `backend/python/diffusers/backend.py:238-242` calls
`StableDiffusion3Pipeline.from_single_file(modelFile)` when the model is a local file or a URL.
Here, as for SD 1.x/2.x/XL (models/sd_single_file.py), the file is converted ONCE into a hidden
sibling directory keyed by the file's size and mtime.

Layout facts the mapping relies on (the public SD3 reference implementation, `mmdit.py`):
* fused `attn.qkv` projections split into to_q|to_k|to_v (image) and add_q|add_k|add_v (text);
* per-head RMS q/k norms `attn.ln_q` / `attn.ln_k` (SD3.5) -> norm_q / norm_k (norm_added_* for text);
* the last joint block's context half is `pre_only` (no attention output projection, no MLP) and,
  like `final_layer.adaLN_modulation.1`, emits (shift, scale) where diffusers'
  AdaLayerNormContinuous reads (scale, shift): the two halves are swapped;
* x_embedder = the 2x2 patch convolution, `pos_embed` [1, S*S, D] the stored sin-cos table,
  t_embedder / y_embedder = timestep / pooled-text MLPs;
* the VAE has no quant / post-quant convolutions (scaling 1.5305, shift 0.0609).
Head width is 64 unless q/k norms give it (or the file's `localai_amd.configs` metadata does).
Text encoders missing from the file come from `tokenizer_dir` (the model config's `clip_model`,
a StableDiffusion3Pipeline directory) -- there is no hub to fetch them from.
Parity unpinned: diffusers is not installed and no real SD3 file is available; the tests check the
mapping as an exact inverse pair and the converted pipeline's output against the source pipeline.
"""
from __future__ import annotations

import json
import logging
import os
import re
import shutil
from typing import Dict, Optional

import torch

from .sd_single_file import META_KEY, UNET_P, VAE_P, load_checkpoint, vae_name_to_ldm

log = logging.getLogger(__name__)

TE_P = {"text_encoder": "text_encoders.clip_l.transformer.", "text_encoder_2": "text_encoders.clip_g.transformer.",
        "text_encoder_3": "text_encoders.t5xxl.transformer."}

_TOP = {
    "x_embedder.proj": "pos_embed.proj",
    "t_embedder.mlp.0": "time_text_embed.timestep_embedder.linear_1",
    "t_embedder.mlp.2": "time_text_embed.timestep_embedder.linear_2",
    "y_embedder.mlp.0": "time_text_embed.text_embedder.linear_1",
    "y_embedder.mlp.2": "time_text_embed.text_embedder.linear_2",
    "context_embedder": "context_embedder",
    "final_layer.linear": "proj_out",
}
_BLOCK = {
    "x_block.attn.proj": "attn.to_out.0",
    "x_block.mlp.fc1": "ff.net.0.proj",
    "x_block.mlp.fc2": "ff.net.2",
    "x_block.adaLN_modulation.1": "norm1.linear",
    "context_block.attn.proj": "attn.to_add_out",
    "context_block.mlp.fc1": "ff_context.net.0.proj",
    "context_block.mlp.fc2": "ff_context.net.2",
    "context_block.adaLN_modulation.1": "norm1_context.linear",
}
_NORMS = {
    "x_block.attn.ln_q.weight": "attn.norm_q.weight",
    "x_block.attn.ln_k.weight": "attn.norm_k.weight",
    "context_block.attn.ln_q.weight": "attn.norm_added_q.weight",
    "context_block.attn.ln_k.weight": "attn.norm_added_k.weight",
}
_QKV = {"x_block": ("to_q", "to_k", "to_v"), "context_block": ("add_q_proj", "add_k_proj", "add_v_proj")}


def is_sd3_file(sd: Dict[str, torch.Tensor]) -> bool:
    return any(k.startswith(UNET_P + "joint_blocks.") for k in sd)


def _swap_halves(t: torch.Tensor) -> torch.Tensor:
    a, b = t.chunk(2, 0)
    return torch.cat([b, a], 0)


def _n_blocks(sd, pat: str) -> int:
    return 1 + max([int(m.group(1)) for k in sd for m in [re.match(pat, k)] if m], default=-1)


def mmdit_to_diffusers(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """MMDiT names (without the `model.diffusion_model.` prefix) -> SD3Transformer2DModel names;
    every tensor is consumed."""
    if any(".attn2." in k for k in sd):
        raise ValueError("SD3.5 dual-attention (MMDiT-X) checkpoints are not supported")
    out: Dict[str, torch.Tensor] = {}
    used = set()
    n = _n_blocks(sd, r"joint_blocks\.(\d+)\.")
    for k, v in sd.items():
        if k == "pos_embed":
            out["pos_embed.pos_embed"] = v
            used.add(k)
            continue
        if k.startswith("final_layer.adaLN_modulation.1."):
            out["norm_out.linear." + k.rsplit(".", 1)[1]] = _swap_halves(v)
            used.add(k)
            continue
        for src, dst in _TOP.items():
            if k.startswith(src + "."):
                out[dst + k[len(src):]] = v
                used.add(k)
        m = re.match(r"joint_blocks\.(\d+)\.(.+)$", k)
        if not m:
            continue
        i, rest = int(m.group(1)), m.group(2)
        pre = f"transformer_blocks.{i}."
        used.add(k)
        if rest in _NORMS:
            out[pre + _NORMS[rest]] = v
            continue
        side = rest.split(".", 1)[0]
        if rest.startswith(side + ".attn.qkv."):
            for name, part in zip(_QKV[side], v.chunk(3, 0)):
                out[pre + "attn." + name + "." + rest.rsplit(".", 1)[1]] = part
            continue
        base, leaf = rest.rsplit(".", 1)
        if base not in _BLOCK:
            raise KeyError(f"unknown SD3 joint-block tensor {k}")
        if base == "context_block.adaLN_modulation.1" and i == n - 1:
            v = _swap_halves(v)  # pre_only context half: AdaLayerNormContinuous (scale, shift)
        out[pre + _BLOCK[base] + "." + leaf] = v
    left = sorted(set(sd) - used)
    if left:
        raise KeyError(f"unmapped SD3 tensors: {left[:8]}")
    return out


def diffusers_to_mmdit(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """The inverse mapping (synthetic single files for the tests, export)."""
    inv = {v: k for k, v in _TOP.items()}
    out: Dict[str, torch.Tensor] = {}
    n = _n_blocks(sd, r"transformer_blocks\.(\d+)\.")
    for k, v in sd.items():
        if k == "pos_embed.pos_embed":
            out["pos_embed"] = v
        elif k.startswith("norm_out.linear."):
            out["final_layer.adaLN_modulation.1." + k.rsplit(".", 1)[1]] = _swap_halves(v)
        else:
            for dst, src in inv.items():
                if k.startswith(dst + "."):
                    out[src + k[len(dst):]] = v
    for i in range(n):
        pre = f"transformer_blocks.{i}."
        for src, dst in _BLOCK.items():
            for leaf in ("weight", "bias"):
                t = sd.get(pre + dst + "." + leaf)
                if t is None:
                    continue
                if src == "context_block.adaLN_modulation.1" and i == n - 1:
                    t = _swap_halves(t)
                out[f"joint_blocks.{i}.{src}.{leaf}"] = t
        for src, dst in _NORMS.items():
            if pre + dst in sd:
                out[f"joint_blocks.{i}.{src}"] = sd[pre + dst]
        for side, names in _QKV.items():
            for leaf in ("weight", "bias"):
                out[f"joint_blocks.{i}.{side}.attn.qkv.{leaf}"] = torch.cat(
                    [sd[pre + "attn." + nm + "." + leaf] for nm in names], 0)
    return out


def infer_config(sd: Dict[str, torch.Tensor], hint: Optional[dict] = None) -> dict:
    """SD3Transformer2DModel config from the MMDiT tensor shapes."""
    w = sd["x_embedder.proj.weight"]
    d, cin, p = int(w.shape[0]), int(w.shape[1]), int(w.shape[2])
    ln_q = sd.get("joint_blocks.0.x_block.attn.ln_q.weight")
    hd = int(ln_q.shape[0]) if ln_q is not None else 64
    npos = int(sd["pos_embed"].shape[1]) if "pos_embed" in sd else 0
    c = {
        "_class_name": "SD3Transformer2DModel",
        "sample_size": 128, "patch_size": p, "in_channels": cin,
        "num_layers": _n_blocks(sd, r"joint_blocks\.(\d+)\."),
        "attention_head_dim": hd, "num_attention_heads": d // hd,
        "joint_attention_dim": int(sd["context_embedder.weight"].shape[1]),
        "caption_projection_dim": d,
        "pooled_projection_dim": int(sd["y_embedder.mlp.0.weight"].shape[1]),
        "out_channels": int(sd["final_layer.linear.weight"].shape[0]) // (p * p),
        "pos_embed_max_size": int(round(npos ** 0.5)) if npos else None,
    }
    if ln_q is not None:
        c["qk_norm"] = "rms_norm"
    if hint:
        c.update(hint)
    return c


def _vae(sd: Dict[str, torch.Tensor], hint: Optional[dict]):
    from . import sd as sdm
    v = {k[len(VAE_P):]: t for k, t in sd.items() if k.startswith(VAE_P)}
    if not v:
        raise ValueError("SD3 single file without its VAE (first_stage_model.*)")
    if hint:
        cfg = dict(hint)
    else:
        L = 1 + max(int(k.split(".")[2]) for k in v if k.startswith("decoder.up."))
        lpb = max(int(k.split(".")[4]) for k in v if k.startswith("decoder.up.0.block."))  # up blocks: lpb + 1
        ch = [int(v[f"decoder.up.{i}.block.0.conv2.weight"].shape[0]) for i in range(L)]
        # GroupNorm's group count is not in the weights: 32 (every published SD3 VAE) when it divides
        groups = next(g for g in (32, 16, 8, 4, 2, 1) if all(c % g == 0 for c in ch))
        cfg = dict(block_out_channels=ch, layers_per_block=lpb, latent_channels=int(v["decoder.conv_in.weight"].shape[1]),
                   norm_num_groups=groups, in_channels=3, out_channels=int(v["decoder.conv_out.weight"].shape[0]),
                   scaling_factor=1.5305, shift_factor=0.0609, use_quant_conv=False, use_post_quant_conv=False)
    out = {}
    for cls in (sdm.VaeDecoder, sdm.VaeEncoder):
        names = []
        with torch.device("meta"):
            names = list(cls(cfg).state_dict().keys())
        got = {}
        for nm in names:
            t = v.get(vae_name_to_ldm(nm, cfg))
            if t is None:
                got = None
                break
            if ".attentions." in nm and nm.endswith(".weight") and t.dim() == 4:
                t = t[:, :, 0, 0]
            got[nm] = t
        if got is None:
            if cls is sdm.VaeDecoder:
                raise ValueError("SD3 single-file VAE decoder incomplete")
            continue   # no encoder half: txt2img only
        out.update(got)
    return dict(cfg, _class_name="AutoencoderKL"), out


def convert(path: str, sd: Optional[Dict[str, torch.Tensor]] = None, hints: Optional[dict] = None,
            out_dir: Optional[str] = None, tokenizer_dir: Optional[str] = None) -> str:
    """Convert (once) and return the StableDiffusion3Pipeline directory of a single-file SD3
    checkpoint.  tokenizer_dir: a diffusers SD3 directory supplying the text encoders /
    tokenizers the file does not carry (and the tokenizers it never carries)."""
    from safetensors.torch import save_file
    st = os.stat(path)
    stamp = f"{st.st_size}:{int(st.st_mtime)}"
    if out_dir is None:
        out_dir = os.path.join(os.path.dirname(os.path.abspath(path)), "." + os.path.basename(path) + ".diffusers")
    mark = os.path.join(out_dir, ".source")
    if os.path.isfile(mark) and open(mark).read() == stamp:
        return out_dir
    if sd is None:
        sd, hints = load_checkpoint(path)
    hints = hints or {}
    tmp = out_dir + ".partial"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)

    def save(sub: str, cfg: dict, tensors: Dict[str, torch.Tensor], fname: str):
        os.makedirs(os.path.join(tmp, sub), exist_ok=True)
        with open(os.path.join(tmp, sub, "config.json"), "w") as f:
            json.dump(cfg, f)
        save_file({k: t.contiguous() for k, t in tensors.items()}, os.path.join(tmp, sub, fname))

    mm = {k[len(UNET_P):]: v for k, v in sd.items() if k.startswith(UNET_P)}
    save("transformer", infer_config(mm, hints.get("transformer")), mmdit_to_diffusers(mm),
         "diffusion_pytorch_model.safetensors")
    vcfg, vsd = _vae(sd, hints.get("vae"))
    save("vae", vcfg, vsd, "diffusion_pytorch_model.safetensors")
    base = tokenizer_dir if tokenizer_dir and os.path.isdir(tokenizer_dir) else None
    for sub, pre in TE_P.items():
        te = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        if te:
            if sub == "text_encoder_3":
                cfg = hints.get(sub) or _t5_config(te)
                cfg = dict(cfg, architectures=["T5EncoderModel"], model_type="t5")
            else:
                from .sd_single_file import _hf_clip_keys, infer_text_config
                te = _hf_clip_keys(te)
                cfg = hints.get(sub) or infer_text_config(te, "gelu", None)
                cfg = dict(cfg, architectures=["CLIPTextModelWithProjection"], model_type="clip_text_model")
            save(sub, cfg, te, "model.safetensors")
        elif base and os.path.isdir(os.path.join(base, sub)):
            shutil.copytree(os.path.join(base, sub), os.path.join(tmp, sub))
        elif sub != "text_encoder_3":
            raise ValueError(f"{path}: the file carries no {sub} (text_encoders.*): set the model's `clip_model` to "
                             "a StableDiffusion3Pipeline directory that supplies the text encoders")
    for tk, need in (("tokenizer", "text_encoder"), ("tokenizer_2", "text_encoder_2"), ("tokenizer_3", "text_encoder_3")):
        if not os.path.isdir(os.path.join(tmp, need)):
            continue
        src = os.path.join(base, tk) if base else None
        if src and os.path.isdir(src):
            shutil.copytree(src, os.path.join(tmp, tk))
        elif tk != "tokenizer_3":
            from .sd_single_file import _write_tokenizer
            with open(os.path.join(tmp, need, "config.json")) as f:
                _write_tokenizer(os.path.join(tmp, tk), None, int(json.load(f)["vocab_size"]))
        else:
            raise ValueError(f"{path}: a T5 text encoder needs its tokenizer: set `clip_model` to a "
                             "StableDiffusion3Pipeline directory with tokenizer_3/")
    os.makedirs(os.path.join(tmp, "scheduler"))
    with open(os.path.join(tmp, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "FlowMatchEulerDiscreteScheduler", "num_train_timesteps": 1000,
                   "shift": float(hints.get("shift", 3.0))}, f)
    with open(os.path.join(tmp, "model_index.json"), "w") as f:
        json.dump({"_class_name": "StableDiffusion3Pipeline"}, f)
    with open(os.path.join(tmp, ".source"), "w") as f:
        f.write(stamp)
    shutil.rmtree(out_dir, ignore_errors=True)
    os.replace(tmp, out_dir)
    log.info("converted single-file SD3 checkpoint %s -> %s", path, out_dir)
    return out_dir


def _t5_config(sd: Dict[str, torch.Tensor]) -> dict:
    emb = sd["shared.weight"] if "shared.weight" in sd else sd["encoder.embed_tokens.weight"]
    n = _n_blocks(sd, r"encoder\.block\.(\d+)\.")
    q = sd["encoder.block.0.layer.0.SelfAttention.q.weight"]
    rel = sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
    gated = "encoder.block.0.layer.1.DenseReluDense.wi_0.weight" in sd
    ff = sd["encoder.block.0.layer.1.DenseReluDense." + ("wi_0" if gated else "wi") + ".weight"]
    heads = int(rel.shape[1])
    return dict(vocab_size=int(emb.shape[0]), d_model=int(emb.shape[1]), d_kv=int(q.shape[0]) // heads,
                d_ff=int(ff.shape[0]), num_layers=n, num_heads=heads,
                relative_attention_num_buckets=int(rel.shape[0]), relative_attention_max_distance=128,
                feed_forward_proj="gated-gelu" if gated else "relu", layer_norm_epsilon=1e-6)


def to_single_file(pipe_dir: str, dst: str, with_text: bool = True, with_hints: bool = True) -> str:
    """A StableDiffusion3Pipeline directory -> one Stability-layout .safetensors file (the inverse
    mapping; synthetic checkpoints for the tests)."""
    from safetensors.torch import load_file, save_file

    from .sd import _load_weights
    tcfg = json.load(open(os.path.join(pipe_dir, "transformer", "config.json")))
    vcfg = json.load(open(os.path.join(pipe_dir, "vae", "config.json")))
    out = {UNET_P + k: v for k, v in diffusers_to_mmdit(_load_weights(os.path.join(pipe_dir, "transformer"))).items()}
    for n, t in _load_weights(os.path.join(pipe_dir, "vae")).items():
        if ".attentions." in n and n.endswith(".weight") and t.dim() == 2:
            t = t[:, :, None, None]
        out[VAE_P + vae_name_to_ldm(n, vcfg)] = t
    hints = {"transformer": {k: tcfg[k] for k in ("attention_head_dim", "num_attention_heads", "sample_size",
                                                  "pos_embed_max_size") if k in tcfg},
             "vae": {k: v for k, v in vcfg.items() if k != "_class_name"}}
    if with_text:
        for sub, pre in TE_P.items():
            f = os.path.join(pipe_dir, sub, "model.safetensors")
            if os.path.isfile(f):
                out.update({pre + k: v for k, v in load_file(f).items()})
                hints[sub] = {k: v for k, v in json.load(open(os.path.join(pipe_dir, sub, "config.json"))).items()
                              if not k.startswith("_")}
    meta = {META_KEY: json.dumps(hints)} if with_hints else None
    save_file({k: v.contiguous() for k, v in out.items()}, dst, metadata=meta)
    return dst
