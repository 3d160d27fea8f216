"""LoRA adapters for the diffusion pipelines: the reference's `LoraAdapter` model option
(`backend/python/diffusers/backend.py:300-314`: a path relative to the model file's directory; a
file goes through diffusers' `pipe.load_lora_weights`, a directory through
`unet.load_attn_procs`).

The adapter is merged into the weights at load, in fp32 before the cast to the compute dtype:

    W += scale * (alpha / rank) * up @ down        (alpha absent: scale * up @ down)

for linear weights, and the same product reshaped to the kernel for convolutions (up [out, r, 1, 1],
down [r, in, kh, kw]).  Merged weights cost nothing per step, and the hipGraph-captured UNet step is
unchanged.  Key layouts read (all naming diffusers modules, which is what this pipeline's modules
are called):

  kohya / sd-scripts   lora_unet_<module_path_with_underscores>.lora_down.weight / .lora_up.weight
                       / .alpha, and lora_te_ (lora_te1_ / lora_te2_ for SDXL's two encoders)
  diffusers / PEFT     unet.<module.path>.lora_A.weight / .lora_B.weight (optional .alpha), and
                       text_encoder. / text_encoder_2.; also the `.lora.down.weight` /
                       `.lora.up.weight` spelling
  attention processors <module.path>.processor.to_q_lora.down.weight / .up.weight (a
                       `load_attn_procs` directory: pytorch_lora_weights.safetensors)

kohya files trained against the original LDM / SGM module names (`lora_unet_input_blocks_4_1_...`,
most SD-1.5 / SDXL LoRAs) are mapped onto the diffusers modules from the UNet's own block layout
(`ldm_unet_path`); any key that still matches nothing makes the load fail with the count of such
keys, instead of the adapter being half applied.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn


def _read(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    if os.path.isdir(path):
        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            bins = sorted(glob.glob(os.path.join(path, "*.bin")))
            if not bins:
                raise FileNotFoundError(f"no LoRA weights in {path}")
            return torch.load(bins[0], map_location="cpu", weights_only=True)
        path = next((f for f in files if "lora" in os.path.basename(f)), files[0])
    if path.endswith(".safetensors"):
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def _group(sd: Dict[str, torch.Tensor]) -> Dict[Tuple[str, str], dict]:
    """-> {(target, module key): {"down", "up", "alpha"}}; target in unet / te / te2, module key
    either dotted (diffusers) or underscored (kohya, resolved later)."""
    out: Dict[Tuple[str, str], dict] = {}

    def put(target, mod, part, v):
        out.setdefault((target, mod), {})[part] = v

    for k, v in sd.items():
        m = re.match(r"lora_(unet|te1|te2|te)_(.+?)\.(lora_down\.weight|lora_up\.weight|alpha)$", k)
        if m:
            target = {"unet": "unet", "te": "te", "te1": "te", "te2": "te2"}[m.group(1)]
            part = {"lora_down.weight": "down", "lora_up.weight": "up", "alpha": "alpha"}[m.group(3)]
            put(target, "_" + m.group(2), part, v)     # leading "_": an underscored kohya path
            continue
        m = re.match(r"(unet|text_encoder_2|text_encoder)\.(.+?)\.(lora_A\.weight|lora_B\.weight|"
                     r"lora\.down\.weight|lora\.up\.weight|alpha)$", k)
        if m:
            target = {"unet": "unet", "text_encoder": "te", "text_encoder_2": "te2"}[m.group(1)]
            part = {"lora_A.weight": "down", "lora.down.weight": "down", "lora_B.weight": "up",
                    "lora.up.weight": "up", "alpha": "alpha"}[m.group(3)]
            put(target, m.group(2), part, v)
            continue
        m = re.match(r"(?:unet\.)?(.+)\.processor\.(to_q|to_k|to_v|to_out)_lora\.(down|up)\.weight$", k)
        if m:
            mod = m.group(1) + "." + (m.group(2) if m.group(2) != "to_out" else "to_out.0")
            put("unet", mod, m.group(3), v)
            continue
        raise ValueError(f"unrecognised LoRA key {k!r}")
    return out


def _params(mod: Optional[nn.Module]) -> Tuple[Dict[str, nn.Parameter], Dict[str, str]]:
    if mod is None:
        return {}, {}
    ps = {n[:-len(".weight")]: p for n, p in mod.named_parameters() if n.endswith(".weight")}
    under = {n.replace(".", "_"): n for n in ps}
    return ps, under


_RES_TAIL = {"in_layers_0": "norm1", "in_layers_2": "conv1", "emb_layers_1": "time_emb_proj",
             "out_layers_0": "norm2", "out_layers_3": "conv2", "skip_connection": "conv_shortcut"}
_TOP = {"time_embed_0": "time_embedding.linear_1", "time_embed_2": "time_embedding.linear_2",
        "label_emb_0_0": "add_embedding.linear_1", "label_emb_0_2": "add_embedding.linear_2",
        "out_0": "conv_norm_out", "out_2": "conv_out", "input_blocks_0_0": "conv_in"}


def ldm_unet_path(key: str, unet: nn.Module) -> Optional[str]:
    """A kohya key body in the original LDM / SGM UNet naming (input_blocks_N_S_..., middle_block_S_...,
    output_blocks_N_S_...) -> the underscored diffusers path of the same module, from the UNet's
    own block layout (layers per block, which blocks carry attentions / up-samplers), as diffusers'
    single-file conversion lays the blocks out."""
    if key in _TOP:
        return _TOP[key].replace(".", "_")
    lpb = len(unet.down_blocks[0].resnets)

    def res(prefix, tail):
        for k, v in _RES_TAIL.items():
            if tail == k or tail.startswith(k + "_"):
                return prefix + "_" + v + tail[len(k):]
        return None

    m = re.match(r"input_blocks_(\d+)_(\d+)_(.+)$", key)
    if m:
        n, sub, tail = int(m.group(1)), int(m.group(2)), m.group(3)
        i, j = (n - 1) // (lpb + 1), (n - 1) % (lpb + 1)
        if n == 0 or i >= len(unet.down_blocks):
            return None
        if j == lpb:
            return f"down_blocks_{i}_downsamplers_0_conv" if tail == "op" else None
        if sub == 0:
            return res(f"down_blocks_{i}_resnets_{j}", tail)
        return f"down_blocks_{i}_attentions_{j}_{tail}" if sub == 1 else None
    m = re.match(r"middle_block_(\d+)_(.+)$", key)
    if m:
        sub, tail = int(m.group(1)), m.group(2)
        if sub == 1:
            return f"mid_block_attentions_0_{tail}"
        return res(f"mid_block_resnets_{sub // 2}", tail) if sub in (0, 2) else None
    m = re.match(r"output_blocks_(\d+)_(\d+)_(.+)$", key)
    if m:
        n, sub, tail = int(m.group(1)), int(m.group(2)), m.group(3)
        i, j = n // (lpb + 1), n % (lpb + 1)
        if i >= len(unet.up_blocks):
            return None
        blk = unet.up_blocks[i]
        if sub == 0:
            return res(f"up_blocks_{i}_resnets_{j}", tail)
        if sub == 1 and hasattr(blk, "attentions"):
            return f"up_blocks_{i}_attentions_{j}_{tail}"
        if tail == "conv" and hasattr(blk, "upsamplers"):
            return f"up_blocks_{i}_upsamplers_0_conv"
    return None


def merge_sd_lora(path: str, unet: nn.Module, text: Optional[nn.Module] = None,
                  text2: Optional[nn.Module] = None, scale: float = 1.0) -> int:
    """Merge the LoRA at `path` into the modules (fp32 in place); returns the number of weights
    updated.  Raises when any adapter entry matches no weight of the pipeline."""
    groups = _group(_read(path))
    targets = {"unet": _params(unet), "te": _params(text), "te2": _params(text2)}
    missing: List[str] = []
    n = 0
    with torch.no_grad():
        for (target, mod), e in groups.items():
            if "down" not in e or "up" not in e:
                missing.append(f"{target}:{mod} (incomplete)")
                continue
            ps, under = targets[target]
            name = under.get(mod[1:]) if mod.startswith("_") else mod
            if name is None and mod.startswith("_") and target == "unet":
                alt = ldm_unet_path(mod[1:], unet)
                name = under.get(alt) if alt else None
            if name not in ps and target != "unet":
                # text encoders: checkpoints with and without the `text_model.` prefix
                alt = ("text_model." + name) if name and not name.startswith("text_model.") else None
                name = alt if alt in ps else name
            p = ps.get(name) if name else None
            if p is None:
                missing.append(f"{target}:{mod}")
                continue
            down, up = e["down"].float(), e["up"].float()
            rank = down.shape[0]
            a = float(e["alpha"]) / rank if "alpha" in e else 1.0
            delta = (up.reshape(up.shape[0], -1) @ down.reshape(rank, -1)).reshape(p.shape)
            p.add_((scale * a * delta).to(p.device, p.dtype))
            n += 1
    if missing:
        raise ValueError(f"LoRA {os.path.basename(path)}: {len(missing)} of {len(groups)} entries match no "
                         f"pipeline weight (first: {missing[0]})")
    return n
