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

kohya files trained against the original LDM / SGM module names (input_blocks.*) are refused with
the count of keys that matched nothing, instead of being half applied.
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
                         f"pipeline weight (first: {missing[0]}); LDM/SGM-named kohya files are not supported")
    return n
