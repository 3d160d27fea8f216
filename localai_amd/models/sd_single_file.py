"""Single-file Stable Diffusion checkpoints (the original LDM / SGM layout: one `.safetensors` or
`.ckpt` holding `model.diffusion_model.*`, `first_stage_model.*` and the text encoder(s)) -> a
diffusers-layout pipeline directory that `models/sd.py` loads.

The reference calls `StableDiffusionPipeline.from_single_file` / `StableDiffusionXLPipeline.
from_single_file` whenever the model is a local file or a URL (backend/python/diffusers/
backend.py:184-191, 214-216, 228-231), which is how its AIO image model
(`aio/gpu-8g/image-gen.yaml`: DreamShaper_8_pruned.safetensors) and `gallery/dreamshaper.yaml`
load.  Here the file is converted ONCE into a hidden sibling directory
(`.<file>.diffusers/`, keyed by the file's size and mtime) and served from there:

  * SD 1.x: CLIP-L stored in transformers layout under `cond_stage_model.transformer.`;
  * SD 2.x: OpenCLIP-H under `cond_stage_model.model.` (fused in_proj, `resblocks`); the
    penultimate layer is the output, so the last block is dropped (diffusers' SD2 configs say
    num_hidden_layers 23);
  * SDXL: CLIP-L under `conditioner.embedders.0.transformer.` and OpenCLIP-bigG with its text
    projection under `conditioner.embedders.1.model.`, `label_emb` -> `add_embedding`.

Configs come from the tensor shapes (levels, layers per block, attention levels, transformer
depth, channels, context width, projection width); the head count -- which weights do not carry
-- follows the published families (cross width 768: 8 heads per level; otherwise 64-wide heads).
A file may carry exact configs in its safetensors metadata (`localai_amd.configs`, written by
`synth.write_sd_single_file`).  The CLIP tokenizer comes from `tokenizer_dir` (the model
config's `clip_model`, a directory), a `tokenizer/` next to the file, $LOCALAI_AMD_CLIP_TOKENIZER,
or -- when the checkpoint's vocabulary is the byte-level one `synth` writes -- that vocabulary.
"""
from __future__ import annotations

import json
import logging
import os
import re
import shutil
from typing import Dict, Optional, Tuple

import torch

log = logging.getLogger(__name__)

SINGLE_FILE_EXT = (".safetensors", ".ckpt", ".pt", ".pth", ".bin")
UNET_P = "model.diffusion_model."
VAE_P = "first_stage_model."
SD1_TE = "cond_stage_model.transformer."
SD2_TE = "cond_stage_model.model."
XL_TE1 = "conditioner.embedders.0.transformer."
XL_TE2 = "conditioner.embedders.1.model."
META_KEY = "localai_amd.configs"


def is_single_file(path: str) -> bool:
    return os.path.isfile(path) and path.lower().endswith(SINGLE_FILE_EXT)


def load_checkpoint(path: str) -> Tuple[Dict[str, torch.Tensor], dict]:
    """(state dict, config hints).  Pickled checkpoints load with weights_only=True (nothing in
    the file is executed); Lightning's {"state_dict": ...} wrapper is unwrapped."""
    hints = {}
    if path.lower().endswith(".safetensors"):
        from safetensors import safe_open
        sd = {}
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            for k in f.keys():
                sd[k] = f.get_tensor(k)
        if META_KEY in meta:
            hints = json.loads(meta[META_KEY])
        return sd, hints
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict) and isinstance(obj.get("state_dict"), dict):
        obj = obj["state_dict"]
    if not isinstance(obj, dict):
        raise ValueError(f"{path}: not a state dict")
    return {k: v for k, v in obj.items() if torch.is_tensor(v)}, hints


def family(sd) -> str:
    if any(k.startswith(XL_TE2) for k in sd):
        return "sdxl"
    if any(k.startswith(SD2_TE) for k in sd):
        return "sd2"
    if any(k.startswith(SD1_TE) for k in sd):
        return "sd1"
    if any(k.startswith(UNET_P) for k in sd):
        raise ValueError("single-file checkpoint without a recognised text encoder (SD 1.x / 2.x / XL expected)")
    raise ValueError("not a Stable Diffusion single-file checkpoint (no model.diffusion_model.* tensors)")


# --------------------------------------------------------------------------- UNet names
_RES = {"norm1": "in_layers.0", "conv1": "in_layers.2", "time_emb_proj": "emb_layers.1", "norm2": "out_layers.0",
        "conv2": "out_layers.3", "conv_shortcut": "skip_connection"}


def _res(rest: str) -> str:
    head, _, tail = rest.partition(".")
    return _RES[head] + "." + tail


def unet_name_to_ldm(k: str, cfg: dict) -> str:
    """diffusers UNet2DConditionModel parameter name -> LDM openaimodel.UNetModel name."""
    lpb = int(cfg.get("layers_per_block", 2))
    ups = cfg["up_block_types"]
    simple = {"conv_in.": "input_blocks.0.0.", "time_embedding.linear_1.": "time_embed.0.",
              "time_embedding.linear_2.": "time_embed.2.", "add_embedding.linear_1.": "label_emb.0.0.",
              "add_embedding.linear_2.": "label_emb.0.2.", "conv_norm_out.": "out.0.", "conv_out.": "out.2."}
    for a, b in simple.items():
        if k.startswith(a):
            return b + k[len(a):]
    m = re.match(r"down_blocks\.(\d+)\.(resnets|attentions|downsamplers)\.(\d+)\.(.*)", k)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "downsamplers":
            return f"input_blocks.{1 + i * (lpb + 1) + lpb}.0.op.{rest.split('.', 1)[1]}"
        idx = 1 + i * (lpb + 1) + j
        return f"input_blocks.{idx}.0.{_res(rest)}" if kind == "resnets" else f"input_blocks.{idx}.1.{rest}"
    m = re.match(r"mid_block\.(resnets|attentions)\.(\d+)\.(.*)", k)
    if m:
        if m[1] == "attentions":
            return f"middle_block.1.{m[3]}"
        return f"middle_block.{2 * int(m[2])}.{_res(m[3])}"
    m = re.match(r"up_blocks\.(\d+)\.(resnets|attentions|upsamplers)\.(\d+)\.(.*)", k)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "upsamplers":
            at = 2 if "CrossAttn" in ups[i] else 1
            return f"output_blocks.{i * (lpb + 1) + lpb}.{at}.{rest}"
        idx = i * (lpb + 1) + j
        return f"output_blocks.{idx}.0.{_res(rest)}" if kind == "resnets" else f"output_blocks.{idx}.1.{rest}"
    raise KeyError(k)


def infer_unet_config(sd: Dict[str, torch.Tensor], fam: str) -> dict:
    """UNet2DConditionModel config from LDM UNet tensor shapes (keys without the prefix)."""
    keys = set(sd)
    n_in = 1 + max(int(k.split(".")[1]) for k in keys if k.startswith("input_blocks."))
    downs = sorted({int(k.split(".")[1]) for k in keys if re.match(r"input_blocks\.\d+\.0\.op\.", k)})
    L = len(downs) + 1
    lpb = (n_in - L) // L
    ch, attn, depth, heads = [], [], [], []
    cross = None
    lin = False
    for i in range(L):
        idx = 1 + i * (lpb + 1)
        ch.append(int(sd[f"input_blocks.{idx}.0.out_layers.3.weight"].shape[0]))
        a = f"input_blocks.{idx}.1.proj_in.weight" in keys
        attn.append(a)
        if a:
            depth.append(1 + max(int(k.split(".")[4]) for k in keys
                                 if k.startswith(f"input_blocks.{idx}.1.transformer_blocks.")))
            cross = int(sd[f"input_blocks.{idx}.1.transformer_blocks.0.attn2.to_k.weight"].shape[1])
            lin = sd[f"input_blocks.{idx}.1.proj_in.weight"].dim() == 2
        else:
            depth.append(1)
    if cross is None:
        cross = int(sd["middle_block.1.transformer_blocks.0.attn2.to_k.weight"].shape[1])
        lin = sd["middle_block.1.proj_in.weight"].dim() == 2
    mid_depth = 1 + max(int(k.split(".")[3]) for k in keys if k.startswith("middle_block.1.transformer_blocks."))
    if fam == "sd1" or cross == 768:
        heads = [8] * L
    else:
        heads = [max(1, c // 64) for c in ch]
    cfg = dict(block_out_channels=ch, layers_per_block=lpb, cross_attention_dim=cross,
               attention_head_dim=heads if len(set(heads)) > 1 else heads[0], norm_num_groups=32,
               in_channels=int(sd["input_blocks.0.0.weight"].shape[1]), out_channels=int(sd["out.2.weight"].shape[0]),
               sample_size=128 if fam == "sdxl" else (96 if fam == "sd2" else 64),
               down_block_types=["CrossAttnDownBlock2D" if a else "DownBlock2D" for a in attn],
               up_block_types=["CrossAttnUpBlock2D" if a else "UpBlock2D" for a in attn[::-1]],
               use_linear_projection=lin, flip_sin_to_cos=True, freq_shift=0)
    if any(d > 1 for d in depth) or mid_depth > 1:
        d = [depth[i] if attn[i] else 1 for i in range(L)]
        if not attn[-1]:
            d[-1] = mid_depth
        cfg["transformer_layers_per_block"] = d
    if "label_emb.0.0.weight" in keys:
        cfg.update(addition_embed_type="text_time", addition_time_embed_dim=256,
                   projection_class_embeddings_input_dim=int(sd["label_emb.0.0.weight"].shape[1]))
    return cfg


# --------------------------------------------------------------------------- VAE names
def vae_name_to_ldm(k: str, cfg: dict) -> str:
    """diffusers AutoencoderKL name -> LDM autoencoder name (attention as diffusers' to_q/...)."""
    L = len(cfg["block_out_channels"])
    for a, b in (("encoder.conv_norm_out.", "encoder.norm_out."), ("decoder.conv_norm_out.", "decoder.norm_out.")):
        if k.startswith(a):
            return b + k[len(a):]
    m = re.match(r"(encoder|decoder)\.mid_block\.(resnets|attentions)\.(\d+)\.(.*)", k)
    if m:
        side, kind, j, rest = m[1], m[2], int(m[3]), m[4]
        if kind == "resnets":
            return f"{side}.mid.block_{j + 1}.{rest.replace('conv_shortcut', 'nin_shortcut')}"
        head, _, tail = rest.partition(".")
        if head == "to_out":
            head, tail = "proj_out", tail.split(".", 1)[1]
        head = {"group_norm": "norm", "to_q": "q", "to_k": "k", "to_v": "v"}.get(head, head)
        return f"{side}.mid.attn_1.{head}.{tail}"
    m = re.match(r"encoder\.down_blocks\.(\d+)\.(resnets|downsamplers)\.(\d+)\.(.*)", k)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "downsamplers":
            return f"encoder.down.{i}.downsample.{rest}"
        return f"encoder.down.{i}.block.{j}.{rest.replace('conv_shortcut', 'nin_shortcut')}"
    m = re.match(r"decoder\.up_blocks\.(\d+)\.(resnets|upsamplers)\.(\d+)\.(.*)", k)
    if m:
        i, kind, j, rest = int(m[1]), m[2], int(m[3]), m[4]
        if kind == "upsamplers":
            return f"decoder.up.{L - 1 - i}.upsample.{rest}"
        return f"decoder.up.{L - 1 - i}.block.{j}.{rest.replace('conv_shortcut', 'nin_shortcut')}"
    return k  # conv_in / conv_out / quant_conv / post_quant_conv


def infer_vae_config(sd: Dict[str, torch.Tensor], fam: str) -> dict:
    keys = set(sd)
    L = 1 + max(int(k.split(".")[2]) for k in keys if k.startswith("encoder.down."))
    lpb = 1 + max(int(k.split(".")[4]) for k in keys if k.startswith("encoder.down.0.block."))
    ch = [int(sd[f"encoder.down.{i}.block.0.conv2.weight"].shape[0]) for i in range(L)]
    return dict(block_out_channels=ch, layers_per_block=lpb, latent_channels=int(sd["quant_conv.weight"].shape[0]) // 2,
                norm_num_groups=32, in_channels=int(sd["encoder.conv_in.weight"].shape[1]),
                out_channels=int(sd["decoder.conv_out.weight"].shape[0]),
                scaling_factor=0.13025 if fam == "sdxl" else 0.18215)


# --------------------------------------------------------------------------- text encoders
def openclip_to_hf(sd: Dict[str, torch.Tensor], drop_last: bool, n_layers: Optional[int] = None
                   ) -> Dict[str, torch.Tensor]:
    """OpenCLIP text tower (keys without the prefix) -> transformers CLIPTextModel(WithProjection);
    drop_last: the penultimate layer is the output (SD 2.x); n_layers overrides both."""
    n = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("transformer.resblocks."))
    if drop_last:
        n -= 1
    if n_layers is not None:
        n = int(n_layers)
    out = {"text_model.embeddings.token_embedding.weight": sd["token_embedding.weight"],
           "text_model.embeddings.position_embedding.weight": sd["positional_embedding"],
           "text_model.final_layer_norm.weight": sd["ln_final.weight"],
           "text_model.final_layer_norm.bias": sd["ln_final.bias"]}
    for i in range(n):
        s, d = f"transformer.resblocks.{i}.", f"text_model.encoder.layers.{i}."
        for a, b in (("ln_1", "layer_norm1"), ("ln_2", "layer_norm2"), ("attn.out_proj", "self_attn.out_proj"),
                     ("mlp.c_fc", "mlp.fc1"), ("mlp.c_proj", "mlp.fc2")):
            for t in ("weight", "bias"):
                out[f"{d}{b}.{t}"] = sd[f"{s}{a}.{t}"]
        for t in ("weight", "bias"):
            q, k, v = sd[f"{s}attn.in_proj_{t}"].chunk(3, 0)
            out[f"{d}self_attn.q_proj.{t}"], out[f"{d}self_attn.k_proj.{t}"], out[f"{d}self_attn.v_proj.{t}"] = q, k, v
    if "text_projection" in sd:
        out["text_projection.weight"] = sd["text_projection"].t().contiguous()
    return out


def hf_to_openclip(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Inverse of openclip_to_hf (no dropped layer): synthetic single files and tests."""
    n = 1 + max(int(k.split(".")[3]) for k in sd if k.startswith("text_model.encoder.layers."))
    out = {"token_embedding.weight": sd["text_model.embeddings.token_embedding.weight"],
           "positional_embedding": sd["text_model.embeddings.position_embedding.weight"],
           "ln_final.weight": sd["text_model.final_layer_norm.weight"],
           "ln_final.bias": sd["text_model.final_layer_norm.bias"]}
    for i in range(n):
        s, d = f"text_model.encoder.layers.{i}.", f"transformer.resblocks.{i}."
        for a, b in (("layer_norm1", "ln_1"), ("layer_norm2", "ln_2"), ("self_attn.out_proj", "attn.out_proj"),
                     ("mlp.fc1", "mlp.c_fc"), ("mlp.fc2", "mlp.c_proj")):
            for t in ("weight", "bias"):
                out[f"{d}{b}.{t}"] = sd[f"{s}{a}.{t}"]
        for t in ("weight", "bias"):
            out[f"{d}attn.in_proj_{t}"] = torch.cat([sd[f"{s}self_attn.{p}_proj.{t}"] for p in "qkv"], 0)
    if "text_projection.weight" in sd:
        out["text_projection"] = sd["text_projection.weight"].t().contiguous()
    return out


def _hf_clip_keys(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    # very old checkpoints predate transformers' `text_model.` level (transformers 5 drops it again)
    return {(k if k.startswith(("text_model.", "text_projection")) else "text_model." + k): v for k, v in sd.items()
            if "position_ids" not in k}


def infer_text_config(sd: Dict[str, torch.Tensor], act: str, vocab: Optional[dict]) -> dict:
    tok = sd["text_model.embeddings.token_embedding.weight"]
    D = int(tok.shape[1])
    n = 1 + max(int(k.split(".")[3]) for k in sd if k.startswith("text_model.encoder.layers."))
    c = dict(hidden_size=D, num_hidden_layers=n, num_attention_heads=12 if D == 768 else max(1, D // 64),
             intermediate_size=int(sd["text_model.encoder.layers.0.mlp.fc1.weight"].shape[0]),
             vocab_size=int(tok.shape[0]),
             max_position_embeddings=int(sd["text_model.embeddings.position_embedding.weight"].shape[0]),
             hidden_act=act, layer_norm_eps=1e-5, bos_token_id=49406, eos_token_id=49407, pad_token_id=49407)
    if vocab and int(tok.shape[0]) == len(vocab):
        c.update(bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
                 pad_token_id=vocab["<|endoftext|>"])
    if "text_projection.weight" in sd:
        c["projection_dim"] = int(sd["text_projection.weight"].shape[0])
    return c


# --------------------------------------------------------------------------- conversion
def _find_tokenizer(path: str, tokenizer_dir: Optional[str]) -> Optional[str]:
    cands = []
    if tokenizer_dir:
        cands += [os.path.join(tokenizer_dir, "tokenizer"), tokenizer_dir]
    cands += [os.path.join(os.path.dirname(os.path.abspath(path)), "tokenizer"),
              os.environ.get("LOCALAI_AMD_CLIP_TOKENIZER", "")]
    for c in cands:
        if c and os.path.isfile(os.path.join(c, "vocab.json")) and os.path.isfile(os.path.join(c, "merges.txt")):
            return c
    return None


def _write_tokenizer(dst: str, src: Optional[str], vocab_size: int):
    os.makedirs(dst, exist_ok=True)
    if src:
        for n in os.listdir(src):
            p = os.path.join(src, n)
            if os.path.isfile(p):
                shutil.copy(p, os.path.join(dst, n))
        return
    from .synth import _clip_byte_vocab
    vocab = _clip_byte_vocab()
    if vocab_size != len(vocab):
        raise ValueError(f"single-file checkpoint with a {vocab_size}-entry CLIP vocabulary needs its tokenizer: "
                         "set the model's `clip_model` to a directory holding vocab.json + merges.txt "
                         "(or a tokenizer/ directory next to the file, or LOCALAI_AMD_CLIP_TOKENIZER)")
    with open(os.path.join(dst, "vocab.json"), "w") as f:
        json.dump(vocab, f)
    with open(os.path.join(dst, "merges.txt"), "w") as f:
        f.write("#version: 0.2\n")


def _save(d: str, name: str, cfg: dict, sd: Dict[str, torch.Tensor], file: str):
    from safetensors.torch import save_file
    os.makedirs(os.path.join(d, name), exist_ok=True)
    with open(os.path.join(d, name, "config.json"), "w") as f:
        json.dump(cfg, f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(d, name, file))


def _expected_names(cls, cfg: dict):
    with torch.device("meta"):
        return list(cls(cfg).state_dict().keys())


def convert(path: str, out_dir: Optional[str] = None, tokenizer_dir: Optional[str] = None) -> str:
    """Convert (once) and return the diffusers-layout directory of a single-file checkpoint."""
    from . import sd as sdm
    st = os.stat(path)
    stamp = f"{st.st_size}:{int(st.st_mtime)}"
    if out_dir is None:
        out_dir = os.path.join(os.path.dirname(os.path.abspath(path)), "." + os.path.basename(path) + ".diffusers")
    mark = os.path.join(out_dir, ".source")
    if os.path.isfile(mark) and open(mark).read() == stamp:
        return out_dir
    sd, hints = load_checkpoint(path)
    from . import sd3_single_file as sd3f
    if hints.get("family") == "sd3" or sd3f.is_sd3_file(sd):
        # backend.py:238-242: StableDiffusion3Pipeline.from_single_file
        return sd3f.convert(path, sd, hints, out_dir, tokenizer_dir)
    fam = hints.get("family") or family(sd)
    tmp = out_dir + ".partial"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    # UNet
    u = {k[len(UNET_P):]: v for k, v in sd.items() if k.startswith(UNET_P)}
    ucfg = hints.get("unet") or infer_unet_config(u, fam)
    names = _expected_names(sdm.UNet, ucfg)
    missing = [n for n in names if unet_name_to_ldm(n, ucfg) not in u]
    if missing:
        raise ValueError(f"single-file UNet lacks {len(missing)} tensors, e.g. {unet_name_to_ldm(missing[0], ucfg)}")
    _save(tmp, "unet", dict(ucfg, _class_name="UNet2DConditionModel"),
          {n: u[unet_name_to_ldm(n, ucfg)] for n in names}, "diffusion_pytorch_model.safetensors")
    # VAE (encoder half included when present: img2img)
    v = {k[len(VAE_P):]: t for k, t in sd.items() if k.startswith(VAE_P)}
    vcfg = hints.get("vae") or infer_vae_config(v, fam)
    vsd = {}
    for cls in (sdm.VaeDecoder, sdm.VaeEncoder):
        for n in _expected_names(cls, vcfg):
            t = v.get(vae_name_to_ldm(n, vcfg))
            if t is None:
                if cls is sdm.VaeEncoder:
                    vsd = {k_: t_ for k_, t_ in vsd.items() if not k_.startswith(("encoder.", "quant_conv."))}
                    break
                raise ValueError(f"single-file VAE lacks {vae_name_to_ldm(n, vcfg)}")
            if ".attentions." in n and n.endswith(".weight") and t.dim() == 4:
                t = t[:, :, 0, 0]
            vsd[n] = t
    _save(tmp, "vae", dict(vcfg, _class_name="AutoencoderKL"), vsd, "diffusion_pytorch_model.safetensors")
    # text encoder(s) + tokenizer(s)
    tok_src = _find_tokenizer(path, tokenizer_dir)
    from .synth import _clip_byte_vocab
    vocab = None if tok_src else _clip_byte_vocab()
    if fam == "sd2":
        hint = hints.get("text_encoder")
        te1 = openclip_to_hf({k[len(SD2_TE):]: t for k, t in sd.items() if k.startswith(SD2_TE)}, drop_last=True,
                             n_layers=hint["num_hidden_layers"] if hint else None)
        if not (hint and "projection_dim" in hint):
            te1.pop("text_projection.weight", None)  # CLIPTextModel: the SD 2.x tower's projection is unused
        act1 = "gelu"
    else:
        te1 = _hf_clip_keys({k[len(SD1_TE if fam == "sd1" else XL_TE1):]: t for k, t in sd.items()
                             if k.startswith(SD1_TE if fam == "sd1" else XL_TE1)})
        act1 = "quick_gelu"
    tc1 = hints.get("text_encoder") or infer_text_config(te1, act1, vocab)
    _save(tmp, "text_encoder", dict(tc1, architectures=["CLIPTextModel"], model_type="clip_text_model"), te1,
          "model.safetensors")
    _write_tokenizer(os.path.join(tmp, "tokenizer"), tok_src, int(tc1["vocab_size"]))
    index = {"_class_name": "StableDiffusionPipeline"}
    if fam == "sdxl":
        te2 = openclip_to_hf({k[len(XL_TE2):]: t for k, t in sd.items() if k.startswith(XL_TE2)}, drop_last=False)
        tc2 = hints.get("text_encoder_2") or infer_text_config(te2, "gelu", vocab)
        _save(tmp, "text_encoder_2", dict(tc2, architectures=["CLIPTextModelWithProjection"],
                                          model_type="clip_text_model"), te2, "model.safetensors")
        _write_tokenizer(os.path.join(tmp, "tokenizer_2"), tok_src, int(tc2["vocab_size"]))
        index = {"_class_name": "StableDiffusionXLPipeline", "force_zeros_for_empty_prompt": True}
    pred = hints.get("prediction_type") or ("v_prediction" if fam == "sd2" else "epsilon")
    os.makedirs(os.path.join(tmp, "scheduler"))
    with open(os.path.join(tmp, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "DDIMScheduler", "beta_start": 0.00085, "beta_end": 0.012,
                   "beta_schedule": "scaled_linear", "num_train_timesteps": 1000, "steps_offset": 1,
                   "set_alpha_to_one": False, "clip_sample": False, "prediction_type": pred}, f)
    with open(os.path.join(tmp, "model_index.json"), "w") as f:
        json.dump(index, f)
    with open(os.path.join(tmp, ".source"), "w") as f:
        f.write(stamp)
    shutil.rmtree(out_dir, ignore_errors=True)
    os.replace(tmp, out_dir)
    log.info("converted single-file %s checkpoint %s -> %s", fam, path, out_dir)
    return out_dir


def to_single_file(pipe_dir: str, dst: str, fam: str, with_hints: bool = True) -> str:
    """A diffusers-layout SD pipeline directory -> one LDM / SGM-layout .safetensors file (the
    inverse mapping; synthetic checkpoints for tests and benchmarks)."""
    from safetensors.torch import load_file, save_file

    from .sd import _load_weights
    ucfg = json.load(open(os.path.join(pipe_dir, "unet", "config.json")))
    vcfg = json.load(open(os.path.join(pipe_dir, "vae", "config.json")))
    out = {}
    for n, t in _load_weights(os.path.join(pipe_dir, "unet")).items():
        out[UNET_P + unet_name_to_ldm(n, ucfg)] = t
    for n, t in _load_weights(os.path.join(pipe_dir, "vae")).items():
        if ".attentions." in n and n.endswith(".weight") and t.dim() == 2:
            t = t[:, :, None, None]
        out[VAE_P + vae_name_to_ldm(n, vcfg)] = t
    te1 = _hf_clip_keys(load_file(os.path.join(pipe_dir, "text_encoder", "model.safetensors")))
    hints = {"family": fam, "unet": ucfg, "vae": vcfg}
    hints["text_encoder"] = json.load(open(os.path.join(pipe_dir, "text_encoder", "config.json")))
    if fam == "sd2":
        out.update({SD2_TE + k: v for k, v in hf_to_openclip(te1).items()})
    else:
        out.update({(SD1_TE if fam == "sd1" else XL_TE1) + k: v for k, v in te1.items()})
    if fam == "sdxl":
        te2 = _hf_clip_keys(load_file(os.path.join(pipe_dir, "text_encoder_2", "model.safetensors")))
        out.update({XL_TE2 + k: v for k, v in hf_to_openclip(te2).items()})
        hints["text_encoder_2"] = json.load(open(os.path.join(pipe_dir, "text_encoder_2", "config.json")))
    sc = os.path.join(pipe_dir, "scheduler", "scheduler_config.json")
    if os.path.isfile(sc):
        hints["prediction_type"] = json.load(open(sc)).get("prediction_type", "epsilon")
    meta = {META_KEY: json.dumps(hints)} if with_hints else None
    save_file({k: v.contiguous() for k, v in out.items()}, dst, metadata=meta)
    return dst
