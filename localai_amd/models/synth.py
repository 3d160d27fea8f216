"""Random-init GGUF models of the BASELINE architectures (no network: no real checkpoints).

Presets reproduce the public hyper-parameters and llama.cpp's Q4_K_M tensor-type mix
(`use_more_bits` layers get Q6_K for attn_v / ffn_down, output is Q6_K), so the engine
streams exactly the bytes a real Llama-3-8B-Instruct-Q4_K_M.gguf would make it stream.
Quantised tensors are written as random *valid* blocks (fast: O(bytes)); small test
models can instead quantise real float weights for exact reference checks.

The tokenizer is a byte-level BPE trained offline on Python sources (assets/bpe32k.json.gz),
padded to the preset vocabulary with unreachable filler tokens plus the preset's special
tokens (Llama-3's <|begin_of_text|> ... <|eot_id|> at 128000+).
"""
from __future__ import annotations

import gzip
import math
import json
import os
from dataclasses import dataclass, field, replace
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np

from ..gguf import (GGMLType, GGUFValueType, GGUFWriter, quantize, random_q4_k_blocks, random_q5_k_blocks,
                    random_q6_k_blocks, random_q8_0_blocks)

ASSETS = Path(__file__).resolve().parent.parent / "assets"

LLAMA3_TEMPLATE = ("{% set loop_messages = messages %}{% for message in loop_messages %}{% set content = "
                   "'<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n'+ message['content'] | trim + "
                   "'<|eot_id|>' %}{% if loop.index0 == 0 %}{% set content = bos_token + content %}{% endif %}"
                   "{{ content }}{% endfor %}{% if add_generation_prompt %}{{ '<|start_header_id|>assistant"
                   "<|end_header_id|>\n\n' }}{% endif %}")


@dataclass
class Preset:
    arch: str = "llama"
    n_layer: int = 32
    n_embd: int = 4096
    n_head: int = 32
    n_head_kv: int = 8
    n_ff: int = 14336
    n_vocab: int = 128256
    ctx: int = 8192
    rope_theta: float = 500000.0
    eps: float = 1e-5
    n_expert: int = 0
    n_expert_used: int = 0
    rope_dim: Optional[int] = None
    head_dim: Optional[int] = None   # default n_embd // n_head (Gemma: 256 with q_dim != n_embd)
    qtype: str = "Q4_K_M"            # Q4_K_M | Q5_K_M | Q4_K | Q8_0 | F16 | F32
    tokenizer: str = "llama3"        # llama3 | mistral | phi2 | chatml
    tied: bool = False               # no output.weight: the lm_head is token_embd (Gemma, small Qwen2)
    attn_softcap: float = 0.0        # Gemma-2 keys
    final_softcap: float = 0.0
    sliding_window: int = 0
    logit_scale: float = 0.0         # Command-R
    n_ff_shexp: int = 0              # Qwen2-MoE shared expert width
    kv_lora_rank: int = 0            # DeepSeek-V2 latent attention (head_dim = key width, rope_dim = rotary part)
    head_dim_v: int = 0
    n_ff_exp: int = 0
    n_expert_shared: int = 0
    n_layer_dense_lead: int = 0
    yarn_factor: float = 0.0
    name: str = "synthetic"

    @property
    def hd(self) -> int:
        return self.head_dim or self.n_embd // self.n_head


PRESETS: Dict[str, Preset] = {
    "llama3-8b": Preset(name="Meta-Llama-3-8B-Instruct (random-init)"),
    "llama3-8b-q8_0": Preset(qtype="Q8_0", name="Meta-Llama-3-8B-Instruct Q8_0 (random-init)"),
    "llama3-8b-q5_k_m": Preset(qtype="Q5_K_M", name="Meta-Llama-3-8B-Instruct Q5_K_M (random-init)"),
    # the Llama-3-8B layer shapes (4096 wide, GQA 32/8, 14336 FFN, Q4_K_M mixed Q4_K/Q6_K, 128256 vocab)
    # on 2 layers: the headline decode path at a size the fp32 oracle can check (tests/test_engine_gpu.py)
    "llama3-8b-2l": Preset(n_layer=2, ctx=1024, name="Llama-3-8B shapes, 2 layers (random-init)"),
    "llama3-70b": Preset(n_layer=80, n_embd=8192, n_head=64, n_head_kv=8, n_ff=28672,
                         name="Meta-Llama-3-70B-Instruct (random-init)"),
    "mixtral-8x7b": Preset(n_layer=32, n_embd=4096, n_head=32, n_head_kv=8, n_ff=14336, n_vocab=32000,
                           ctx=32768, rope_theta=1e6, n_expert=8, n_expert_used=2, tokenizer="mistral",
                           name="Mixtral-8x7B-Instruct-v0.1 (random-init)"),
    "mistral-7b": Preset(n_vocab=32000, ctx=32768, rope_theta=1e6, tokenizer="mistral",
                         name="Mistral-7B-Instruct (random-init)"),
    "phi2": Preset(arch="phi2", n_layer=32, n_embd=2560, n_head=32, n_head_kv=32, n_ff=10240, n_vocab=51200,
                   ctx=2048, rope_theta=10000.0, rope_dim=32, tokenizer="phi2", name="phi-2 (random-init)"),
    # small shapes for tests (CPU reference runs) -- K dims multiples of 256 so every kernel path is used
    "tiny-llama": Preset(n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32256, ctx=512,
                         qtype="Q4_K", name="tiny-llama"),
    "tiny-llama-q5km": Preset(n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32256, ctx=512,
                              qtype="Q5_K_M", name="tiny-llama-q5km"),
    "tiny-llama-q8": Preset(n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32256, ctx=512,
                            qtype="Q8_0", name="tiny-llama-q8"),
    "tiny-mixtral": Preset(n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32256, ctx=512,
                           n_expert=4, n_expert_used=2, qtype="Q4_K", name="tiny-mixtral"),
    # Mixtral's 32000-entry SentencePiece-style vocabulary on the tiny MoE shapes
    "tiny-mixtral-spm": Preset(n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32000, ctx=512,
                               n_expert=4, n_expert_used=2, qtype="Q4_K", tokenizer="mistral",
                               name="tiny-mixtral-spm"),
    "tiny-phi2": Preset(arch="phi2", n_layer=2, n_embd=256, n_head=4, n_head_kv=4, n_ff=512, n_vocab=32256,
                        ctx=512, rope_theta=10000.0, rope_dim=32, qtype="Q8_0", tokenizer="phi2", name="tiny-phi2"),
    # Qwen2: q/k/v biases, NEOX rotary, ChatML; Phi-3: fused attn_qkv and gate|up ffn_up, head dim 96;
    # Gemma: head dim 256 (q_dim != n_embd), GeGLU, sqrt(n_embd)-scaled embeddings, tied lm_head
    "tiny-qwen2": Preset(arch="qwen2", n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512, n_vocab=32256,
                         ctx=512, rope_theta=1e6, eps=1e-6, qtype="Q4_K", tokenizer="chatml", name="tiny-qwen2"),
    "tiny-phi3": Preset(arch="phi3", n_layer=2, n_embd=768, n_head=8, n_head_kv=8, n_ff=512, n_vocab=32064,
                        ctx=512, rope_theta=10000.0, qtype="Q4_K", tokenizer="mistral", name="tiny-phi3"),
    "tiny-gemma": Preset(arch="gemma", n_layer=2, n_embd=256, n_head=2, n_head_kv=1, head_dim=256, n_ff=512,
                         n_vocab=32256, ctx=512, rope_theta=10000.0, eps=1e-6, qtype="Q4_K", tokenizer="mistral",
                         tied=True, name="tiny-gemma"),
    "tiny-gemma2": Preset(arch="gemma2", n_layer=2, n_embd=256, n_head=2, n_head_kv=1, head_dim=256, n_ff=512,
                          n_vocab=32256, ctx=512, rope_theta=10000.0, eps=1e-6, qtype="Q4_K", tokenizer="mistral",
                          tied=True, attn_softcap=50.0, final_softcap=30.0, sliding_window=24, name="tiny-gemma2"),
    "gemma2-9b": Preset(arch="gemma2", n_layer=42, n_embd=3584, n_head=16, n_head_kv=8, head_dim=256, n_ff=14336,
                        n_vocab=256000, ctx=8192, rope_theta=10000.0, eps=1e-6, tokenizer="mistral", tied=True,
                        attn_softcap=50.0, final_softcap=30.0, sliding_window=4096,
                        name="gemma-2-9b-it (random-init)"),
    # Command-R: bias-free LayerNorm, parallel residual, logit scale, tied lm_head; StarCoder2: LayerNorm
    # with bias, biased projections, gelu MLP without a gate, NEOX rotary
    "tiny-command-r": Preset(arch="command-r", n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512,
                             n_vocab=32256, ctx=512, rope_theta=8e6, qtype="Q4_K", tokenizer="llama3", tied=True,
                             logit_scale=0.0625, name="tiny-command-r"),
    "tiny-starcoder2": Preset(arch="starcoder2", n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=512,
                              n_vocab=32256, ctx=512, rope_theta=1e5, qtype="Q8_0", tokenizer="phi2",
                              name="tiny-starcoder2"),
    # Qwen2-MoE: routed experts without top-k renormalisation + a sigmoid-gated shared expert
    "tiny-qwen2moe": Preset(arch="qwen2moe", n_layer=2, n_embd=256, n_head=4, n_head_kv=2, n_ff=256, n_vocab=32256,
                            ctx=512, rope_theta=1e6, eps=1e-6, n_expert=4, n_expert_used=2, n_ff_shexp=512,
                            qtype="Q4_K", tokenizer="chatml", name="tiny-qwen2moe"),
    # DeepSeek-V2: latent attention (kv_lora_rank, 192-wide keys with a 64-dim shared rotary part,
    # 128-wide values), a leading dense layer, fine-grained experts plus shared experts, YaRN
    "tiny-deepseek2": Preset(arch="deepseek2", n_layer=2, n_embd=256, n_head=4, n_head_kv=4, head_dim=192,
                             head_dim_v=128, rope_dim=64, kv_lora_rank=256, n_ff=512, n_ff_exp=256, n_expert=4,
                             n_expert_used=2, n_expert_shared=1, n_layer_dense_lead=1, n_vocab=32256, ctx=512,
                             rope_theta=10000.0, eps=1e-6, yarn_factor=4.0, qtype="Q8_0", tokenizer="llama3",
                             name="tiny-deepseek2"),
    "qwen2-7b": Preset(arch="qwen2", n_layer=28, n_embd=3584, n_head=28, n_head_kv=4, n_ff=18944, n_vocab=152064,
                       ctx=32768, rope_theta=1e6, eps=1e-6, tokenizer="chatml", name="Qwen2-7B-Instruct (random-init)"),
    "phi3-mini": Preset(arch="phi3", n_layer=32, n_embd=3072, n_head=32, n_head_kv=32, n_ff=8192, n_vocab=32064,
                        ctx=4096, rope_theta=10000.0, tokenizer="mistral", name="Phi-3-mini-4k-instruct (random-init)"),
    "gemma-7b": Preset(arch="gemma", n_layer=28, n_embd=3072, n_head=16, n_head_kv=16, head_dim=256, n_ff=24576,
                       n_vocab=256000, ctx=8192, rope_theta=10000.0, eps=1e-6, tokenizer="mistral", tied=True,
                       name="gemma-7b-it (random-init)"),
}

CHATML_TEMPLATE = ("{% for message in messages %}{{'<|im_start|>' + message['role'] + '\n' + message['content'] + "
                   "'<|im_end|>' + '\n'}}{% endfor %}{% if add_generation_prompt %}{{ '<|im_start|>assistant\n' }}"
                   "{% endif %}")


def _bpe_asset():
    with gzip.open(ASSETS / "bpe32k.json.gz", "rt") as f:
        return json.load(f)


LLAMA3_SPECIAL = {0: "<|begin_of_text|>", 1: "<|end_of_text|>", 6: "<|start_header_id|>",
                  7: "<|end_header_id|>", 9: "<|eot_id|>"}


def build_vocab(p: Preset):
    """-> (model, tokens, types, merges, bos, eos, extra kv)"""
    a = _bpe_asset()
    base, merges = a["tokens"], a["merges"]
    if p.tokenizer == "mistral":
        # SentencePiece-style vocab: <unk> <s> </s>, byte tokens, then pieces; scores favour frequent merges
        toks = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)]
        types = [2, 3, 3] + [6] * 256
        from ..tokenizer import unicode_to_bytes
        u2b = unicode_to_bytes()
        seen = set(toks)
        for t in base:
            try:
                s = bytes(u2b[c] for c in t).decode("utf-8")
            except (KeyError, UnicodeDecodeError):
                continue
            s = s.replace(" ", "▁")
            if s in seen or not s:
                continue
            seen.add(s)
            toks.append(s)
            types.append(1)
            if len(toks) >= p.n_vocab:
                break
        i = 0
        while len(toks) < p.n_vocab:
            toks.append(f"▁filler{i}")
            types.append(1)
            i += 1
        scores = [0.0] * 259 + [-float(i) for i in range(len(toks) - 259)]
        return "llama", toks, types, None, scores, 1, 2, {"tokenizer.ggml.add_bos_token": True}
    n_special = {"llama3": 256, "chatml": 3}.get(p.tokenizer, 1)
    n_normal = p.n_vocab - n_special
    toks = list(base[:n_normal])
    i = 0
    while len(toks) < n_normal:
        toks.append(f"Ġfill{i}")
        i += 1
    types = [1] * n_normal
    if p.tokenizer == "llama3":
        for k in range(256):
            toks.append(LLAMA3_SPECIAL.get(k, f"<|reserved_special_token_{k}|>"))
            types.append(3)
        bos, eos = n_normal + 0, n_normal + 9
        extra = {"tokenizer.ggml.pre": "llama-bpe", "tokenizer.chat_template": LLAMA3_TEMPLATE,
                 "tokenizer.ggml.add_bos_token": True, "tokenizer.ggml.eot_token_id": n_normal + 9}
    elif p.tokenizer == "chatml":  # Qwen2: <|endoftext|>, <|im_start|>, <|im_end|> (eos of the instruct models)
        toks += ["<|endoftext|>", "<|im_start|>", "<|im_end|>"]
        types += [3, 3, 3]
        bos, eos = n_normal, n_normal + 2
        extra = {"tokenizer.ggml.pre": "qwen2", "tokenizer.chat_template": CHATML_TEMPLATE,
                 "tokenizer.ggml.add_bos_token": False, "tokenizer.ggml.eot_token_id": n_normal + 2}
    else:  # phi2: <|endoftext|> is bos = eos
        toks.append("<|endoftext|>")
        types.append(3)
        bos = eos = n_normal
        extra = {"tokenizer.ggml.pre": "phi-2", "tokenizer.ggml.add_bos_token": False}
    return "gpt2", toks, types, merges, None, bos, eos, extra


def _more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def _tensor_types(p: Preset, name: str, layer: int) -> int:
    if name.endswith("norm.weight") or name.endswith(".bias") or name == "rope_freqs.weight" or \
            name.endswith("ffn_gate_inp.weight") or name.endswith("ffn_gate_inp_shexp.weight"):
        return GGMLType.F32
    q = p.qtype
    if q == "F32":
        return GGMLType.F32
    if q == "F16":
        return GGMLType.F16
    if q == "Q8_0":
        return GGMLType.Q8_0
    if q == "Q4_K":
        return GGMLType.Q6_K if name == "output.weight" else GGMLType.Q4_K
    # Q4_K_M / Q5_K_M (llama.cpp's mixes: Q6_K output, and Q6_K attn_v / ffn_down on the
    # use_more_bits layers)
    if name == "output.weight":
        return GGMLType.Q6_K
    if name.endswith("attn_v.weight") and _more_bits(layer, p.n_layer):
        return GGMLType.Q6_K
    if (name.endswith("ffn_down.weight") or name.endswith("ffn_down_exps.weight")) and _more_bits(layer, p.n_layer):
        return GGMLType.Q6_K
    return GGMLType.Q5_K if q == "Q5_K_M" else GGMLType.Q4_K


def tensor_list(p: Preset):
    """(name, shape, layer) for every tensor of the preset, torch/numpy order."""
    d, hd = p.n_embd, p.hd
    qd, kvd = p.n_head * hd, p.n_head_kv * hd
    out = [("token_embd.weight", (p.n_vocab, d), -1)]
    for i in range(p.n_layer):
        b = f"blk.{i}."
        if p.arch == "phi2":
            out += [(b + "attn_norm.weight", (d,), i), (b + "attn_norm.bias", (d,), i),
                    (b + "attn_qkv.weight", (qd + 2 * kvd, d), i), (b + "attn_qkv.bias", (qd + 2 * kvd,), i),
                    (b + "attn_output.weight", (d, qd), i), (b + "attn_output.bias", (d,), i),
                    (b + "ffn_up.weight", (p.n_ff, d), i), (b + "ffn_up.bias", (p.n_ff,), i),
                    (b + "ffn_down.weight", (d, p.n_ff), i), (b + "ffn_down.bias", (d,), i)]
            continue
        if p.arch in ("command-r", "starcoder2"):
            out += [(b + "attn_norm.weight", (d,), i), (b + "attn_q.weight", (qd, d), i),
                    (b + "attn_k.weight", (kvd, d), i), (b + "attn_v.weight", (kvd, d), i),
                    (b + "attn_output.weight", (d, qd), i)]
            if p.arch == "command-r":  # parallel block: one norm, gated MLP
                out += [(b + "ffn_gate.weight", (p.n_ff, d), i), (b + "ffn_up.weight", (p.n_ff, d), i),
                        (b + "ffn_down.weight", (d, p.n_ff), i)]
            else:
                out += [(b + "attn_norm.bias", (d,), i), (b + "attn_q.bias", (qd,), i), (b + "attn_k.bias", (kvd,), i),
                        (b + "attn_v.bias", (kvd,), i), (b + "attn_output.bias", (d,), i),
                        (b + "ffn_norm.weight", (d,), i), (b + "ffn_norm.bias", (d,), i),
                        (b + "ffn_up.weight", (p.n_ff, d), i), (b + "ffn_up.bias", (p.n_ff,), i),
                        (b + "ffn_down.weight", (d, p.n_ff), i), (b + "ffn_down.bias", (d,), i)]
            continue
        if p.arch == "deepseek2":
            vd, rk = p.head_dim_v, p.kv_lora_rank
            out += [(b + "attn_norm.weight", (d,), i), (b + "attn_q.weight", (qd, d), i),
                    (b + "attn_kv_a_mqa.weight", (rk + p.rope_dim, d), i), (b + "attn_kv_a_norm.weight", (rk,), i),
                    (b + "attn_kv_b.weight", (p.n_head * (hd - p.rope_dim + vd), rk), i),
                    (b + "attn_output.weight", (d, p.n_head * vd), i), (b + "ffn_norm.weight", (d,), i)]
            if i < p.n_layer_dense_lead:
                out += [(b + "ffn_gate.weight", (p.n_ff, d), i), (b + "ffn_up.weight", (p.n_ff, d), i),
                        (b + "ffn_down.weight", (d, p.n_ff), i)]
            else:
                E, fe, fs_ = p.n_expert, p.n_ff_exp, p.n_ff_exp * p.n_expert_shared
                out += [(b + "ffn_gate_inp.weight", (E, d), i), (b + "ffn_gate_exps.weight", (E, fe, d), i),
                        (b + "ffn_up_exps.weight", (E, fe, d), i), (b + "ffn_down_exps.weight", (E, d, fe), i),
                        (b + "ffn_gate_shexp.weight", (fs_, d), i), (b + "ffn_up_shexp.weight", (fs_, d), i),
                        (b + "ffn_down_shexp.weight", (d, fs_), i)]
            continue
        if p.arch == "phi3":
            out += [(b + "attn_norm.weight", (d,), i), (b + "attn_qkv.weight", (qd + 2 * kvd, d), i),
                    (b + "attn_output.weight", (d, qd), i), (b + "ffn_norm.weight", (d,), i),
                    (b + "ffn_up.weight", (2 * p.n_ff, d), i), (b + "ffn_down.weight", (d, p.n_ff), i)]
            continue
        out += [(b + "attn_norm.weight", (d,), i), (b + "attn_q.weight", (qd, d), i),
                (b + "attn_k.weight", (kvd, d), i), (b + "attn_v.weight", (kvd, d), i),
                (b + "attn_output.weight", (d, qd), i), (b + "ffn_norm.weight", (d,), i)]
        if p.arch in ("qwen2", "qwen2moe"):
            out += [(b + "attn_q.bias", (qd,), i), (b + "attn_k.bias", (kvd,), i), (b + "attn_v.bias", (kvd,), i)]
        if p.n_ff_shexp:
            out += [(b + "ffn_gate_inp_shexp.weight", (d,), i), (b + "ffn_gate_shexp.weight", (p.n_ff_shexp, d), i),
                    (b + "ffn_up_shexp.weight", (p.n_ff_shexp, d), i), (b + "ffn_down_shexp.weight", (d, p.n_ff_shexp), i)]
        if p.arch == "gemma2":
            out += [(b + "post_attention_norm.weight", (d,), i), (b + "post_ffw_norm.weight", (d,), i)]
        if p.n_expert:
            E = p.n_expert
            out += [(b + "ffn_gate_inp.weight", (E, d), i), (b + "ffn_gate_exps.weight", (E, p.n_ff, d), i),
                    (b + "ffn_up_exps.weight", (E, p.n_ff, d), i), (b + "ffn_down_exps.weight", (E, d, p.n_ff), i)]
        else:
            out += [(b + "ffn_gate.weight", (p.n_ff, d), i), (b + "ffn_up.weight", (p.n_ff, d), i),
                    (b + "ffn_down.weight", (d, p.n_ff), i)]
    out.append(("output_norm.weight", (d,), -1))
    if p.arch == "phi2":
        out.append(("output_norm.bias", (d,), -1))
        out.append(("output.bias", (p.n_vocab,), -1))
    if p.arch == "starcoder2":
        out.append(("output_norm.bias", (d,), -1))
    if not p.tied:
        out.append(("output.weight", (p.n_vocab, d), -1))
    return out


def write_model(path: str, preset: str | Preset, seed: int = 0, exact: bool = False, std: float = 0.02,
                **overrides) -> str:
    """Write a random-init GGUF.  exact=True quantises real float weights (slow; tests only)."""
    p = PRESETS[preset] if isinstance(preset, str) else preset
    if overrides:
        p = replace(p, **overrides)
    model, toks, types, merges, scores, bos, eos, extra = build_vocab(p)
    w = GGUFWriter(path, p.arch)
    a = p.arch
    hd = p.hd
    w.add_string("general.name", p.name)
    w.add_uint32("general.file_type", {"Q4_K_M": 15, "Q5_K_M": 17}.get(p.qtype, 7))
    w.add_uint32(f"{a}.context_length", p.ctx)
    w.add_uint32(f"{a}.embedding_length", p.n_embd)
    w.add_uint32(f"{a}.block_count", p.n_layer)
    w.add_uint32(f"{a}.feed_forward_length", p.n_ff)
    w.add_uint32(f"{a}.attention.head_count", p.n_head)
    w.add_uint32(f"{a}.attention.head_count_kv", p.n_head_kv)
    w.add_float32(f"{a}.rope.freq_base", p.rope_theta)
    w.add_uint32(f"{a}.rope.dimension_count", p.rope_dim or hd)
    if p.head_dim:
        w.add_uint32(f"{a}.attention.key_length", hd)
        w.add_uint32(f"{a}.attention.value_length", p.head_dim_v or hd)
    if p.attn_softcap:
        w.add_float32(f"{a}.attn_logit_softcapping", p.attn_softcap)
    if p.final_softcap:
        w.add_float32(f"{a}.final_logit_softcapping", p.final_softcap)
    if p.sliding_window:
        w.add_uint32(f"{a}.attention.sliding_window", p.sliding_window)
    if p.logit_scale:
        w.add_float32(f"{a}.logit_scale", p.logit_scale)
    if p.kv_lora_rank:
        w.add_uint32(f"{a}.attention.kv_lora_rank", p.kv_lora_rank)
        w.add_uint32(f"{a}.expert_feed_forward_length", p.n_ff_exp)
        w.add_uint32(f"{a}.expert_shared_count", p.n_expert_shared)
        w.add_uint32(f"{a}.leading_dense_block_count", p.n_layer_dense_lead)
        w.add_float32(f"{a}.expert_weights_scale", 1.0)
    if p.yarn_factor:
        w.add_string(f"{a}.rope.scaling.type", "yarn")
        w.add_float32(f"{a}.rope.scaling.factor", p.yarn_factor)
        w.add_uint32(f"{a}.rope.scaling.original_context_length", p.ctx // int(p.yarn_factor))
        w.add_float32(f"{a}.rope.scaling.yarn_log_multiplier", 0.0707)
    if a in ("phi2", "command-r", "starcoder2"):
        w.add_float32(f"{a}.attention.layer_norm_epsilon", p.eps)
    else:
        w.add_float32(f"{a}.attention.layer_norm_rms_epsilon", p.eps)
        w.add_uint32(f"{a}.vocab_size", p.n_vocab)
    if p.n_expert:
        w.add_uint32(f"{a}.expert_count", p.n_expert)
        w.add_uint32(f"{a}.expert_used_count", p.n_expert_used)
    if p.n_ff_shexp:
        w.add_uint32(f"{a}.expert_feed_forward_length", p.n_ff)
        w.add_uint32(f"{a}.expert_shared_feed_forward_length", p.n_ff_shexp)
    w.add_string("tokenizer.ggml.model", model)
    w.add_array("tokenizer.ggml.tokens", toks, GGUFValueType.STRING)
    w.add_array("tokenizer.ggml.token_type", types, GGUFValueType.INT32)
    if merges is not None:
        w.add_array("tokenizer.ggml.merges", merges, GGUFValueType.STRING)
    if scores is not None:
        w.add_array("tokenizer.ggml.scores", scores, GGUFValueType.FLOAT32)
    w.add_uint32("tokenizer.ggml.bos_token_id", bos)
    w.add_uint32("tokenizer.ggml.eos_token_id", eos)
    for k, v in extra.items():
        if isinstance(v, bool):
            w.add_bool(k, v)
        elif isinstance(v, int):
            w.add_uint32(k, v)
        else:
            w.add_string(k, v)

    rng_master = np.random.default_rng(seed)
    for name, shape, layer in tensor_list(p):
        t = _tensor_types(p, name, layer)
        tseed = int(rng_master.integers(0, 2 ** 31))
        n = int(np.prod(shape))

        def payload(shape=shape, t=t, tseed=tseed, name=name, n=n):
            rng = np.random.default_rng(tseed)
            if name.endswith("norm.weight"):
                return (1.0 + 0.1 * rng.standard_normal(n)).astype(np.float32)
            if name.endswith(".bias"):
                return (0.02 * rng.standard_normal(n)).astype(np.float32)
            if name.endswith("ffn_gate_inp.weight") or name.endswith("ffn_gate_inp_shexp.weight"):
                return (std * rng.standard_normal(n)).astype(np.float32)
            sd = std
            if name == "token_embd.weight":
                sd = 1.0  # embeddings feed an RMSNorm; unit scale keeps activations O(1)
            if exact or t in (GGMLType.F32, GGMLType.F16, GGMLType.BF16):
                x = (sd * rng.standard_normal(n)).astype(np.float32)
                return quantize(x, t)
            if t == GGMLType.Q4_K:
                return random_q4_k_blocks(rng, n // 256, sd)
            if t == GGMLType.Q6_K:
                return random_q6_k_blocks(rng, n // 256, sd)
            if t == GGMLType.Q5_K:
                return random_q5_k_blocks(rng, n // 256, sd)
            if t == GGMLType.Q8_0:
                return random_q8_0_blocks(rng, n // 32, sd)
            raise NotImplementedError(t)

        w.add_tensor(name, shape, t, payload)
    w.write()
    return path


def write_lora(path: str, base_path: str, targets: Sequence[str] = ("attn_q", "ffn_down"), rank: int = 4,
               alpha: float = 8.0, seed: int = 0, std: float = 0.05) -> str:
    """A LoRA adapter GGUF for the model at base_path in llama.cpp's adapter layout: every weight
    `blk.N.<target>.weight` gets `.lora_a` [rank, K] and `.lora_b` [N, rank] (F32)."""
    from ..gguf import GGUFReader
    base = GGUFReader(base_path, load_tensors=False)
    w = GGUFWriter(path, base.architecture)
    w.add_string("general.type", "adapter")
    w.add_string("adapter.type", "lora")
    w.add_float32("adapter.lora.alpha", alpha)
    rng = np.random.default_rng(seed)
    for name, t in base.tensors.items():
        if not any(name.endswith(f".{tg}.weight") for tg in targets):
            continue
        N, K = t.shape[-2], t.shape[-1]
        a = (std * rng.standard_normal((rank, K))).astype(np.float32)
        b = (std * rng.standard_normal((N, rank))).astype(np.float32)
        w.add_tensor(name + ".lora_a", (rank, K), GGMLType.F32, a.reshape(-1))
        w.add_tensor(name + ".lora_b", (N, rank), GGMLType.F32, b.reshape(-1))
    w.write()
    return path


def write_whisper(path: str, n_audio_state: int = 64, n_audio_head: int = 2, n_audio_layer: int = 2,
                  n_text_state: int = 64, n_text_head: int = 2, n_text_layer: int = 2, n_mels: int = 80,
                  multilingual: bool = True, seed: int = 0, std: float = 0.05) -> str:
    """Random-init whisper.cpp GGML model (the `ggml-*.bin` layout of the reference's whisper
    backend) with the real vocabulary size, a Slaney mel filterbank and the OpenAI tensor names."""
    from ..tokenizer import unicode_to_bytes
    from .whisper import WhisperHParams, mel_filters, write_ggml
    n_vocab = 51865 if multilingual else 51864
    hp = WhisperHParams(n_vocab, 1500, n_audio_state, n_audio_head, n_audio_layer, 448, n_text_state, n_text_head,
                        n_text_layer, n_mels, 1)
    u2b = unicode_to_bytes()
    words = []
    for t in _bpe_asset()["tokens"]:
        try:
            words.append(bytes(u2b[c] for c in t))
        except KeyError:
            continue
        if len(words) == 50256:
            break
    while len(words) < 50256:
        words.append(b"<fill%d>" % len(words))
    rng = np.random.default_rng(seed)
    t = {}

    def r(*shape, sd=std):
        return (sd * rng.standard_normal(shape)).astype(np.float32)

    da, dt = n_audio_state, n_text_state
    t["encoder.positional_embedding"] = r(1500, da, sd=0.5)
    t["encoder.conv1.weight"], t["encoder.conv1.bias"] = r(da, n_mels, 3, sd=0.2), r(da)
    t["encoder.conv2.weight"], t["encoder.conv2.bias"] = r(da, da, 3, sd=0.2), r(da)

    def block(p, d, cross):
        for ln in ("attn_ln", "mlp_ln") + (("cross_attn_ln",) if cross else ()):
            t[p + ln + ".weight"], t[p + ln + ".bias"] = 1 + r(d, sd=0.1), r(d)
        for a in ("attn",) + (("cross_attn",) if cross else ()):
            for nm in ("query", "key", "value", "out"):
                t[f"{p}{a}.{nm}.weight"] = r(d, d, sd=1.0 / math.sqrt(d))
                if nm != "key":
                    t[f"{p}{a}.{nm}.bias"] = r(d)
        t[p + "mlp.0.weight"], t[p + "mlp.0.bias"] = r(4 * d, d, sd=1.0 / math.sqrt(d)), r(4 * d)
        t[p + "mlp.2.weight"], t[p + "mlp.2.bias"] = r(d, 4 * d, sd=0.5 / math.sqrt(d)), r(d)

    for i in range(n_audio_layer):
        block(f"encoder.blocks.{i}.", da, False)
    t["encoder.ln_post.weight"], t["encoder.ln_post.bias"] = 1 + r(da, sd=0.1), r(da)
    t["decoder.positional_embedding"] = r(448, dt, sd=0.1)
    t["decoder.token_embedding.weight"] = r(n_vocab, dt, sd=0.5)
    for i in range(n_text_layer):
        block(f"decoder.blocks.{i}.", dt, True)
    t["decoder.ln.weight"], t["decoder.ln.bias"] = 1 + r(dt, sd=0.1), r(dt)
    write_ggml(path, hp, mel_filters(n_mels), words, t)
    return path


def ensure_model(preset: str, cache_dir: Optional[str] = None, **kw) -> str:
    cache_dir = cache_dir or os.environ.get("LOCALAI_AMD_CACHE", os.path.join(os.path.expanduser("~"), ".cache",
                                                                               "localai_amd"))
    os.makedirs(cache_dir, exist_ok=True)
    tag = "-".join(f"{k}{v}" for k, v in sorted(kw.items()))
    path = os.path.join(cache_dir, f"{preset}{'-' + tag if tag else ''}.gguf")
    if not os.path.exists(path):
        tmp = path + ".partial"
        write_model(tmp, preset, **kw)
        os.replace(tmp, path)
    return path


def write_mmproj(path: str, out_dim: int, dim: int = 1024, n_layer: int = 23, heads: int = 16, ffn: int = 4096,
                 image_size: int = 336, patch: int = 14, seed: int = 0, std: float = 0.02,
                 pinpoints: Optional[List[int]] = None, siglip: bool = False) -> str:
    """Random-init llama.cpp-style LLaVA mmproj GGUF (CLIP ViT-L/14 layout + mlp2x_gelu projector).
    Defaults are the LLaVA-1.5/1.6 vision tower; tests pass tiny dims.  `siglip`: the moondream2
    layout instead -- no class token, post-LayerNorm instead of pre-LayerNorm, GELU, mean/std 0.5."""
    w = GGUFWriter(path, "clip")
    w.add_bool("clip.has_vision_encoder", True)
    w.add_bool("clip.has_llava_projector", True)
    w.add_string("clip.projector_type", "mlp")
    w.add_uint32("clip.vision.image_size", image_size)
    w.add_uint32("clip.vision.patch_size", patch)
    w.add_uint32("clip.vision.embedding_length", dim)
    w.add_uint32("clip.vision.feed_forward_length", ffn)
    w.add_uint32("clip.vision.projection_dim", out_dim)
    w.add_uint32("clip.vision.attention.head_count", heads)
    w.add_float32("clip.vision.attention.layer_norm_epsilon", 1e-5)
    w.add_uint32("clip.vision.block_count", n_layer)
    mean = [0.5, 0.5, 0.5] if siglip else [0.48145466, 0.4578275, 0.40821073]
    sd = [0.5, 0.5, 0.5] if siglip else [0.26862954, 0.26130258, 0.27577711]
    w.add_array("clip.vision.image_mean", mean, GGUFValueType.FLOAT32)
    w.add_array("clip.vision.image_std", sd, GGUFValueType.FLOAT32)
    w.add_bool("clip.use_gelu", siglip)
    if pinpoints:
        w.add_array("clip.vision.image_grid_pinpoints", pinpoints, GGUFValueType.INT32)
        w.add_string("clip.vision.mm_patch_merge_type", "spatial_unpad")
    rng = np.random.default_rng(seed)
    npatch = (image_size // patch) ** 2
    if siglip:
        tensors = [("v.patch_embd.weight", (dim, 3, patch, patch)), ("v.patch_embd.bias", (dim,)),
                   ("v.position_embd.weight", (npatch, dim)), ("v.post_ln.weight", (dim,)), ("v.post_ln.bias", (dim,))]
    else:
        tensors = [("v.patch_embd.weight", (dim, 3, patch, patch)), ("v.class_embd", (dim,)),
                   ("v.position_embd.weight", (npatch + 1, dim)), ("v.pre_ln.weight", (dim,)),
                   ("v.pre_ln.bias", (dim,))]
    for i in range(n_layer):
        b = f"v.blk.{i}."
        for nm in ("attn_q", "attn_k", "attn_v", "attn_out"):
            tensors += [(b + nm + ".weight", (dim, dim)), (b + nm + ".bias", (dim,))]
        tensors += [(b + "ln1.weight", (dim,)), (b + "ln1.bias", (dim,)), (b + "ln2.weight", (dim,)),
                    (b + "ln2.bias", (dim,)), (b + "ffn_down.weight", (ffn, dim)), (b + "ffn_down.bias", (ffn,)),
                    (b + "ffn_up.weight", (dim, ffn)), (b + "ffn_up.bias", (dim,))]
    tensors += [("mm.0.weight", (out_dim, dim)), ("mm.0.bias", (out_dim,)), ("mm.2.weight", (out_dim, out_dim)),
                ("mm.2.bias", (out_dim,))]
    if pinpoints:
        tensors.append(("model.image_newline", (out_dim,)))
    for name, shape in tensors:
        n = int(np.prod(shape))
        if name.endswith(("ln1.weight", "ln2.weight", "pre_ln.weight", "post_ln.weight")):
            a = (1.0 + 0.05 * rng.standard_normal(n)).astype(np.float32)
        else:
            a = (std * rng.standard_normal(n)).astype(np.float32)
        big = len(shape) >= 2 and n >= 1 << 16
        t = GGMLType.F16 if big else GGMLType.F32
        w.add_tensor(name, shape, t, quantize(a, t))
    w.write()
    return path


def write_bert(path: str, dim: int = 384, n_layer: int = 6, heads: int = 12, ffn: int = 1536, ctx: int = 512,
               seed: int = 0, std: float = 0.05, words: Optional[List[str]] = None, ranker: bool = False) -> str:
    """Random-init llama.cpp-style `bert` GGUF (all-MiniLM-L6-v2 geometry by default) with a small
    WordPiece vocabulary (specials, U+2581-prefixed word pieces, bare continuation pieces).
    ranker=True writes a cross-encoder (pooling_type 4 = RANK, cls / cls.output head)."""
    words = words or ("the a an of to and in is it that for on with as was at by be this are from or have "
                      "model server token request graph kernel memory stream batch hello world image text "
                      "quick brown fox dog cat red green blue gpu fast slow").split()
    toks = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    toks += ["▁" + c for c in ".,!?;:'\"()-"]
    toks += ["▁" + w for w in words]
    toks += list("abcdefghijklmnopqrstuvwxyz0123456789")
    toks += ["▁" + c for c in "abcdefghijklmnopqrstuvwxyz0123456789"]
    w = GGUFWriter(path, "bert")
    w.add_string("general.name", "synthetic-minilm")
    w.add_uint32("bert.context_length", ctx)
    w.add_uint32("bert.embedding_length", dim)
    w.add_uint32("bert.feed_forward_length", ffn)
    w.add_uint32("bert.block_count", n_layer)
    w.add_uint32("bert.attention.head_count", heads)
    w.add_float32("bert.attention.layer_norm_epsilon", 1e-12)
    w.add_bool("bert.attention.causal", False)
    w.add_uint32("bert.pooling_type", 4 if ranker else 1)
    w.add_string("tokenizer.ggml.model", "bert")
    w.add_array("tokenizer.ggml.tokens", toks, GGUFValueType.STRING)
    w.add_array("tokenizer.ggml.token_type", [3] * 5 + [1] * (len(toks) - 5), GGUFValueType.INT32)
    w.add_uint32("tokenizer.ggml.unknown_token_id", 1)
    w.add_uint32("tokenizer.ggml.cls_token_id", 2)
    w.add_uint32("tokenizer.ggml.seperator_token_id", 3)
    w.add_uint32("tokenizer.ggml.padding_token_id", 0)
    rng = np.random.default_rng(seed)
    V = len(toks)
    tensors = [("token_embd.weight", (V, dim)), ("token_types.weight", (2, dim)), ("position_embd.weight", (ctx, dim)),
               ("token_embd_norm.weight", (dim,)), ("token_embd_norm.bias", (dim,))]
    for i in range(n_layer):
        b = f"blk.{i}."
        for nm in ("attn_q", "attn_k", "attn_v", "attn_output"):
            tensors += [(b + nm + ".weight", (dim, dim)), (b + nm + ".bias", (dim,))]
        tensors += [(b + "attn_output_norm.weight", (dim,)), (b + "attn_output_norm.bias", (dim,)),
                    (b + "ffn_up.weight", (ffn, dim)), (b + "ffn_up.bias", (ffn,)),
                    (b + "ffn_down.weight", (dim, ffn)), (b + "ffn_down.bias", (dim,)),
                    (b + "layer_output_norm.weight", (dim,)), (b + "layer_output_norm.bias", (dim,))]
    if ranker:
        tensors += [("cls.weight", (dim, dim)), ("cls.bias", (dim,)), ("cls.output.weight", (1, dim)),
                    ("cls.output.bias", (1,))]
    for name, shape in tensors:
        n = int(np.prod(shape))
        if name.endswith("norm.weight"):
            a = (1.0 + 0.05 * rng.standard_normal(n)).astype(np.float32)
        else:
            a = (std * rng.standard_normal(n)).astype(np.float32)
        t = GGMLType.F16 if len(shape) >= 2 else GGMLType.F32
        w.add_tensor(name, shape, t, quantize(a, t))
    w.write()
    return path


def write_hf_checkpoint(out_dir: str, kind: str = "llama", n_layer: int = 2, hidden: int = 64, heads: int = 4,
                        kv_heads: int = 2, ffn: int = 128, n_experts: int = 0, seed: int = 0,
                        rope_scaling: Optional[dict] = None, dtype: str = "float32") -> str:
    """Random-init Hugging Face checkpoint directory (config.json, model.safetensors, tokenizer.json,
    tokenizer_config.json) built with `transformers` itself, so a test can compare the engine with
    the library's own forward.  kind: llama | mistral | qwen2 | mixtral.  The tokenizer is a byte-level
    BPE (this package's 32k asset + the Llama-3 special tokens) with the Llama-3 chat template."""
    import torch
    import transformers as tf
    from tokenizers import Regex, Tokenizer as HFTok, decoders, models, pre_tokenizers

    from ..tokenizer import LLAMA3_PAT
    a = _bpe_asset()
    n_normal = len(a["tokens"])
    vocab = {t: i for i, t in enumerate(a["tokens"])}
    specials = [LLAMA3_SPECIAL.get(k, f"<|reserved_special_token_{k}|>") for k in range(16)]
    n_vocab = n_normal + len(specials)
    bos, eos = n_normal + 0, n_normal + 9
    torch.manual_seed(seed)
    common = dict(vocab_size=n_vocab, hidden_size=hidden, intermediate_size=ffn, num_hidden_layers=n_layer,
                  num_attention_heads=heads, num_key_value_heads=kv_heads, max_position_embeddings=512,
                  rms_norm_eps=1e-5, bos_token_id=bos, eos_token_id=eos, tie_word_embeddings=False)
    if rope_scaling:
        common["rope_scaling"] = rope_scaling
    if kind in ("llama", "mistral"):
        cfg = (tf.LlamaConfig if kind == "llama" else tf.MistralConfig)(rope_theta=500000.0, **common)
        model = (tf.LlamaForCausalLM if kind == "llama" else tf.MistralForCausalLM)(cfg)
    elif kind == "qwen2":
        model = tf.Qwen2ForCausalLM(tf.Qwen2Config(rope_theta=1000000.0, **common))
    elif kind == "mixtral":
        model = tf.MixtralForCausalLM(tf.MixtralConfig(num_local_experts=n_experts or 4, num_experts_per_tok=2,
                                                       rope_theta=1000000.0, **common))
    else:
        raise ValueError(kind)
    with torch.no_grad():  # larger-than-default weights so the logits are not all near zero
        for n, p in model.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, 0.08)
            elif "norm" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            else:
                p.normal_(0.0, 0.05)
    model = model.to(getattr(torch, dtype))
    os.makedirs(out_dir, exist_ok=True)
    model.save_pretrained(out_dir, safe_serialization=True)
    tok = HFTok(models.BPE(vocab=vocab, merges=[tuple(m.split(" ", 1)) for m in a["merges"]], ignore_merges=True))
    tok.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.Split(Regex(LLAMA3_PAT), behavior="isolated"),
                                                 pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    from tokenizers import AddedToken
    tok.add_special_tokens([AddedToken(s, special=True, normalized=False) for s in specials])
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": specials[0], "eos_token": specials[9], "add_bos_token": True,
                   "chat_template": LLAMA3_TEMPLATE, "tokenizer_class": "PreTrainedTokenizerFast"}, f)
    return out_dir


def write_hf_mamba(out_dir: str, hidden: int = 64, n_layer: int = 2, state: int = 16, seed: int = 0,
                   dtype: str = "float32") -> str:
    """Random-init transformers `MambaForCausalLM` directory with this package's byte-level BPE
    tokenizer (`<|endoftext|>` = eos, the MAMBA_CHAT convention)."""
    import torch
    import transformers as tf
    from tokenizers import AddedToken, Regex, Tokenizer as HFTok, decoders, models, pre_tokenizers

    from ..tokenizer import GPT2_PAT
    a = _bpe_asset()
    vocab = {t: i for i, t in enumerate(a["tokens"])}
    n_vocab = len(vocab) + 1
    torch.manual_seed(seed)
    cfg = tf.MambaConfig(vocab_size=n_vocab, hidden_size=hidden, state_size=state, num_hidden_layers=n_layer,
                         eos_token_id=n_vocab - 1, bos_token_id=n_vocab - 1, pad_token_id=n_vocab - 1)
    m = tf.MambaForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2 and "conv1d" not in n:
                p.normal_(0.0, 0.08)
    m.to(getattr(torch, dtype)).save_pretrained(out_dir, safe_serialization=True)
    tok = HFTok(models.BPE(vocab=vocab, merges=[tuple(x.split(" ", 1)) for x in a["merges"]]))
    tok.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.Split(Regex(GPT2_PAT), behavior="isolated"),
                                                 pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tok.add_special_tokens([AddedToken("<|endoftext|>", special=True)])
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    return out_dir


def gptq_quantize_checkpoint(src_dir: str, out_dir: str, oracle_dir: str, group_size: int = 32, bits: int = 4,
                             act_order: bool = False, seed: int = 0) -> str:
    """GPTQ-format copy of an HF checkpoint (every decoder linear as qweight / qzeros / scales /
    g_idx, AutoGPTQ v1 packing with zero - 1 stored) plus, in `oracle_dir`, the same model with the
    quantised-then-dequantised float weights -- what a GPTQ loader must reproduce.  Plain
    round-to-nearest asymmetric quantisation per (group, output column); act_order shuffles which
    input rows share a group (g_idx), as desc_act checkpoints do."""
    import shutil

    import torch
    from safetensors.torch import load_file, save_file
    rng = np.random.default_rng(seed)
    sd = load_file(os.path.join(src_dir, "model.safetensors"))
    pack, qmax = 32 // bits, (1 << bits) - 1
    out, orc = {}, {}
    for k, t in sd.items():
        lin = k.endswith(".weight") and t.dim() == 2 and ".layers." in k and "norm" not in k
        if not lin:
            out[k] = t
            orc[k] = t
            continue
        W = t.float().numpy().T.copy()                       # [K, N]
        K, N = W.shape
        G = K // group_size
        order = rng.permutation(K) if act_order else np.arange(K)
        g_idx = np.empty(K, dtype=np.int32)
        g_idx[order] = np.arange(K) // group_size           # rows order[j] share group j // group_size
        scales = np.zeros((G, N), np.float32)
        zeros = np.zeros((G, N), np.int64)
        for g in range(G):
            rows = W[g_idx == g]
            lo, hi = np.minimum(rows.min(0), 0), np.maximum(rows.max(0), 0)
            sc = np.maximum((hi - lo) / qmax, 1e-8).astype(np.float16).astype(np.float32)
            scales[g], zeros[g] = sc, np.clip(np.round(-lo / sc), 0, qmax)
        q = np.clip(np.round(W / scales[g_idx]) + zeros[g_idx], 0, qmax).astype(np.int64)   # [K, N]
        deq = (q - zeros[g_idx]) * scales[g_idx]
        qw = np.zeros((K // pack, N), np.int64)
        for j in range(pack):
            qw |= q[j::pack] << (bits * j)
        zs = zeros - 1                                       # AutoGPTQ v1 stores zero - 1 (as unsigned bits)
        qz = np.zeros((G, N // pack), np.int64)
        for j in range(pack):
            qz |= (zs[:, j::pack] & qmax) << (bits * j)
        base = k[:-len(".weight")]
        out[base + ".qweight"] = torch.from_numpy(qw.astype(np.uint32).view(np.int32))
        out[base + ".qzeros"] = torch.from_numpy(qz.astype(np.uint32).view(np.int32))
        out[base + ".scales"] = torch.from_numpy(scales.astype(np.float16))
        out[base + ".g_idx"] = torch.from_numpy(g_idx)
        orc[k] = torch.from_numpy(deq.T.astype(np.float32)).to(t.dtype)
    for d, tensors in ((out_dir, out), (oracle_dir, orc)):
        os.makedirs(d, exist_ok=True)
        for fn in os.listdir(src_dir):
            if fn != "model.safetensors":
                shutil.copy(os.path.join(src_dir, fn), os.path.join(d, fn))
        save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(d, "model.safetensors"),
                  metadata={"format": "pt"})
    with open(os.path.join(out_dir, "quantize_config.json"), "w") as f:
        json.dump({"bits": bits, "group_size": group_size, "desc_act": act_order, "sym": False,
                   "quant_method": "gptq", "checkpoint_format": "gptq"}, f)
    return out_dir


def write_hf_rwkv(out_dir: str, hidden: int = 64, n_layer: int = 2, seed: int = 0) -> str:
    """Random-init transformers `RwkvForCausalLM` (RWKV-4) directory with this package's byte-level
    BPE tokenizer; rescale_every=0 so eval-mode forwards are not rescaled."""
    import torch
    import transformers as tf
    from tokenizers import Regex, Tokenizer as HFTok, decoders, models, pre_tokenizers

    from ..tokenizer import GPT2_PAT
    a = _bpe_asset()
    vocab = {t: i for i, t in enumerate(a["tokens"])}
    torch.manual_seed(seed)
    cfg = tf.RwkvConfig(vocab_size=len(vocab), hidden_size=hidden, num_hidden_layers=n_layer,
                        attention_hidden_size=hidden, intermediate_size=4 * hidden, context_length=256,
                        rescale_every=0, bos_token_id=0, eos_token_id=0)
    m = tf.RwkvForCausalLM(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if p.dim() >= 2:
                p.normal_(0.0, 0.1)
            elif "time_decay" in n:
                p.copy_(torch.randn_like(p) * 0.5 - 1.0)
            elif "time_first" in n:
                p.copy_(torch.randn_like(p) * 0.3)
            elif "time_mix" in n:
                p.copy_(torch.rand_like(p))
    m.save_pretrained(out_dir, safe_serialization=True)
    tok = HFTok(models.BPE(vocab=vocab, merges=[tuple(x.split(" ", 1)) for x in a["merges"]]))
    tok.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.Split(Regex(GPT2_PAT), behavior="isolated"),
                                                 pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    return out_dir


SD15_UNET = dict(block_out_channels=[320, 640, 1280, 1280], layers_per_block=2, cross_attention_dim=768,
                 attention_head_dim=8, norm_num_groups=32, in_channels=4, out_channels=4, sample_size=64,
                 down_block_types=["CrossAttnDownBlock2D"] * 3 + ["DownBlock2D"],
                 up_block_types=["UpBlock2D"] + ["CrossAttnUpBlock2D"] * 3, flip_sin_to_cos=True, freq_shift=0)
SD15_VAE = dict(block_out_channels=[128, 256, 512, 512], layers_per_block=2, latent_channels=4, norm_num_groups=32,
                in_channels=3, out_channels=3, scaling_factor=0.18215)
SD15_TEXT = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                 vocab_size=49408, max_position_embeddings=77, hidden_act="quick_gelu")
# Stable Diffusion XL base 1.0 (diffusers configs): 2.6 B-parameter UNet, CLIP-L + OpenCLIP bigG
SDXL_UNET = dict(block_out_channels=[320, 640, 1280], layers_per_block=2, cross_attention_dim=2048,
                 attention_head_dim=[5, 10, 20], transformer_layers_per_block=[1, 2, 10], norm_num_groups=32,
                 in_channels=4, out_channels=4, sample_size=128, use_linear_projection=True,
                 down_block_types=["DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"],
                 up_block_types=["CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"],
                 addition_embed_type="text_time", addition_time_embed_dim=256,
                 projection_class_embeddings_input_dim=2816, flip_sin_to_cos=True, freq_shift=0)
SDXL_VAE = dict(SD15_VAE, scaling_factor=0.13025, sample_size=1024)
SDXL_TEXT2 = dict(hidden_size=1280, num_hidden_layers=32, num_attention_heads=20, intermediate_size=5120,
                  vocab_size=49408, max_position_embeddings=77, hidden_act="gelu", projection_dim=1280)


def _clip_byte_vocab():
    """A byte-level CLIP BPE vocabulary with no merges: every byte, every byte + `</w>`, and the
    two specials -- enough for transformers' CLIPTokenizer to tokenise any text."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs, n = bs[:], 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    chars = [chr(c) for c in cs]
    toks = chars + [c + "</w>" for c in chars] + ["<|startoftext|>", "<|endoftext|>"]
    return {t: i for i, t in enumerate(toks)}


def write_sd_pipeline(out_dir: str, size: str = "tiny", seed: int = 0, v_prediction: bool = False,
                      depth: bool = False) -> str:
    """Random-init Stable Diffusion pipeline directory in the diffusers layout (model_index.json,
    unet/, vae/, text_encoder/ (transformers CLIPTextModel), tokenizer/, scheduler/; SDXL adds
    text_encoder_2/ (CLIPTextModelWithProjection) and tokenizer_2/).
    size="sd15": the SD-1.5 architecture (860M-parameter UNet); "sdxl": SDXL base 1.0;
    "tiny": a two-level toy; "tiny-xl": a two-level SDXL-shaped toy.
    depth=True: a StableDiffusionDepth2ImgPipeline (5-channel UNet input, a transformers DPT
    depth_estimator/ and its feature_extractor/)."""
    import torch
    import transformers as tf
    from safetensors.torch import save_file

    from .sd import UNet, VaeDecoder, VaeEncoder
    xl = size in ("sdxl", "tiny-xl")
    tc2 = None
    if size == "sd15":
        uc, vc, tc = dict(SD15_UNET), dict(SD15_VAE), dict(SD15_TEXT)
    elif size == "sdxl":
        uc, vc, tc, tc2 = dict(SDXL_UNET), dict(SDXL_VAE), dict(SD15_TEXT), dict(SDXL_TEXT2)
    elif size == "tiny-xl":
        vocab = _clip_byte_vocab()
        sp = dict(vocab_size=len(vocab), bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
                  pad_token_id=vocab["<|endoftext|>"])
        tc = dict(SD15_TEXT, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64, **sp)
        tc2 = dict(SDXL_TEXT2, hidden_size=48, num_hidden_layers=3, num_attention_heads=2, intermediate_size=96,
                   projection_dim=16, **sp)
        uc = dict(SDXL_UNET, block_out_channels=[32, 64], layers_per_block=1, cross_attention_dim=32 + 48,
                  attention_head_dim=[2, 4], transformer_layers_per_block=[1, 2], norm_num_groups=8, sample_size=8,
                  down_block_types=["DownBlock2D", "CrossAttnDownBlock2D"],
                  up_block_types=["CrossAttnUpBlock2D", "UpBlock2D"], addition_time_embed_dim=8,
                  projection_class_embeddings_input_dim=16 + 6 * 8)
        vc = dict(SDXL_VAE, block_out_channels=[16, 32], layers_per_block=1, norm_num_groups=8)
    else:
        uc = dict(SD15_UNET, block_out_channels=[32, 64], layers_per_block=1, cross_attention_dim=32,
                  attention_head_dim=[2, 4], norm_num_groups=8, sample_size=8,
                  down_block_types=["CrossAttnDownBlock2D", "DownBlock2D"],
                  up_block_types=["UpBlock2D", "CrossAttnUpBlock2D"])
        vc = dict(SD15_VAE, block_out_channels=[16, 32], layers_per_block=1, norm_num_groups=8)
        vocab = _clip_byte_vocab()
        tc = dict(SD15_TEXT, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64,
                  vocab_size=len(vocab), bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
                  pad_token_id=vocab["<|endoftext|>"])
    if v_prediction:
        uc["use_linear_projection"] = True
    if depth:
        uc["in_channels"] = 5
    torch.manual_seed(seed)
    subs = ["unet", "vae", "text_encoder", "tokenizer", "scheduler"] + (["text_encoder_2", "tokenizer_2"] if xl else [])
    for sub in subs:
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    for sub, cls, c in (("unet", UNet, uc), ("vae", VaeDecoder, vc)):
        m = cls(c)
        with open(os.path.join(out_dir, sub, "config.json"), "w") as f:
            json.dump(dict(c, _class_name="UNet2DConditionModel" if sub == "unet" else "AutoencoderKL"), f)
        dt = torch.bfloat16 if size in ("sd15", "sdxl") else torch.float32  # halves the multi-GB UNet files
        sd = m.state_dict()
        if sub == "vae":  # the full AutoencoderKL: the encoder half too (img2img)
            sd.update(VaeEncoder(c).state_dict())
        save_file({k: v.to(dt).contiguous() for k, v in sd.items()},
                  os.path.join(out_dir, sub, "diffusion_pytorch_model.safetensors"))
    te = tf.CLIPTextModel(tf.CLIPTextConfig(**tc))
    te.save_pretrained(os.path.join(out_dir, "text_encoder"), safe_serialization=True)
    if tc2 is not None:
        te2 = tf.CLIPTextModelWithProjection(tf.CLIPTextConfig(**tc2))
        if size == "sdxl":
            te2 = te2.to(torch.bfloat16)
        te2.save_pretrained(os.path.join(out_dir, "text_encoder_2"), safe_serialization=True)
    vocab = _clip_byte_vocab()
    for tk in ("tokenizer", "tokenizer_2") if xl else ("tokenizer",):
        with open(os.path.join(out_dir, tk, "vocab.json"), "w") as f:
            json.dump(vocab, f)
        with open(os.path.join(out_dir, tk, "merges.txt"), "w") as f:
            f.write("#version: 0.2\n")
    with open(os.path.join(out_dir, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "DDIMScheduler", "beta_start": 0.00085, "beta_end": 0.012,
                   "beta_schedule": "scaled_linear", "num_train_timesteps": 1000, "steps_offset": 1,
                   "set_alpha_to_one": False, "clip_sample": False,
                   "prediction_type": "v_prediction" if v_prediction else "epsilon"}, f)
    if depth:
        tiny = size.startswith("tiny")
        dc = tf.DPTConfig(hidden_size=32, num_hidden_layers=4, num_attention_heads=2, intermediate_size=64,
                          image_size=64, patch_size=16, backbone_out_indices=[0, 1, 2, 3],
                          neck_hidden_sizes=[8, 16, 32, 32], fusion_hidden_size=16) if tiny else tf.DPTConfig()
        tf.DPTForDepthEstimation(dc).save_pretrained(os.path.join(out_dir, "depth_estimator"), safe_serialization=True)
        px = 64 if tiny else 384
        tf.DPTImageProcessor(size={"height": px, "width": px}, keep_aspect_ratio=False).save_pretrained(
            os.path.join(out_dir, "feature_extractor"))
    with open(os.path.join(out_dir, "model_index.json"), "w") as f:
        json.dump({"_class_name": "StableDiffusionXLPipeline", "force_zeros_for_empty_prompt": True} if xl
                  else {"_class_name": "StableDiffusionDepth2ImgPipeline" if depth else "StableDiffusionPipeline"}, f)
    return out_dir


def write_t2v_pipeline(out_dir: str, seed: int = 0) -> str:
    """Random-init text-to-video pipeline (diffusers TextToVideoSDPipeline layout: a two-level
    UNet3DConditionModel toy, the SD VAE, a CLIP text encoder and its byte-level tokenizer, a DDIM
    scheduler) for models/video.py."""
    import torch
    import transformers as tf
    from safetensors.torch import save_file

    from .sd import VaeDecoder, VaeEncoder
    from .video import UNet3D
    uc = {"_class_name": "UNet3DConditionModel", "act_fn": "silu", "attention_head_dim": 8,
          "block_out_channels": [32, 64], "cross_attention_dim": 32, "layers_per_block": 1, "in_channels": 4,
          "out_channels": 4, "norm_num_groups": 8, "norm_eps": 1e-5, "sample_size": 8,
          "down_block_types": ["CrossAttnDownBlock3D", "DownBlock3D"],
          "up_block_types": ["UpBlock3D", "CrossAttnUpBlock3D"]}
    vc = dict(SD15_VAE, block_out_channels=[16, 32], layers_per_block=1, norm_num_groups=8)
    vocab = _clip_byte_vocab()
    tc = dict(SD15_TEXT, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64,
              vocab_size=len(vocab), bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
              pad_token_id=vocab["<|endoftext|>"], hidden_act="gelu")
    torch.manual_seed(seed)
    for sub in ("unet", "vae", "text_encoder", "tokenizer", "scheduler"):
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    unet = UNet3D(uc)
    with open(os.path.join(out_dir, "unet", "config.json"), "w") as f:
        json.dump(uc, f)
    save_file({k: v.contiguous() for k, v in unet.state_dict().items()},
              os.path.join(out_dir, "unet", "diffusion_pytorch_model.safetensors"))
    sd = VaeDecoder(vc).state_dict()
    sd.update(VaeEncoder(vc).state_dict())
    with open(os.path.join(out_dir, "vae", "config.json"), "w") as f:
        json.dump(dict(vc, _class_name="AutoencoderKL"), f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(out_dir, "vae", "diffusion_pytorch_model.safetensors"))
    tf.CLIPTextModel(tf.CLIPTextConfig(**tc)).save_pretrained(os.path.join(out_dir, "text_encoder"), safe_serialization=True)
    with open(os.path.join(out_dir, "tokenizer", "vocab.json"), "w") as f:
        json.dump(vocab, f)
    with open(os.path.join(out_dir, "tokenizer", "merges.txt"), "w") as f:
        f.write("#version: 0.2\n")
    with open(os.path.join(out_dir, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "DDIMScheduler", "beta_start": 0.00085, "beta_end": 0.012,
                   "beta_schedule": "scaled_linear", "num_train_timesteps": 1000, "steps_offset": 1,
                   "set_alpha_to_one": False, "clip_sample": False, "prediction_type": "epsilon"}, f)
    with open(os.path.join(out_dir, "model_index.json"), "w") as f:
        json.dump({"_class_name": "TextToVideoSDPipeline", "unet": ["diffusers", "UNet3DConditionModel"],
                   "vae": ["diffusers", "AutoencoderKL"], "text_encoder": ["transformers", "CLIPTextModel"],
                   "tokenizer": ["transformers", "CLIPTokenizer"], "scheduler": ["diffusers", "DDIMScheduler"]}, f)
    return out_dir


def write_svd_pipeline(out_dir: str, seed: int = 0) -> str:
    """Random-init image-to-video pipeline (diffusers StableVideoDiffusionPipeline layout: a
    two-level UNetSpatioTemporalConditionModel toy, an AutoencoderKLTemporalDecoder toy, a
    transformers CLIPVisionModelWithProjection image encoder, an EulerDiscrete scheduler with
    Karras sigmas / v-prediction) for models/svd.py."""
    import torch
    import transformers as tf
    from safetensors.torch import save_file

    from .sd import VaeEncoder
    from .svd import TemporalVaeDecoder, UNetSTC
    uc = {"_class_name": "UNetSpatioTemporalConditionModel", "block_out_channels": [32, 64], "layers_per_block": 1,
          "num_attention_heads": [2, 4], "cross_attention_dim": 32, "addition_time_embed_dim": 8,
          "projection_class_embeddings_input_dim": 24, "in_channels": 8, "out_channels": 4, "num_frames": 4,
          "norm_num_groups": 8, "transformer_layers_per_block": 1,
          "down_block_types": ["CrossAttnDownBlockSpatioTemporal", "DownBlockSpatioTemporal"],
          "up_block_types": ["UpBlockSpatioTemporal", "CrossAttnUpBlockSpatioTemporal"]}
    vc = dict(SD15_VAE, _class_name="AutoencoderKLTemporalDecoder", block_out_channels=[16, 32], layers_per_block=2,
              norm_num_groups=8)
    torch.manual_seed(seed)
    for sub in ("unet", "vae", "image_encoder", "feature_extractor", "scheduler"):
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    unet = UNetSTC(uc)
    with open(os.path.join(out_dir, "unet", "config.json"), "w") as f:
        json.dump(uc, f)
    save_file({k: v.contiguous() for k, v in unet.state_dict().items()},
              os.path.join(out_dir, "unet", "diffusion_pytorch_model.safetensors"))
    sd = TemporalVaeDecoder(vc).state_dict()
    sd.update(VaeEncoder(vc).state_dict())
    sd = {k: v for k, v in sd.items() if not k.startswith("post_quant_conv.")}
    with open(os.path.join(out_dir, "vae", "config.json"), "w") as f:
        json.dump(vc, f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(out_dir, "vae", "diffusion_pytorch_model.safetensors"))
    ic = tf.CLIPVisionConfig(hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64,
                             image_size=32, patch_size=16, projection_dim=32)
    tf.CLIPVisionModelWithProjection(ic).save_pretrained(os.path.join(out_dir, "image_encoder"), safe_serialization=True)
    with open(os.path.join(out_dir, "feature_extractor", "preprocessor_config.json"), "w") as f:
        json.dump({"image_processor_type": "CLIPImageProcessor", "crop_size": 32, "size": {"shortest_edge": 32},
                   "image_mean": [0.48145466, 0.4578275, 0.40821073],
                   "image_std": [0.26862954, 0.26130258, 0.27577711]}, f)
    with open(os.path.join(out_dir, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "EulerDiscreteScheduler", "sigma_min": 0.002, "sigma_max": 700.0,
                   "use_karras_sigmas": True, "prediction_type": "v_prediction", "timestep_type": "continuous",
                   "timestep_spacing": "leading", "num_train_timesteps": 1000}, f)
    with open(os.path.join(out_dir, "model_index.json"), "w") as f:
        json.dump({"_class_name": "StableVideoDiffusionPipeline", "unet": ["diffusers", "UNetSpatioTemporalConditionModel"],
                   "vae": ["diffusers", "AutoencoderKLTemporalDecoder"],
                   "image_encoder": ["transformers", "CLIPVisionModelWithProjection"],
                   "feature_extractor": ["transformers", "CLIPImageProcessor"],
                   "scheduler": ["diffusers", "EulerDiscreteScheduler"]}, f)
    return out_dir


def write_sd_single_file(path: str, size: str = "tiny", seed: int = 0, fam: str = "", hints: bool = True) -> str:
    """A random-init Stable Diffusion checkpoint as ONE file in the original LDM / SGM layout
    (what `from_single_file` reads: the AIO DreamShaper_8_pruned.safetensors shape at
    size="sd15"); fam: sd1 / sd2 / sdxl (default from size).  The exact configs ride along in
    the safetensors metadata unless hints=False (then the loader infers them)."""
    import tempfile

    from .sd_single_file import to_single_file
    fam = fam or ("sdxl" if size in ("sdxl", "tiny-xl") else "sd1")
    with tempfile.TemporaryDirectory() as td:
        d = write_sd_pipeline(os.path.join(td, "p"), size=size, seed=seed, v_prediction=(fam == "sd2"))
        return to_single_file(d, path, fam, with_hints=hints)


def write_controlnet(out_dir: str, pipe_dir: str, seed: int = 0, zero: bool = True) -> str:
    """Random-init diffusers ControlNetModel directory matching the UNet of `pipe_dir` (same block
    layout; conditioning_embedding_out_channels scaled down for toy pipelines).  zero=True keeps
    the zero-initialised output convolutions of a fresh ControlNet (its residuals are exactly 0)."""
    import torch
    from safetensors.torch import save_file

    from .sd import ControlNet
    with open(os.path.join(pipe_dir, "unet", "config.json")) as f:
        uc = json.load(f)
    c = {k: v for k, v in uc.items() if k not in ("up_block_types", "out_channels", "sample_size", "_class_name")}
    small = uc["block_out_channels"][0] < 128
    c["conditioning_embedding_out_channels"] = [4, 8] if small else [16, 32, 96, 256]
    if small and len(uc["block_out_channels"]) > 2:
        c["conditioning_embedding_out_channels"] = [4, 8, 8]
    c["_class_name"] = "ControlNetModel"
    torch.manual_seed(seed)
    m = ControlNet(c)
    if zero:
        for conv in list(m.controlnet_down_blocks) + [m.controlnet_mid_block, m.controlnet_cond_embedding.conv_out]:
            torch.nn.init.zeros_(conv.weight)
            torch.nn.init.zeros_(conv.bias)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(c, f)
    save_file({k: v.contiguous() for k, v in m.state_dict().items()},
              os.path.join(out_dir, "diffusion_pytorch_model.safetensors"))
    return out_dir


FLUX_DEV_TRANSFORMER = dict(in_channels=64, num_layers=19, num_single_layers=38, attention_head_dim=128,
                            num_attention_heads=24, joint_attention_dim=4096, pooled_projection_dim=768,
                            guidance_embeds=True, axes_dims_rope=[16, 56, 56], patch_size=1)
FLUX_VAE = dict(SD15_VAE, latent_channels=16, scaling_factor=0.3611, shift_factor=0.1159,
                use_post_quant_conv=False, use_quant_conv=False)
FLUX_SCHEDULER = {"_class_name": "FlowMatchEulerDiscreteScheduler", "base_image_seq_len": 256, "base_shift": 0.5,
                  "max_image_seq_len": 4096, "max_shift": 1.15, "num_train_timesteps": 1000, "shift": 3.0,
                  "use_dynamic_shifting": True}


def _t5_byte_tokenizer(out_dir: str) -> int:
    """A byte-level tokenizer.json for a toy T5 (pad 0, eos 1 appended, unk 2) + its config."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, processors
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))
    cs, n = bs[:], 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    vocab = {"<pad>": 0, "</s>": 1, "<unk>": 2}
    for c in cs:
        vocab[chr(c)] = len(vocab)
    tk = Tokenizer(models.BPE(vocab=vocab, merges=[], unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tk.post_processor = processors.TemplateProcessing(single="$A </s>", special_tokens=[("</s>", 1)])
    os.makedirs(out_dir, exist_ok=True)
    tk.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"pad_token": "<pad>", "eos_token": "</s>", "unk_token": "<unk>",
                   "tokenizer_class": "PreTrainedTokenizerFast"}, f)
    return len(vocab)


def write_flux_pipeline(out_dir: str, size: str = "tiny", seed: int = 0, guidance: bool = True) -> str:
    """Random-init FLUX.1 pipeline directory in the diffusers layout (model_index.json,
    transformer/, text_encoder/ (CLIPTextModel), text_encoder_2/ (T5EncoderModel), tokenizer/,
    tokenizer_2/, vae/ (16-channel KL-VAE), scheduler/).  size="dev": FLUX.1-dev shapes (12 B
    transformer); "tiny": a toy with the same structure."""
    import torch
    import transformers as tf
    from safetensors.torch import save_file

    from .flux import FluxTransformer
    from .sd import VaeDecoder, VaeEncoder
    torch.manual_seed(seed)
    for sub in ("transformer", "vae", "text_encoder", "text_encoder_2", "tokenizer", "tokenizer_2", "scheduler"):
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    vocab = _clip_byte_vocab()
    sp = dict(vocab_size=len(vocab), bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
              pad_token_id=vocab["<|endoftext|>"])
    n_t5 = _t5_byte_tokenizer(os.path.join(out_dir, "tokenizer_2"))
    if size == "dev":
        trc, vc = dict(FLUX_DEV_TRANSFORMER), dict(FLUX_VAE)
        tc = dict(SD15_TEXT, **sp)
        t5c = dict(vocab_size=32128, d_model=4096, d_kv=64, d_ff=10240, num_layers=24, num_heads=64,
                   feed_forward_proj="gated-gelu")
    else:
        tc = dict(SD15_TEXT, hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64, **sp)
        t5c = dict(vocab_size=n_t5, d_model=48, d_kv=8, d_ff=96, num_layers=2, num_heads=4,
                   feed_forward_proj="gated-gelu")
        trc = dict(FLUX_DEV_TRANSFORMER, num_layers=1, num_single_layers=2, attention_head_dim=16,
                   num_attention_heads=2, joint_attention_dim=48, pooled_projection_dim=32, axes_dims_rope=[4, 6, 6])
        vc = dict(FLUX_VAE, block_out_channels=[16, 32], layers_per_block=1, norm_num_groups=8)
    trc["guidance_embeds"] = guidance
    dt = torch.bfloat16 if size == "dev" else torch.float32
    m = FluxTransformer(trc)
    with open(os.path.join(out_dir, "transformer", "config.json"), "w") as f:
        json.dump(dict(trc, _class_name="FluxTransformer2DModel"), f)
    save_file({k: v.to(dt).contiguous() for k, v in m.state_dict().items()},
              os.path.join(out_dir, "transformer", "diffusion_pytorch_model.safetensors"))
    del m
    sd = VaeDecoder(vc).state_dict()
    sd.update(VaeEncoder(vc).state_dict())
    with open(os.path.join(out_dir, "vae", "config.json"), "w") as f:
        json.dump(dict(vc, _class_name="AutoencoderKL"), f)
    save_file({k: v.to(dt).contiguous() for k, v in sd.items()},
              os.path.join(out_dir, "vae", "diffusion_pytorch_model.safetensors"))
    tf.CLIPTextModel(tf.CLIPTextConfig(**tc)).save_pretrained(os.path.join(out_dir, "text_encoder"),
                                                              safe_serialization=True)
    t5 = tf.T5EncoderModel(tf.T5Config(**t5c))
    t5.to(dt).save_pretrained(os.path.join(out_dir, "text_encoder_2"), safe_serialization=True)
    with open(os.path.join(out_dir, "tokenizer", "vocab.json"), "w") as f:
        json.dump(vocab, f)
    with open(os.path.join(out_dir, "tokenizer", "merges.txt"), "w") as f:
        f.write("#version: 0.2\n")
    with open(os.path.join(out_dir, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump(FLUX_SCHEDULER, f)
    with open(os.path.join(out_dir, "model_index.json"), "w") as f:
        json.dump({"_class_name": "FluxPipeline"}, f)
    return out_dir


SD3_TRANSFORMER = dict(sample_size=128, patch_size=2, in_channels=16, num_layers=24, attention_head_dim=64,
                       num_attention_heads=24, joint_attention_dim=4096, caption_projection_dim=1536,
                       pooled_projection_dim=2048, out_channels=16, pos_embed_max_size=192)
SD3_VAE = dict(FLUX_VAE, scaling_factor=1.5305, shift_factor=0.0609)


def write_sd3_pipeline(out_dir: str, seed: int = 0, t5: bool = True) -> str:
    """Random-init toy StableDiffusion3Pipeline directory (diffusers layout: transformer/, vae/,
    text_encoder/ + text_encoder_2/ (CLIPTextModelWithProjection), text_encoder_3/ (T5, optional),
    tokenizer/, tokenizer_2/, tokenizer_3/, scheduler/ (FlowMatch, shift 3))."""
    import torch
    import transformers as tf
    from safetensors.torch import save_file

    from .sd import VaeDecoder, VaeEncoder
    from .sd3 import SD3Transformer
    torch.manual_seed(seed)
    subs = ["transformer", "vae", "text_encoder", "text_encoder_2", "tokenizer", "tokenizer_2", "scheduler"]
    for sub in subs:
        os.makedirs(os.path.join(out_dir, sub), exist_ok=True)
    vocab = _clip_byte_vocab()
    sp = dict(vocab_size=len(vocab), bos_token_id=vocab["<|startoftext|>"], eos_token_id=vocab["<|endoftext|>"],
              pad_token_id=vocab["<|endoftext|>"])
    for sub, hid, nl in (("text_encoder", 32, 2), ("text_encoder_2", 48, 3)):
        c = dict(SD15_TEXT, hidden_size=hid, num_hidden_layers=nl, num_attention_heads=2, intermediate_size=2 * hid,
                 projection_dim=16, hidden_act="gelu", **sp)
        tf.CLIPTextModelWithProjection(tf.CLIPTextConfig(**c)).save_pretrained(os.path.join(out_dir, sub),
                                                                              safe_serialization=True)
    for tk in ("tokenizer", "tokenizer_2"):
        with open(os.path.join(out_dir, tk, "vocab.json"), "w") as f:
            json.dump(vocab, f)
        with open(os.path.join(out_dir, tk, "merges.txt"), "w") as f:
            f.write("#version: 0.2\n")
    if t5:
        n_t5 = _t5_byte_tokenizer(os.path.join(out_dir, "tokenizer_3"))
        tf.T5EncoderModel(tf.T5Config(vocab_size=n_t5, d_model=96, d_kv=8, d_ff=128, num_layers=2, num_heads=4,
                                      feed_forward_proj="gated-gelu")).save_pretrained(
            os.path.join(out_dir, "text_encoder_3"), safe_serialization=True)
    trc = dict(SD3_TRANSFORMER, sample_size=16, num_layers=2, attention_head_dim=16, num_attention_heads=2,
               joint_attention_dim=96, caption_projection_dim=32, pooled_projection_dim=32, pos_embed_max_size=24)
    m = SD3Transformer(trc)
    with open(os.path.join(out_dir, "transformer", "config.json"), "w") as f:
        json.dump(dict(trc, _class_name="SD3Transformer2DModel"), f)
    save_file({k: v.contiguous() for k, v in m.state_dict().items()},
              os.path.join(out_dir, "transformer", "diffusion_pytorch_model.safetensors"))
    vc = dict(SD3_VAE, block_out_channels=[16, 32], layers_per_block=1, norm_num_groups=8)
    sd = VaeDecoder(vc).state_dict()
    sd.update(VaeEncoder(vc).state_dict())
    with open(os.path.join(out_dir, "vae", "config.json"), "w") as f:
        json.dump(dict(vc, _class_name="AutoencoderKL"), f)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(out_dir, "vae", "diffusion_pytorch_model.safetensors"))
    with open(os.path.join(out_dir, "scheduler", "scheduler_config.json"), "w") as f:
        json.dump({"_class_name": "FlowMatchEulerDiscreteScheduler", "num_train_timesteps": 1000, "shift": 3.0}, f)
    with open(os.path.join(out_dir, "model_index.json"), "w") as f:
        json.dump({"_class_name": "StableDiffusion3Pipeline"}, f)
    return out_dir


PIPER_SYMBOLS = "_^$ abcdefghijklmnopqrstuvwxyz',.?!"


def write_piper_voice(path: str, seed: int = 0, sampling_rate: int = 8000):
    """A piper-layout voice (`<name>.onnx` + `<name>.onnx.json`, phoneme_type "text") exported
    from a random-init transformers VitsModel with the noise scales at 0 (deterministic), through
    torch's TorchScript ONNX exporter.  Returns the VitsModel (the test oracle).  The exporter's
    last pass (attaching onnxscript functions) imports the onnx package, which is not installed;
    a graph without such functions leaves that pass a no-op, so it is skipped when onnx is absent."""
    import io

    import torch
    from transformers import VitsConfig, VitsModel
    try:
        import onnx  # noqa: F401
    except ImportError:
        import torch.onnx._internal.torchscript_exporter.onnx_proto_utils as opu
        opu._add_onnxscript_fn = lambda model_bytes, custom_opsets: model_bytes
    cfg = VitsConfig(vocab_size=len(PIPER_SYMBOLS), hidden_size=16, num_hidden_layers=2, num_attention_heads=2,
                     window_size=2, ffn_dim=24, flow_size=8, upsample_initial_channel=16, upsample_rates=[4, 2],
                     upsample_kernel_sizes=[8, 4], resblock_kernel_sizes=[3, 5],
                     resblock_dilation_sizes=[[1, 3], [1, 3]], duration_predictor_filter_channels=12,
                     prior_encoder_num_wavenet_layers=2, sampling_rate=sampling_rate)
    torch.manual_seed(seed)
    m = VitsModel(cfg).eval()
    m.noise_scale = 0.0
    m.noise_scale_duration = 0.0

    class PiperSig(torch.nn.Module):  # piper's graph signature: input, input_lengths, scales
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, input, input_lengths, scales):
            w = self.m(input_ids=input).waveform
            keep = (scales[0] * 0 + 1) * (input_lengths[0] * 0 + 1).to(w.dtype)
            return (w * keep).unsqueeze(1)

    ids = torch.tensor([[1, 0, 10, 0, 2]])
    buf = io.BytesIO()
    with torch.no_grad():
        torch.onnx.export(PiperSig(m).eval(), (ids, torch.tensor([5]), torch.tensor([0.667, 1.0, 0.8])), buf,
                          dynamo=False, opset_version=15, input_names=["input", "input_lengths", "scales"],
                          output_names=["output"], dynamic_axes={"input": {1: "phonemes"}, "output": {2: "time"}})
    m.eval()  # the exporter restores the wrapper's training flag recursively
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(buf.getvalue())
    conf = {"audio": {"sample_rate": sampling_rate, "quality": "x_low"}, "espeak": {"voice": "en-us"},
            "inference": {"noise_scale": 0.667, "length_scale": 1, "noise_w": 0.8}, "phoneme_type": "text",
            "phoneme_map": {}, "phoneme_id_map": {c: [i] for i, c in enumerate(PIPER_SYMBOLS)},
            "num_symbols": len(PIPER_SYMBOLS), "num_speakers": 1, "speaker_id_map": {}, "piper_version": "1.0.0"}
    with open(path + ".json", "w", encoding="utf-8") as f:
        json.dump(conf, f, ensure_ascii=False)
    return m
