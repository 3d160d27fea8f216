"""Hugging Face checkpoint directories (config.json + *.safetensors + tokenizer files) as engine models.

The reference's `vllm` and `transformers` backends load HF checkpoints (`backend/python/vllm/
backend.py:77-110`, `backend/python/transformers/backend.py:70-180`); its llama.cpp backend loads
GGUF.  This engine serves both: `HFCheckpointReader` presents a checkpoint through the same
interface as `gguf.GGUFReader` (`kv` with llama.cpp metadata keys, `tensors` with GGUF names and
raw little-endian payloads), so the decoder, the tokenizer and tensor parallelism need no second
code path.  The mapping is what llama.cpp's `convert_hf_to_gguf.py` does for these families
(behaviour, not code):
  - LlamaForCausalLM / MistralForCausalLM / MixtralForCausalLM -> `llama`: q/k rows permuted from
    HF's rotate-half pairing to the interleaved pairs the llama RoPE uses; Mixtral experts stacked
    into `ffn_{gate,up,down}_exps`; Llama-3.1 `rope_scaling: llama3` becomes `rope_freqs.weight`.
  - Qwen2ForCausalLM -> `qwen2` (NEOX RoPE, no permutation, q/k/v biases).
Weights keep their stored dtype (bf16 / f16 / f32); the engine serves them on its bf16 paths.
Tokenizers: `tokenizer.model` (SentencePiece: pieces, scores, types) or `tokenizer.json`
(byte-level BPE, encoded by the `tokenizers` library from that file); ids and special tokens
from `config.json` / `tokenizer_config.json`, whose `chat_template` serves
`use_tokenizer_template`.
"""
from __future__ import annotations

import glob
import json
import math
import os
from typing import Any, Dict, List, Optional

import numpy as np

from ..gguf import GGMLType, GGUFTensor

ARCH_OF = {"LlamaForCausalLM": "llama", "MistralForCausalLM": "llama", "MixtralForCausalLM": "llama",
           "Qwen2ForCausalLM": "qwen2",
           # sentence-transformers encoders and cross-encoder rerankers (models/bert.py)
           "BertModel": "bert", "BertForMaskedLM": "bert", "BertForSequenceClassification": "bert"}

# token types (llama.cpp / GGUF)
T_NORMAL, T_UNKNOWN, T_CONTROL, T_USER, T_UNUSED, T_BYTE = 1, 2, 3, 4, 5, 6


def is_hf_checkpoint(path: str) -> bool:
    return os.path.isdir(path) and os.path.isfile(os.path.join(path, "config.json")) and bool(
        glob.glob(os.path.join(path, "*.safetensors")))


def hf_architecture(path: str) -> str:
    """Engine architecture name of an HF checkpoint directory ("" when unknown)."""
    try:
        with open(os.path.join(path, "config.json")) as f:
            archs = json.load(f).get("architectures") or []
    except (OSError, ValueError):
        return ""
    return ARCH_OF.get(archs[0], "") if archs else ""


# `quantization` of the transformers backend (backend/python/transformers/backend.py:93-106:
# bitsandbytes nf4 / int8, XPU 4 / 8 bit) -> the GGML block formats the engine's HIP GEMMs read
# directly: the checkpoint's linear weights are quantised once at load (llama.cpp's Q4_K_M recipe
# for the 4-bit modes: Q4_K projections, Q6_K for the output head and ffn_down / attn_v; Q8_0 for
# the 8-bit modes).  Same memory class and the same load-time semantics as bnb (quantise on load,
# compute in bf16); the numbers are the GGML formats', not bnb's.
QUANT_MODES = {"bnb_4bit": "q4_k_m", "xpu_4bit": "q4_k_m", "q4_k_m": "q4_k_m", "q4_k": "q4_k_m",
               "bnb_8bit": "q8_0", "xpu_8bit": "q8_0", "q8_0": "q8_0"}


def open_model(path: str, quantization: str = ""):
    """GGUF file, HF checkpoint directory or pre-GGUF ggjt v3 file -> reader with the GGUFReader
    interface.  `quantization`: load-time quantisation of an HF checkpoint (QUANT_MODES)."""
    if is_hf_checkpoint(path):
        return HFCheckpointReader(path, quantization=quantization)
    from .ggml_legacy import GGJTReader, is_ggjt
    if is_ggjt(path):
        return GGJTReader(path)
    from ..gguf import GGUFReader
    return GGUFReader(path)


def _permute_rope(w: np.ndarray, n_head: int) -> np.ndarray:
    """HF q/k rows [n_head * hd, ...] in rotate-half order -> interleaved (x0, x1) pairs per head."""
    hd = w.shape[0] // n_head
    return w.reshape(n_head, 2, hd // 2, *w.shape[1:]).swapaxes(1, 2).reshape(w.shape)


def _llama3_rope_freqs(rs: dict, head_dim: int, theta: float) -> np.ndarray:
    """Per-frequency divisors for `rope_scaling: {rope_type: llama3}` (what llama.cpp stores as
    rope_freqs.weight): long wavelengths divided by `factor`, short ones kept, smooth between."""
    factor = float(rs.get("factor", 8.0))
    lo, hi = float(rs.get("low_freq_factor", 1.0)), float(rs.get("high_freq_factor", 4.0))
    old = float(rs.get("original_max_position_embeddings", 8192))
    lo_wl, hi_wl = old / lo, old / hi
    out = []
    for i in range(0, head_dim, 2):
        freq = 1.0 / (theta ** (i / head_dim))
        wl = 2 * math.pi / freq
        if wl < hi_wl:
            out.append(1.0)
        elif wl > lo_wl:
            out.append(factor)
        else:
            smooth = (old / wl - lo) / (hi - lo)
            out.append(1.0 / ((1 - smooth) / factor + smooth))
    return np.asarray(out, dtype=np.float32)


class HFCheckpointReader:
    def __init__(self, path: str, quantization: str = ""):
        self.path = path
        q = (quantization or "").lower()
        if q and q not in QUANT_MODES:
            raise ValueError(f"quantization {quantization!r} is not supported; one of {', '.join(sorted(QUANT_MODES))}")
        self.quant = QUANT_MODES.get(q, "")
        with open(os.path.join(path, "config.json")) as f:
            self.config: Dict[str, Any] = json.load(f)
        archs = self.config.get("architectures") or []
        cls = archs[0] if archs else ""
        if cls not in ARCH_OF:
            raise ValueError(f"{path}: unsupported HF architecture {cls or '(none)'}; "
                             f"supported: {', '.join(sorted(ARCH_OF))}")
        self.hf_class = cls
        self.arch = ARCH_OF[cls]
        self.kv: Dict[str, Any] = {}
        self.tensors: Dict[str, GGUFTensor] = {}
        if self.arch == "bert":
            self._bert()
            return
        self._hparams()
        self._load_tensors()
        self._tokenizer()

    # ---- GGUFReader interface ------------------------------------------------------------
    @property
    def architecture(self) -> str:
        return self.arch

    def get(self, key: str, default=None):
        return self.kv.get(key, default)

    def arch_kv(self, suffix: str, default=None):
        return self.kv.get(f"{self.arch}.{suffix}", default)

    def close(self):
        self.tensors = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- metadata --------------------------------------------------------------------------
    def _hparams(self):
        c, a = self.config, self.arch
        n_embd = int(c["hidden_size"])
        n_head = int(c["num_attention_heads"])
        n_kv = int(c.get("num_key_value_heads") or n_head)
        hd = int(c.get("head_dim") or n_embd // n_head)
        self.n_head, self.n_kv, self.head_dim = n_head, n_kv, hd
        kv = self.kv
        kv["general.architecture"] = a
        kv["general.name"] = str(c.get("_name_or_path") or os.path.basename(os.path.normpath(self.path)))
        kv[f"{a}.context_length"] = int(c.get("max_position_embeddings", 4096))
        kv[f"{a}.embedding_length"] = n_embd
        kv[f"{a}.block_count"] = int(c["num_hidden_layers"])
        kv[f"{a}.feed_forward_length"] = int(c["intermediate_size"])
        kv[f"{a}.attention.head_count"] = n_head
        kv[f"{a}.attention.head_count_kv"] = n_kv
        if hd != n_embd // n_head:
            kv[f"{a}.attention.key_length"] = hd
            kv[f"{a}.attention.value_length"] = hd
        kv[f"{a}.rope.dimension_count"] = hd
        # transformers < 5 writes rope_theta / rope_scaling; 5.x folds both into rope_parameters
        rp = c.get("rope_parameters") or {}
        kv[f"{a}.rope.freq_base"] = float(c.get("rope_theta") or rp.get("rope_theta") or 10000.0)
        kv[f"{a}.attention.layer_norm_rms_epsilon"] = float(c.get("rms_norm_eps", 1e-6))
        kv[f"{a}.vocab_size"] = int(c["vocab_size"])
        if c.get("num_local_experts"):
            kv[f"{a}.expert_count"] = int(c["num_local_experts"])
            kv[f"{a}.expert_used_count"] = int(c.get("num_experts_per_tok", 2))
        rs = c.get("rope_scaling") or (rp if rp.get("rope_type") not in (None, "default") else {})
        rtype = str(rs.get("rope_type") or rs.get("type") or "")
        if rtype in ("linear", "yarn"):
            kv[f"{a}.rope.scaling.type"] = rtype
            kv[f"{a}.rope.scaling.factor"] = float(rs.get("factor", 1.0))
            if rtype == "yarn":
                kv[f"{a}.rope.scaling.original_context_length"] = int(
                    rs.get("original_max_position_embeddings", kv[f"{a}.context_length"]))
        self._rope_freqs = (_llama3_rope_freqs(rs, hd, kv[f"{a}.rope.freq_base"]) if rtype == "llama3" else None)

    # ---- tensors ---------------------------------------------------------------------------
    def _put(self, name: str, arr: np.ndarray, ggml_type: int):
        arr = np.ascontiguousarray(arr)
        data = arr.view(np.uint8).reshape(-1)
        self.tensors[name] = GGUFTensor(name, tuple(int(s) for s in arr.shape), int(ggml_type), 0, data.nbytes, data)

    @staticmethod
    def _np(t) -> tuple:
        """torch tensor -> (numpy array holding its raw bits, ggml type)."""
        import torch
        if t.dtype == torch.bfloat16:
            return t.contiguous().view(torch.int16).numpy().view(np.uint16), GGMLType.BF16
        if t.dtype == torch.float16:
            return t.contiguous().numpy(), GGMLType.F16
        return t.float().contiguous().numpy(), GGMLType.F32

    def _gptq_config(self) -> Optional[dict]:
        q = self.config.get("quantization_config") or self._json("quantize_config.json")
        if not q:
            return None
        if str(q.get("quant_method", "gptq")).lower() != "gptq":
            raise ValueError(f"{self.path}: quantization {q.get('quant_method')} is not supported (GPTQ is)")
        return q

    @staticmethod
    def _gptq_dequant(qweight, qzeros, scales, g_idx, bits: int, v1_zero_offset: bool):
        """GPTQ linear -> float weight [N, K] (torch, fp32).  qweight int32 [K*bits/32, N] packs
        32/bits input rows per word (low bits first); qzeros int32 [G, N*bits/32] packs output
        columns the same way (AutoGPTQ's v1 format stores zero - 1); scales [G, N]; g_idx [K] maps
        each input row to its group (act-order checkpoints permute it)."""
        import torch
        pack, mask = 32 // bits, (1 << bits) - 1
        sh = torch.arange(pack, dtype=torch.int32) * bits
        Kp, N = qweight.shape
        q = ((qweight.unsqueeze(1) >> sh.view(1, pack, 1)) & mask).reshape(Kp * pack, N)        # [K, N]
        G = qzeros.shape[0]
        z = ((qzeros.unsqueeze(2) >> sh.view(1, 1, pack)) & mask).reshape(G, -1)[:, :N]         # [G, N]
        if v1_zero_offset:
            z = z + 1
        gi = g_idx.long()
        w = (q.float() - z[gi].float()) * scales.float()[gi]                                    # [K, N]
        return w.t().contiguous()

    def _load_tensors(self):
        from safetensors import safe_open
        files = sorted(glob.glob(os.path.join(self.path, "*.safetensors")))
        hf: Dict[str, Any] = {}
        for fn in files:
            with safe_open(fn, framework="pt") as f:
                for k in f.keys():
                    hf[k] = f.get_tensor(k)
        gq = self._gptq_config()
        if gq is not None:
            import torch
            bits = int(gq.get("bits", 4))
            if bits not in (2, 4, 8):
                raise ValueError(f"{self.path}: GPTQ bits={bits} not supported")
            gs = int(gq.get("group_size", 128))
            v1 = str(gq.get("checkpoint_format", "gptq")).lower() != "gptq_v2"
            for k in [k for k in hf if k.endswith(".qweight")]:
                base = k[:-len(".qweight")]
                qw = hf.pop(k)
                K = qw.shape[0] * (32 // bits)
                gi = hf.pop(base + ".g_idx", None)
                if gi is None:  # no act-order: consecutive groups of group_size input rows
                    gi = torch.arange(K, dtype=torch.int32) // (gs if gs > 0 else K)
                w = self._gptq_dequant(qw, hf.pop(base + ".qzeros"), hf.pop(base + ".scales"), gi, bits, v1)
                hf[base + ".weight"] = w.to(torch.float16)  # served on the bf16 paths like any f16 weight
        c = self.config
        n_layer = int(c["num_hidden_layers"])
        llama = self.arch == "llama"

        def take(k: str) -> Optional[tuple]:
            t = hf.pop(k, None)
            return None if t is None else self._np(t)

        def put(gname: str, hname: str, permute_heads: int = 0, required: bool = True):
            v = take(hname)
            if v is None:
                if required:
                    raise KeyError(f"{self.path}: missing tensor {hname}")
                return
            arr, t = v
            if permute_heads:
                arr = _permute_rope(arr, permute_heads)
            self._put(gname, arr, t)

        put("token_embd.weight", "model.embed_tokens.weight")
        put("output_norm.weight", "model.norm.weight")
        if not c.get("tie_word_embeddings", False):
            put("output.weight", "lm_head.weight", required=False)
        for i in range(n_layer):
            p, b = f"model.layers.{i}.", f"blk.{i}."
            put(b + "attn_norm.weight", p + "input_layernorm.weight")
            put(b + "ffn_norm.weight", p + "post_attention_layernorm.weight")
            put(b + "attn_q.weight", p + "self_attn.q_proj.weight", self.n_head if llama else 0)
            put(b + "attn_k.weight", p + "self_attn.k_proj.weight", self.n_kv if llama else 0)
            put(b + "attn_v.weight", p + "self_attn.v_proj.weight")
            put(b + "attn_output.weight", p + "self_attn.o_proj.weight")
            for nm, hn, ph in (("attn_q", "q_proj", self.n_head), ("attn_k", "k_proj", self.n_kv), ("attn_v", "v_proj", 0)):
                put(b + nm + ".bias", p + f"self_attn.{hn}.bias", ph if (llama and ph) else 0, required=False)
            if c.get("num_local_experts"):
                E = int(c["num_local_experts"])
                put(b + "ffn_gate_inp.weight", p + "block_sparse_moe.gate.weight")
                for gname, w in (("ffn_gate_exps", "w1"), ("ffn_up_exps", "w3"), ("ffn_down_exps", "w2")):
                    parts = [take(p + f"block_sparse_moe.experts.{e}.{w}.weight") for e in range(E)]
                    if any(x is None for x in parts):
                        raise KeyError(f"{self.path}: missing experts for {p}{w}")
                    self._put(b + gname + ".weight", np.stack([x[0] for x in parts]), parts[0][1])
            else:
                put(b + "ffn_gate.weight", p + "mlp.gate_proj.weight")
                put(b + "ffn_up.weight", p + "mlp.up_proj.weight")
                put(b + "ffn_down.weight", p + "mlp.down_proj.weight")
        if self._rope_freqs is not None:
            self._put("rope_freqs.weight", self._rope_freqs, GGMLType.F32)
        if self.quant:
            self._quantize_weights()
        rest = [k for k in hf if not k.endswith("rotary_emb.inv_freq")]
        if rest:
            raise ValueError(f"{self.path}: unmapped tensors {rest[:5]}")

    _QUANT_TARGETS = ("attn_q.weight", "attn_k.weight", "attn_v.weight", "attn_output.weight", "ffn_gate.weight",
                      "ffn_up.weight", "ffn_down.weight", "ffn_gate_exps.weight", "ffn_up_exps.weight",
                      "ffn_down_exps.weight", "output.weight")

    def _quantize_weights(self):
        """Linear weights -> Q4_K_M mix or Q8_0 (QUANT_MODES); norms, embeddings, biases stay."""
        from ..gguf import quantize
        for name, t in list(self.tensors.items()):
            if not name.endswith(self._QUANT_TARGETS):
                continue
            K = t.shape[-1]
            if self.quant == "q8_0":
                gt = GGMLType.Q8_0 if K % 32 == 0 else None
            else:
                six = name.endswith(("output.weight", "ffn_down.weight", "ffn_down_exps.weight", "attn_v.weight")) \
                    and not name.endswith("attn_output.weight")
                gt = (GGMLType.Q6_K if six else GGMLType.Q4_K) if K % 256 == 0 else \
                    (GGMLType.Q8_0 if K % 32 == 0 else None)
            if gt is None:
                continue
            src = {GGMLType.BF16: lambda d: (d.view(np.uint16).astype(np.uint32) << 16).view(np.float32),
                   GGMLType.F16: lambda d: d.view(np.float16).astype(np.float32),
                   GGMLType.F32: lambda d: d.view(np.float32)}[GGMLType(t.ggml_type)](t.data)
            q = quantize(src.reshape(t.shape), gt)
            self.tensors[name] = GGUFTensor(name, t.shape, int(gt), 0, q.nbytes, q)

    # ---- tokenizer -------------------------------------------------------------------------
    def _json(self, name: str) -> dict:
        p = os.path.join(self.path, name)
        if not os.path.isfile(p):
            return {}
        with open(p) as f:
            return json.load(f)

    def _tokenizer(self):
        kv, c = self.kv, self.config
        tcfg = self._json("tokenizer_config.json")
        gcfg = self._json("generation_config.json")
        spm = os.path.join(self.path, "tokenizer.model")
        tj = os.path.join(self.path, "tokenizer.json")
        n_vocab = int(c["vocab_size"])
        if os.path.isfile(spm):
            import sentencepiece as sp_mod
            sp = sp_mod.SentencePieceProcessor(model_file=spm)
            tokens, scores, types = [], [], []
            for i in range(sp.get_piece_size()):
                tokens.append(sp.id_to_piece(i))
                scores.append(float(sp.get_score(i)))
                types.append(T_UNKNOWN if sp.is_unknown(i) else T_CONTROL if sp.is_control(i)
                             else T_UNUSED if sp.is_unused(i) else T_BYTE if sp.is_byte(i) else T_NORMAL)
            for tok in self._added_tokens(tcfg, tj):  # added tokens beyond the SPM model
                if tok["id"] >= len(tokens):
                    while len(tokens) < tok["id"]:
                        tokens.append(f"[PAD{len(tokens)}]"), scores.append(-1000.0), types.append(T_UNUSED)
                    tokens.append(tok["content"]), scores.append(0.0)
                    types.append(T_CONTROL if tok.get("special") else T_USER)
            kv["tokenizer.ggml.model"] = "llama"
            kv["tokenizer.ggml.scores"] = scores
            kv["tokenizer.ggml.add_space_prefix"] = True
        elif os.path.isfile(tj):
            doc = self._json("tokenizer.json")
            model = doc.get("model") or {}
            if model.get("type") != "BPE":
                raise ValueError(f"{self.path}: tokenizer.json model {model.get('type')} is not supported")
            vocab = model.get("vocab") or {}
            size = max([n_vocab] + [i + 1 for i in vocab.values()] + [t["id"] + 1 for t in doc.get("added_tokens", [])])
            tokens = [f"[PAD{i}]" for i in range(size)]
            types = [T_UNUSED] * size
            for s, i in vocab.items():
                tokens[i], types[i] = s, T_NORMAL
            for t in doc.get("added_tokens", []):
                tokens[t["id"]] = t["content"]
                types[t["id"]] = T_CONTROL if t.get("special") else T_USER
            merges = [m if isinstance(m, str) else " ".join(m) for m in model.get("merges") or []]
            kv["tokenizer.ggml.model"] = "gpt2"
            kv["tokenizer.ggml.merges"] = merges
            kv["tokenizer.ggml.pre"] = "hf-json"
            kv["tokenizer.hf.json"] = tj  # encode with the checkpoint's own pre-tokenizer / model
        else:
            raise ValueError(f"{self.path}: no tokenizer.model or tokenizer.json")
        kv["tokenizer.ggml.tokens"] = tokens
        kv["tokenizer.ggml.token_type"] = types

        def tok_id(v):
            if isinstance(v, list):
                return int(v[0]) if v else None
            return None if v is None else int(v)

        def special_id(name):
            t = tcfg.get(name)
            if isinstance(t, dict):
                t = t.get("content")
            if isinstance(t, str) and t in tokens:
                return tokens.index(t)
            return None
        bos = tok_id(c.get("bos_token_id", gcfg.get("bos_token_id")))
        eos_raw = gcfg.get("eos_token_id", c.get("eos_token_id"))
        eos = tok_id(eos_raw)
        if bos is None:
            bos = special_id("bos_token")
        if eos is None:
            eos = special_id("eos_token")
        if bos is not None:
            kv["tokenizer.ggml.bos_token_id"] = bos
        if eos is not None:
            kv["tokenizer.ggml.eos_token_id"] = eos
        if isinstance(eos_raw, list) and len(eos_raw) > 1:
            kv["tokenizer.ggml.eot_token_id"] = int(eos_raw[1])
        add_bos = tcfg.get("add_bos_token")
        if add_bos is None:  # Llama-3 style: the post-processor template inserts BOS
            post = json.dumps(self._json("tokenizer.json").get("post_processor") or {}) if os.path.isfile(tj) else ""
            bos_tok = tokens[bos] if bos is not None and 0 <= bos < len(tokens) else None
            add_bos = bool(bos_tok and bos_tok in post)
        kv["tokenizer.ggml.add_bos_token"] = bool(add_bos)
        if tcfg.get("chat_template"):
            tpl = tcfg["chat_template"]
            if isinstance(tpl, list):  # named templates: take "default"
                tpl = next((t.get("template") for t in tpl if t.get("name") == "default"), tpl[0].get("template"))
            kv["tokenizer.chat_template"] = tpl

    def _added_tokens(self, tcfg: dict, tj: str) -> List[dict]:
        if os.path.isfile(tj):
            return sorted(self._json("tokenizer.json").get("added_tokens", []), key=lambda t: t["id"])
        out = []
        for i, t in (tcfg.get("added_tokens_decoder") or {}).items():
            out.append({"id": int(i), "content": t.get("content", ""), "special": t.get("special", False)})
        return sorted(out, key=lambda t: t["id"])

    # ---- BERT encoders (sentence-transformers / cross-encoders) ---------------------------
    def _bert(self):
        """BertModel / BertForSequenceClassification -> the `bert` layout models/bert.py reads
        (llama.cpp's bert GGUF names): post-LN encoder, WordPiece vocab with word-initial pieces
        marked by U+2581 and "##" continuations bare, pooling from sentence-transformers'
        1_Pooling/config.json (CLS or mean), RANK pooling plus the `cls.*` head for a
        single-logit sequence classifier (a cross-encoder reranker)."""
        from safetensors import safe_open
        c, kv = self.config, self.kv
        hf: Dict[str, Any] = {}
        for fn in sorted(glob.glob(os.path.join(self.path, "*.safetensors"))):
            with safe_open(fn, framework="pt") as f:
                for k in f.keys():
                    hf[k[5:] if k.startswith("bert.") else k] = f.get_tensor(k)
        kv["general.architecture"] = "bert"
        kv["general.name"] = os.path.basename(os.path.normpath(self.path))
        kv["bert.context_length"] = int(c.get("max_position_embeddings", 512))
        kv["bert.embedding_length"] = int(c["hidden_size"])
        kv["bert.feed_forward_length"] = int(c["intermediate_size"])
        kv["bert.block_count"] = int(c["num_hidden_layers"])
        kv["bert.attention.head_count"] = int(c["num_attention_heads"])
        kv["bert.attention.layer_norm_epsilon"] = float(c.get("layer_norm_eps", 1e-12))
        kv["bert.attention.causal"] = False
        ranker = self.hf_class == "BertForSequenceClassification"
        pool = 1
        pc = self._json(os.path.join("1_Pooling", "config.json"))
        if pc.get("pooling_mode_cls_token"):
            pool = 2
        kv["bert.pooling_type"] = 4 if ranker else pool

        def put(gname, hname, required=True):
            t = hf.pop(hname, None)
            if t is None:
                if required:
                    raise KeyError(f"{self.path}: missing tensor {hname}")
                return
            arr, ty = self._np(t)
            self._put(gname, arr, ty)
        put("token_embd.weight", "embeddings.word_embeddings.weight")
        put("token_types.weight", "embeddings.token_type_embeddings.weight", required=False)
        put("position_embd.weight", "embeddings.position_embeddings.weight")
        put("token_embd_norm.weight", "embeddings.LayerNorm.weight")
        put("token_embd_norm.bias", "embeddings.LayerNorm.bias")
        for i in range(int(c["num_hidden_layers"])):
            p, b = f"encoder.layer.{i}.", f"blk.{i}."
            for g, h in (("attn_q", "attention.self.query"), ("attn_k", "attention.self.key"),
                         ("attn_v", "attention.self.value"), ("attn_output", "attention.output.dense"),
                         ("attn_output_norm", "attention.output.LayerNorm"), ("ffn_up", "intermediate.dense"),
                         ("ffn_down", "output.dense"), ("layer_output_norm", "output.LayerNorm")):
                put(b + g + ".weight", p + h + ".weight")
                put(b + g + ".bias", p + h + ".bias")
        if ranker:
            put("cls.weight", "pooler.dense.weight")
            put("cls.bias", "pooler.dense.bias")
            put("cls.output.weight", "classifier.weight")
            put("cls.output.bias", "classifier.bias")
        # vocabulary: vocab.txt (one piece per line) or tokenizer.json's WordPiece vocab
        vt = os.path.join(self.path, "vocab.txt")
        if os.path.isfile(vt):
            with open(vt, encoding="utf-8") as f:
                pieces = [ln.rstrip("\n") for ln in f]
        else:
            model = (self._json("tokenizer.json").get("model") or {})
            if model.get("type") != "WordPiece":
                raise ValueError(f"{self.path}: no vocab.txt and no WordPiece tokenizer.json")
            voc = model["vocab"]
            pieces = [""] * (max(voc.values()) + 1)
            for t, i in voc.items():
                pieces[i] = t
        toks, types = [], []
        for t in pieces:
            if t.startswith("[") and t.endswith("]"):
                toks.append(t)
                types.append(T_CONTROL)
            elif t.startswith("##"):
                toks.append(t[2:])
                types.append(T_NORMAL)
            else:
                toks.append("\u2581" + t)
                types.append(T_NORMAL)
        kv["tokenizer.ggml.model"] = "bert"
        kv["tokenizer.ggml.tokens"] = toks
        kv["tokenizer.ggml.token_type"] = types
        for key, name in (("unknown_token_id", "[UNK]"), ("cls_token_id", "[CLS]"), ("seperator_token_id", "[SEP]"),
                          ("padding_token_id", "[PAD]")):
            if name in toks:
                kv[f"tokenizer.ggml.{key}"] = toks.index(name)
