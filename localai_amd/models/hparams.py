"""Model hyper-parameters read from GGUF metadata (llama.cpp's llm_load_hparams equivalent)."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional


@dataclass
class HParams:
    arch: str
    n_layer: int
    n_embd: int
    n_head: int
    n_head_kv: int
    head_dim: int
    n_ff: int
    n_vocab: int
    n_ctx_train: int = 4096
    rope_theta: float = 10000.0
    rope_dim: int = 0                 # rotary dims (partial rotary for phi-2)
    rope_mode: int = 0                # 0 = NORM (llama), 1 = NEOX (phi2, qwen2, ...)
    rope_scaling: str = "none"
    rope_freq_scale: float = 1.0
    rope_orig_ctx: int = 0
    norm_eps: float = 1e-5
    norm_type: str = "rms"            # "rms" | "layer"
    n_expert: int = 0
    n_expert_used: int = 0
    moe_renorm: bool = True           # renormalise the top-k routing weights (Mixtral); Qwen2-MoE does not
    n_ff_shexp: int = 0               # Qwen2-MoE shared expert width (0: none)
    # DeepSeek-V2 multi-head latent attention + fine-grained MoE
    kv_lora_rank: int = 0             # MLA: compressed kv width (0: regular attention)
    q_lora_rank: int = 0              # MLA: compressed q width (0: one q projection, V2-Lite)
    head_dim_v: int = 0               # MLA: value head width (keys: head_dim = nope + rope dims)
    n_ff_exp: int = 0                 # routed / shared expert width when it differs from n_ff
    n_layer_dense_lead: int = 0       # leading layers with a dense FFN instead of experts
    expert_weights_scale: float = 1.0
    yarn_log_mul: float = 0.0         # DeepSeek-V2: query scale mscale = 1 + yarn_log_mul * ln(factor)
    parallel_residual: bool = False   # phi-2: h = x + attn(ln x) + mlp(ln x)
    act: str = "swiglu"               # "swiglu" | "gelu" | "geglu" (Gemma: gelu(gate) * up)
    embed_scale: float = 1.0          # Gemma scales the token embeddings by sqrt(n_embd)
    attn_softcap: float = 0.0         # Gemma-2: scores -> cap * tanh(scores / cap)
    final_softcap: float = 0.0        # Gemma-2: logits -> cap * tanh(logits / cap)
    sliding_window: int = 0           # Gemma-2: even layers attend to the last `sliding_window` keys
    attn_scale: float = 0.0           # query scale override (0: 1/sqrt(head_dim))
    logit_scale: float = 1.0          # Command-R multiplies the logits (0.0625)
    tied_embeddings: bool = False
    name: str = ""

    @property
    def q_dim(self) -> int:
        return self.n_head * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_head_kv * self.head_dim

    @staticmethod
    def from_gguf(r) -> "HParams":
        a = r.architecture
        g = lambda k, d=None: r.kv.get(f"{a}.{k}", d)  # noqa: E731
        n_embd = int(g("embedding_length"))
        n_head = int(g("attention.head_count"))
        n_head_kv = int(g("attention.head_count_kv", n_head))
        head_dim = int(g("attention.key_length", n_embd // n_head))
        tokens = r.kv.get("tokenizer.ggml.tokens") or []
        n_vocab = int(g("vocab_size", len(tokens)))
        if "token_embd.weight" in r.tensors:
            n_vocab = r.tensors["token_embd.weight"].shape[0]
        rope_dim = int(g("rope.dimension_count", head_dim))
        neox_archs = {"phi2", "phi3", "qwen2", "qwen2moe", "gptneox", "stablelm", "gemma", "gemma2", "falcon",
                      "starcoder2"}
        eps = g("attention.layer_norm_rms_epsilon")
        norm_type = "rms"
        if eps is None:
            eps = g("attention.layer_norm_epsilon", 1e-5)
            norm_type = "layer"
        n_ff = g("feed_forward_length")
        if isinstance(n_ff, list):
            n_ff = n_ff[0]
        if a == "qwen2moe":  # the routed experts' width; no dense FFN
            n_ff = g("expert_feed_forward_length", n_ff)
        ds2 = a == "deepseek2"
        if ds2:
            # DeepSeek-V3 / R1 GGUFs also say arch deepseek2 but route with sigmoid gating, a
            # selection bias (exp_probs_b) and normalised weights; the fused router implements
            # V2's softmax routing only, so refuse those instead of routing experts wrongly
            gating = int(g("expert_gating_func", 1) or 1)   # llama.cpp: 1 = softmax, 2 = sigmoid
            if gating != 1 or bool(g("expert_weights_norm", False)):
                raise ValueError("deepseek2 GGUF with sigmoid expert gating / normalised expert weights "
                                 "(DeepSeek-V3/R1 routing) is not supported; only DeepSeek-V2 softmax routing")
        hp = HParams(
            arch=a,
            n_layer=int(g("block_count")),
            n_embd=n_embd,
            n_head=n_head,
            n_head_kv=n_head_kv,
            head_dim=head_dim,
            n_ff=int(n_ff),
            n_vocab=n_vocab,
            n_ctx_train=int(g("context_length", 4096)),
            rope_theta=float(g("rope.freq_base", 10000.0)),
            rope_dim=rope_dim,
            rope_mode=1 if a in neox_archs else 0,
            rope_scaling=str(g("rope.scaling.type", "none")),
            rope_freq_scale=1.0 / float(g("rope.scaling.factor", 1.0) or 1.0),
            rope_orig_ctx=int(g("rope.scaling.original_context_length", 0) or 0),
            norm_eps=float(eps),
            norm_type=norm_type,
            n_expert=int(g("expert_count", 0) or 0),
            n_expert_used=int(g("expert_used_count", 0) or 0),
            moe_renorm=a not in ("qwen2moe", "deepseek2"),
            n_ff_shexp=int(g("expert_shared_feed_forward_length", 0) or 0) if a == "qwen2moe" else 0,
            kv_lora_rank=int(g("attention.kv_lora_rank", 0) or 0) if ds2 else 0,
            q_lora_rank=int(g("attention.q_lora_rank", 0) or 0) if ds2 else 0,
            head_dim_v=int(g("attention.value_length", head_dim) or head_dim) if ds2 else 0,
            n_ff_exp=int(g("expert_feed_forward_length", 0) or 0) if ds2 else 0,
            n_layer_dense_lead=int(g("leading_dense_block_count", 0) or 0) if ds2 else 0,
            expert_weights_scale=float(g("expert_weights_scale", 1.0) or 1.0) if ds2 else 1.0,
            yarn_log_mul=float(g("rope.scaling.yarn_log_multiplier", 0.0) or 0.0) if ds2 else 0.0,
            # phi-2 / Command-R: h = x + attn(ln x) + mlp(ln x)
            parallel_residual=a in ("phi2", "command-r"),
            act="gelu" if a in ("phi2", "gptneox", "falcon", "starcoder2")
            else ("geglu" if a in ("gemma", "gemma2") else "swiglu"),
            logit_scale=float(g("logit_scale", 1.0) or 1.0),
            embed_scale=float(n_embd) ** 0.5 if a in ("gemma", "gemma2") else 1.0,
            attn_softcap=float(g("attn_logit_softcapping", 0.0) or 0.0) if a == "gemma2" else 0.0,
            final_softcap=float(g("final_logit_softcapping", 0.0) or 0.0) if a == "gemma2" else 0.0,
            sliding_window=int(g("attention.sliding_window", 0) or 0) if a == "gemma2" else 0,
            # Gemma-2 27B scales queries by 1/sqrt(n_embd / n_head) (query_pre_attn_scalar 144), not
            # 1/sqrt(head_dim) (llama.cpp build_gemma2)
            attn_scale=(float(n_embd // n_head) ** -0.5
                        if a == "gemma2" and int(g("block_count")) == 46 else 0.0),
            tied_embeddings="output.weight" not in r.tensors,
            name=str(r.kv.get("general.name", "")),
        )
        if ds2:
            hp.n_ff_shexp = hp.n_ff_exp * int(g("expert_shared_count", 0) or 0)
            if hp.rope_scaling == "yarn" and hp.rope_freq_scale < 1.0:
                # llama.cpp build_deepseek2: kq_scale = mscale^2 / sqrt(head_dim_k)
                import math
                ms = 1.0 + hp.yarn_log_mul * math.log(1.0 / hp.rope_freq_scale)
                hp.attn_scale = ms * ms / math.sqrt(hp.head_dim)
        return hp
