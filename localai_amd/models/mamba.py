"""Mamba selective state-space language models: the reference's `mamba` backend
(`backend/python/mamba/backend.py`: mamba_ssm's MambaLMHeadModel, one request at a time,
MAMBA_CHAT eos `<|endoftext|>`, default max tokens 2000, top_p 0.9 when unset).

Checkpoints: transformers `MambaForCausalLM` directories (config.json with hidden_size /
state_size / conv_kernel / expand / time_step_rank, `backbone.embeddings`) and mamba_ssm
directories (config.json with d_model / n_layer / ssm_cfg, `backbone.embedding`, weights in
safetensors or a `pytorch_model.bin` read with `torch.load(weights_only=True)`); tokenizer from the
directory's tokenizer.json.

Per layer: RMSNorm -> in_proj -> (x, z); x -> causal depthwise conv (kernel K) -> SiLU -> x_proj ->
(dt, B, C); dt -> dt_proj -> softplus; h_t = exp(dt A) h_{t-1} + dt B x_t; y = <h_t, C> + D x;
y *= SiLU(z) -> out_proj; residual in fp32.  The prompt is scanned in one pass over its tokens
(per-token state updates vectorised over channels and states); decode is one recurrent step per
token with the conv window and SSM state kept per request -- on the GPU the conv roll and the
state update are the two HIP kernels of `ops/csrc/mamba.hip`, the projections are library GEMMs.
"""
from __future__ import annotations

import glob
import json
import math
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F


def is_mamba_checkpoint(path: str) -> bool:
    cfg = os.path.join(path, "config.json")
    if not (os.path.isdir(path) and os.path.isfile(cfg)):
        return False
    try:
        with open(cfg) as f:
            c = json.load(f)
    except (OSError, ValueError):
        return False
    archs = c.get("architectures") or []
    return c.get("model_type") == "mamba" or "MambaForCausalLM" in archs or "ssm_cfg" in c


def _load_state_dict(path: str) -> Dict[str, torch.Tensor]:
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    sd: Dict[str, torch.Tensor] = {}
    if files:
        from safetensors.torch import load_file
        for fn in files:
            sd.update(load_file(fn))
        return sd
    bins = sorted(glob.glob(os.path.join(path, "pytorch_model*.bin")))
    if not bins:
        raise FileNotFoundError(f"{path}: no *.safetensors or pytorch_model.bin")
    for fn in bins:
        sd.update(torch.load(fn, map_location="cpu", weights_only=True))  # tensors only, no pickled code
    return sd


class MambaLM:
    def __init__(self, path: str, device: str = "cpu"):
        self.path = path
        self.device = torch.device(device)
        with open(os.path.join(path, "config.json")) as f:
            c = json.load(f)
        if "d_model" in c:  # mamba_ssm layout
            ssm = c.get("ssm_cfg") or {}
            self.D = int(c["d_model"])
            self.n_layer = int(c["n_layer"])
            self.N = int(ssm.get("d_state", 16))
            self.K = int(ssm.get("d_conv", 4))
            self.I = int(ssm.get("expand", 2)) * self.D
            dtr = ssm.get("dt_rank", "auto")
            self.eps = 1e-5
        else:  # transformers MambaConfig
            self.D = int(c["hidden_size"])
            self.n_layer = int(c["num_hidden_layers"])
            self.N = int(c.get("state_size", 16))
            self.K = int(c.get("conv_kernel", 4))
            self.I = int(c.get("intermediate_size") or int(c.get("expand", 2)) * self.D)
            dtr = c.get("time_step_rank", "auto")
            self.eps = float(c.get("layer_norm_epsilon", 1e-5))
        self.R = math.ceil(self.D / 16) if dtr in (None, "auto") else int(dtr)
        sd = _load_state_dict(path)
        emb = sd.get("backbone.embeddings.weight", sd.get("backbone.embedding.weight"))
        if emb is None:
            raise KeyError(f"{path}: no backbone embedding")
        dev, mm = self.device, torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.mm = mm
        f32 = lambda t: t.to(dev, torch.float32).contiguous()  # noqa: E731
        w = lambda t: t.to(dev, mm).contiguous()  # noqa: E731
        self.emb = f32(emb)
        self.vocab = self.emb.shape[0]
        self.norm_f = f32(sd["backbone.norm_f.weight"])
        self.lm_head = w(sd.get("lm_head.weight", emb))
        self.layers = []
        for i in range(self.n_layer):
            p = f"backbone.layers.{i}."
            m = p + "mixer."
            conv_w = sd[m + "conv1d.weight"]  # [I, 1, K]
            self.layers.append(dict(
                norm=f32(sd[p + "norm.weight"]),
                in_proj=w(sd[m + "in_proj.weight"]),
                in_b=f32(sd[m + "in_proj.bias"]) if m + "in_proj.bias" in sd else None,
                conv_w=f32(conv_w.reshape(self.I, self.K)),
                conv_b=f32(sd[m + "conv1d.bias"]) if m + "conv1d.bias" in sd else None,
                x_proj=w(sd[m + "x_proj.weight"]),
                dt_proj=w(sd[m + "dt_proj.weight"]), dt_b=f32(sd[m + "dt_proj.bias"]),
                A=f32(-torch.exp(sd[m + "A_log"].float())), Dp=f32(sd[m + "D"]),
                out_proj=w(sd[m + "out_proj.weight"]),
                out_b=f32(sd[m + "out_proj.bias"]) if m + "out_proj.bias" in sd else None))
        del sd
        self._tok = None
        tj = os.path.join(path, "tokenizer.json")
        if os.path.isfile(tj):
            from tokenizers import Tokenizer
            self._tok = Tokenizer.from_file(tj)
        tc = {}
        if os.path.isfile(os.path.join(path, "tokenizer_config.json")):
            with open(os.path.join(path, "tokenizer_config.json")) as f:
                tc = json.load(f)
        eos = os.environ.get("MAMBA_EOS") or ("<|endoftext|>" if os.environ.get("MAMBA_CHAT", "1") == "1"
                                                 else tc.get("eos_token"))
        if isinstance(eos, dict):
            eos = eos.get("content")
        self.eos_id = self._tok.token_to_id(eos) if (self._tok is not None and eos) else None
        if self.eos_id is None:
            self.eos_id = c.get("eos_token_id")

    # ---- tokenizer ---------------------------------------------------------------------------
    def tokenize(self, text: str) -> List[int]:
        if self._tok is None:
            raise RuntimeError("mamba: checkpoint has no tokenizer.json")
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, ids: List[int]) -> str:
        return self._tok.decode(ids, skip_special_tokens=False) if self._tok is not None else ""

    # ---- model ----------------------------------------------------------------------------
    def _lin(self, x: torch.Tensor, wt: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
        y = (x.to(self.mm) @ wt.t()).float()
        return y + b if b is not None else y

    def _rms(self, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps) * w

    def new_state(self, B: int = 1) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        return [(z(B, self.I, self.K), z(B, self.I, self.N)) for _ in range(self.n_layer)]

    @torch.no_grad()
    def prefill(self, ids: List[int], state) -> torch.Tensor:
        """Scan the prompt (batch 1) from `state` (updated in place); -> logits [L, V] fp32."""
        L, I, K, N, R = len(ids), self.I, self.K, self.N, self.R
        h = self.emb[torch.tensor(ids, device=self.device)]                      # [L, D] fp32 residual
        for ly, (cs, ss) in zip(self.layers, state):
            xz = self._lin(self._rms(h, ly["norm"]), ly["in_proj"], ly["in_b"])    # [L, 2I]
            x, z = xz[:, :I], xz[:, I:]
            win = torch.cat([cs[0].t(), x], 0)                                    # [K + L, I] (K history rows)
            xc = F.conv1d(win.t().unsqueeze(0), ly["conv_w"].unsqueeze(1), ly["conv_b"], groups=I)[0, :, 1:].t()
            cs[0].copy_(win[-K:].t())
            xc = F.silu(xc)                                                       # [L, I]
            dbc = self._lin(xc, ly["x_proj"])                                     # [L, R + 2N]
            dt = F.softplus(self._lin(dbc[:, :R], ly["dt_proj"], ly["dt_b"]))     # [L, I]
            Bm, Cm = dbc[:, R:R + N], dbc[:, R + N:]
            dA = torch.exp(dt.unsqueeze(-1) * ly["A"])                            # [L, I, N]
            dBx = (dt * xc).unsqueeze(-1) * Bm.unsqueeze(1)                       # [L, I, N]
            hs = ss[0]
            ys = torch.empty(L, I, dtype=torch.float32, device=self.device)
            for t in range(L):
                hs = dA[t] * hs + dBx[t]
                ys[t] = hs @ Cm[t]
            ss[0].copy_(hs)
            y = (ys + xc * ly["Dp"]) * F.silu(z)
            h = h + self._lin(y, ly["out_proj"], ly["out_b"])
        return self._lin(self._rms(h, self.norm_f), self.lm_head)

    @torch.no_grad()
    def step(self, tokens: torch.Tensor, state) -> torch.Tensor:
        """One recurrent step for B sequences: tokens [B] -> logits [B, V]; state updated in place."""
        I, N, R = self.I, self.N, self.R
        h = self.emb[tokens]
        gpu = self.device.type == "cuda"
        if gpu:
            from .. import ops
        for ly, (cs, ss) in zip(self.layers, state):
            xz = self._lin(self._rms(h, ly["norm"]), ly["in_proj"], ly["in_b"]).contiguous()
            if gpu:
                xc = ops.mamba_conv_step(cs, xz, ly["conv_w"], ly["conv_b"], torch.empty_like(xz[:, :I]))
            else:
                cs.copy_(torch.cat([cs[:, :, 1:], xz[:, :I].unsqueeze(-1)], -1))
                xc = (cs * ly["conv_w"]).sum(-1)
                if ly["conv_b"] is not None:
                    xc = xc + ly["conv_b"]
                xc = F.silu(xc)
            dbc = self._lin(xc, ly["x_proj"]).contiguous()
            dt = self._lin(dbc[:, :R], ly["dt_proj"], ly["dt_b"]).contiguous()
            if gpu:
                y = ops.mamba_ssm_step(ss, xc, dt, dbc, R, R + N, ly["A"], ly["Dp"], xz, torch.empty_like(xc))
            else:
                d = F.softplus(dt)
                hs = torch.exp(d.unsqueeze(-1) * ly["A"]) * ss + (d * xc).unsqueeze(-1) * dbc[:, R:R + N].unsqueeze(1)
                ss.copy_(hs)
                y = ((hs * dbc[:, R + N:].unsqueeze(1)).sum(-1) + xc * ly["Dp"]) * F.silu(xz[:, I:])
            h = h + self._lin(y, ly["out_proj"], ly["out_b"])
        return self._lin(self._rms(h, self.norm_f), self.lm_head)


def sample(logits: torch.Tensor, temperature: float, top_p: float, top_k: int, gen: torch.Generator) -> int:
    """Greedy at temperature <= 0; else temperature, top-k, top-p (nucleus) sampling."""
    if temperature <= 0:
        return int(logits.argmax())
    lg = logits.float() / temperature
    if top_k > 0:
        kth = torch.topk(lg, min(top_k, lg.numel())).values[-1]
        lg = lg.masked_fill(lg < kth, -math.inf)
    p = torch.softmax(lg, -1)
    if 0 < top_p < 1:
        sp, si = torch.sort(p, descending=True)
        keep = torch.cumsum(sp, 0) - sp < top_p
        p = torch.zeros_like(p).scatter_(0, si[keep], sp[keep])
        p = p / p.sum()
    return int(torch.multinomial(p.cpu(), 1, generator=gen))
