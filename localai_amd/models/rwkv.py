"""RWKV-4 recurrent language models: the reference's `rwkv` backend (go-rwkv.cpp,
`backend/go/llm/rwkv/rwkv.go`: the tokenizer file sits next to the model as
`<model>.tokenizer.json` unless `tokenizer` names one; one request at a time; stop word "\\n"
unless the request gives stop words).

Checkpoints: transformers `RwkvForCausalLM` directories (config.json + safetensors / bin) or the
original BlinkDL `.pth` state dict (`emb.weight`, `blocks.N.att.*`, `blocks.N.ffn.*`, loaded with
`torch.load(weights_only=True)`).  rwkv.cpp's own binary container is not read.

Per layer (x in fp32): time-mix attention -- token shift against the previous token's
LayerNorm output, k / v / r projections, the WKV recurrence kept in log-sum-exp form
(numerator, denominator, running max) with `time_first` bonus for the current token and
`-exp(time_decay)` decay -- then the channel-mix FFN (squared ReLU, sigmoid receptance gate).
Projections run as bf16 GEMMs on the GPU, the recurrence in fp32.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, List

import torch
import torch.nn.functional as F


def _hf_names(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """BlinkDL names -> transformers names (so one loader reads both)."""
    if "rwkv.embeddings.weight" in sd:
        return sd
    out = {}
    for k, v in sd.items():
        n = k
        n = n.replace("emb.weight", "rwkv.embeddings.weight").replace("ln_out.", "rwkv.ln_out.")
        if n.startswith("blocks."):
            n = "rwkv." + n.replace(".att.", ".attention.").replace(".ffn.", ".feed_forward.")
            n = n.replace("ln0.", "pre_ln.").replace("time_mix_k", "time_mix_key").replace(
                "time_mix_v", "time_mix_value").replace("time_mix_r", "time_mix_receptance")
        out[n] = v
    return out


def is_rwkv_checkpoint(path: str) -> bool:
    if os.path.isdir(path):
        try:
            with open(os.path.join(path, "config.json")) as f:
                c = json.load(f)
        except (OSError, ValueError):
            return False
        return c.get("model_type") == "rwkv" or "RwkvForCausalLM" in (c.get("architectures") or [])
    return path.endswith(".pth") and os.path.isfile(path)


class RwkvLM:
    def __init__(self, path: str, device: str = "cpu", tokenizer: str = ""):
        self.path = path
        self.device = torch.device(device)
        if os.path.isdir(path):
            files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
            sd: Dict[str, torch.Tensor] = {}
            if files:
                from safetensors.torch import load_file
                for fn in files:
                    sd.update(load_file(fn))
            else:
                for fn in sorted(glob.glob(os.path.join(path, "pytorch_model*.bin"))):
                    sd.update(torch.load(fn, map_location="cpu", weights_only=True))
            with open(os.path.join(path, "config.json")) as f:
                cfg = json.load(f)
            self.eps = float(cfg.get("layer_norm_epsilon", 1e-5))
            tok_path = tokenizer or os.path.join(path, "tokenizer.json")
        else:
            sd = torch.load(path, map_location="cpu", weights_only=True)
            self.eps = 1e-5
            # rwkv.go:23-30: `<model file>.tokenizer.json` beside the model unless `tokenizer` is given
            tok_path = os.path.join(os.path.dirname(path), tokenizer) if tokenizer else path + ".tokenizer.json"
        sd = _hf_names(sd)
        dev = self.device
        mm = torch.bfloat16 if dev.type == "cuda" else torch.float32
        self.mm = mm
        f32 = lambda t: t.to(dev, torch.float32).reshape(-1).contiguous()  # noqa: E731
        w = lambda t: t.to(dev, mm).contiguous()  # noqa: E731
        self.emb = sd["rwkv.embeddings.weight"].to(dev, torch.float32)
        self.n_layer = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("rwkv.blocks."))
        self.D = self.emb.shape[1]
        b0 = "rwkv.blocks.0."
        self.pre_ln = (f32(sd[b0 + "pre_ln.weight"]), f32(sd[b0 + "pre_ln.bias"])) if b0 + "pre_ln.weight" in sd else None
        self.layers = []
        for i in range(self.n_layer):
            p = f"rwkv.blocks.{i}."
            a, ff = p + "attention.", p + "feed_forward."
            self.layers.append(dict(
                ln1=(f32(sd[p + "ln1.weight"]), f32(sd[p + "ln1.bias"])),
                ln2=(f32(sd[p + "ln2.weight"]), f32(sd[p + "ln2.bias"])),
                decay=-torch.exp(f32(sd[a + "time_decay"])), first=f32(sd[a + "time_first"]),
                a_mk=f32(sd[a + "time_mix_key"]), a_mv=f32(sd[a + "time_mix_value"]),
                a_mr=f32(sd[a + "time_mix_receptance"]),
                k=w(sd[a + "key.weight"]), v=w(sd[a + "value.weight"]), r=w(sd[a + "receptance.weight"]),
                o=w(sd[a + "output.weight"]),
                f_mk=f32(sd[ff + "time_mix_key"]), f_mr=f32(sd[ff + "time_mix_receptance"]),
                fk=w(sd[ff + "key.weight"]), fr=w(sd[ff + "receptance.weight"]), fv=w(sd[ff + "value.weight"])))
        self.A = self.layers[0]["k"].shape[0]
        self.ln_out = (f32(sd["rwkv.ln_out.weight"]), f32(sd["rwkv.ln_out.bias"]))
        self.head = w(sd["head.weight"])
        self._tok = None
        if os.path.isfile(tok_path):
            from tokenizers import Tokenizer
            self._tok = Tokenizer.from_file(tok_path)
        self.eos_id = 0  # RWKV vocabularies end text with token 0 (<|endoftext|>)

    def tokenize(self, text: str) -> List[int]:
        if self._tok is None:
            raise RuntimeError("rwkv: no tokenizer file next to the model")
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, ids: List[int]) -> str:
        return self._tok.decode(ids, skip_special_tokens=False) if self._tok is not None else ""

    def new_state(self, B: int = 1):
        z = lambda n, v=0.0: torch.full((B, n), v, dtype=torch.float32, device=self.device)  # noqa: E731
        # per layer: previous ln1 output, previous ln2 output, WKV numerator / denominator / running max
        return [[z(self.D), z(self.D), z(self.A), z(self.A), z(self.A, -1e38)] for _ in range(self.n_layer)]

    def _lin(self, x, wt):
        return (x.to(self.mm) @ wt.t()).float()

    @torch.no_grad()
    def step(self, tokens: torch.Tensor, state) -> torch.Tensor:
        """One token for B sequences -> logits [B, V]; state updated in place."""
        D = self.D
        x = self.emb[tokens]
        if self.pre_ln is not None:
            x = F.layer_norm(x, (D,), self.pre_ln[0], self.pre_ln[1], self.eps)
        for ly, st in zip(self.layers, state):
            h = F.layer_norm(x, (D,), ly["ln1"][0], ly["ln1"][1], self.eps)
            prev = st[0]
            k = self._lin(h * ly["a_mk"] + prev * (1 - ly["a_mk"]), ly["k"])
            v = self._lin(h * ly["a_mv"] + prev * (1 - ly["a_mv"]), ly["v"])
            r = torch.sigmoid(self._lin(h * ly["a_mr"] + prev * (1 - ly["a_mr"]), ly["r"]))
            st[0] = h
            num, den, mx = st[2], st[3], st[4]
            m_out = torch.maximum(mx, k + ly["first"])
            e1, e2 = torch.exp(mx - m_out), torch.exp(k + ly["first"] - m_out)
            wkv = (e1 * num + e2 * v) / (e1 * den + e2)
            m_st = torch.maximum(mx + ly["decay"], k)
            e1, e2 = torch.exp(mx + ly["decay"] - m_st), torch.exp(k - m_st)
            st[2], st[3], st[4] = e1 * num + e2 * v, e1 * den + e2, m_st
            x = x + self._lin(r * wkv, ly["o"])
            h = F.layer_norm(x, (D,), ly["ln2"][0], ly["ln2"][1], self.eps)
            prev = st[1]
            fk = torch.square(torch.relu(self._lin(h * ly["f_mk"] + prev * (1 - ly["f_mk"]), ly["fk"])))
            fr = torch.sigmoid(self._lin(h * ly["f_mr"] + prev * (1 - ly["f_mr"]), ly["fr"]))
            st[1] = h
            x = x + fr * self._lin(fk, ly["fv"])
        x = F.layer_norm(x, (D,), self.ln_out[0], self.ln_out[1], self.eps)
        return self._lin(x, self.head)

    @torch.no_grad()
    def prefill(self, ids: List[int], state) -> torch.Tensor:
        """Feed the prompt token by token (batch 1); -> logits [L, V]."""
        out = [self.step(torch.tensor([t], device=self.device), state)[0] for t in ids]
        return torch.stack(out)
