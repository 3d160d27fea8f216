"""Native Bark text-to-audio: the `bark` TTS backend.

Reference behaviour: `backend/python/bark/backend.py:44-60` (text -> `generate_audio` -> wav at
`dst`, `voice` = a history prompt / speaker preset).  Checkpoints in the Hugging Face layout
(`config.json` with semantic / coarse_acoustics / fine_acoustics / codec sub-configs,
`generation_config.json`, `*.safetensors`, BERT `tokenizer.json`, optional
`speaker_embeddings_path.json` -> per-voice .npy/.npz prompts, loaded with allow_pickle=False).

Pipeline, all on the device:
  semantic   causal GPT over [text embeddings + semantic-history embeddings | infer token]
             (257 positions), greedy/sampled semantic tokens until EOS; tokens above the
             semantic vocabulary (except EOS) are suppressed
  coarse     causal GPT over [semantic window | infer | coarse history], sliding windows of
             new tokens alternating between the two coarse codebooks (each restricted to its
             own id range)
  fine       non-causal GPT filling codebooks 2..7 one at a time over 1024-frame windows
             (input = sum of the embeddings of codebooks 0..k)
  codec      EnCodec 24 kHz decoder (models/musicgen.py EncodecDecoder)
Causal stages keep a KV cache, so each new token costs one position.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .musicgen import _ENC, EncodecDecoder, _hp, load_safetensors_dir
from .tts import _fold_weight_norm

_SUB = dict(block_size=1024, input_vocab_size=10048, output_vocab_size=10048, num_layers=12, num_heads=12,
            hidden_size=768, bias=True, n_codes_total=8, n_codes_given=1)
_SEM = dict(eos_token_id=10000, max_new_tokens=768, temperature=1.0, do_sample=False, top_k=None, top_p=None,
            text_encoding_offset=10048, text_pad_token=129595, semantic_infer_token=129599, semantic_vocab_size=10000,
            max_input_semantic_length=256, semantic_rate_hz=49.9, min_eos_p=None)
_COA = dict(temperature=1.0, do_sample=False, top_k=None, top_p=None, coarse_semantic_pad_token=12048,
            coarse_rate_hz=75, n_coarse_codebooks=2, coarse_infer_token=12050, max_coarse_input_length=256,
            max_coarse_history=630, sliding_window_len=60)
_FIN = dict(temperature=1.0, max_fine_history_length=512, max_fine_input_length=1024, n_fine_codebooks=8)


def is_bark_dir(path: str) -> bool:
    try:
        with open(os.path.join(path, "config.json")) as f:
            return json.load(f).get("model_type") == "bark"
    except (OSError, ValueError):
        return False


class _GPT:
    """Bark GPT stack (pre-LN blocks, fused qkv projection, exact-GELU MLP)."""

    def __init__(self, W: Dict[str, torch.Tensor], prefix: str, hp: dict, causal: bool):
        self.W, self.p, self.hp, self.causal = W, prefix, hp, causal
        self.H, self.nh = hp["hidden_size"], hp["num_heads"]
        self.hd = self.H // self.nh
        self.k = self.v = None

    def _ln(self, x, name):
        return F.layer_norm(x, (self.H,), self.W[self.p + name + ".weight"], self.W.get(self.p + name + ".bias"))

    def _lin(self, x, name):
        return F.linear(x, self.W[self.p + name + ".weight"], self.W.get(self.p + name + ".bias"))

    def reset(self, B: int, T: int, device):
        L = self.hp["num_layers"]
        self.k = [torch.zeros(B, self.nh, T, self.hd, device=device) for _ in range(L)]
        self.v = [torch.zeros(B, self.nh, T, self.hd, device=device) for _ in range(L)]

    def __call__(self, x: torch.Tensor, pos0: int = 0, cache: bool = False) -> torch.Tensor:
        """x [B, T, H] (embeddings, positions added here) -> final-LN hidden [B, T, H]."""
        B, T, H = x.shape
        x = x + self.W[self.p + "position_embeds_layer.weight"][pos0:pos0 + T]
        S = pos0 + T
        if self.causal:
            qi = torch.arange(pos0, S, device=x.device)[:, None]
            mask = torch.arange(S, device=x.device)[None, :] > qi            # future keys
        for i in range(self.hp["num_layers"]):
            b = f"layers.{i}."
            h = self._ln(x, b + "layernorm_1")
            q, k, v = self._lin(h, b + "attn.att_proj").split(H, -1)
            sh = lambda t: t.view(B, T, self.nh, self.hd).transpose(1, 2)  # noqa: E731
            q, k, v = sh(q), sh(k), sh(v)
            if cache:
                self.k[i][:, :, pos0:S] = k
                self.v[i][:, :, pos0:S] = v
                k, v = self.k[i][:, :, :S], self.v[i][:, :, :S]
            s = (q @ k.transpose(-1, -2)) * (1.0 / math.sqrt(self.hd))
            if self.causal:
                s = s.masked_fill(mask, torch.finfo(s.dtype).min)
            a = torch.softmax(s, -1) @ v
            x = x + self._lin(a.transpose(1, 2).reshape(B, T, H), b + "attn.out_proj")
            h = self._ln(x, b + "layernorm_2")
            x = x + self._lin(F.gelu(self._lin(h, b + "mlp.in_proj")), b + "mlp.out_proj")
        return self._ln(x, "layernorm_final")


def _pick(logits: torch.Tensor, cfg: dict, gen: Optional[torch.Generator]) -> torch.Tensor:
    """logits [B, V] (already masked) -> token ids [B]: argmax, or temperature/top-k/top-p sampling."""
    if not cfg.get("do_sample"):
        return logits.argmax(-1)
    lg = torch.log_softmax(logits.float(), -1) / max(float(cfg.get("temperature") or 1.0), 1e-5)
    k = cfg.get("top_k")
    if k:
        kth = torch.topk(lg, min(int(k), lg.shape[-1]), -1).values[:, -1:]
        lg = lg.masked_fill(lg < kth, float("-inf"))
    p = cfg.get("top_p")
    if p is not None and p < 1.0:
        srt, idx = torch.sort(lg, descending=False)
        cum = torch.softmax(srt, -1).cumsum(-1)
        drop = cum <= (1 - p)
        drop[:, -1] = False
        lg = lg.masked_fill(torch.zeros_like(drop).scatter(1, idx, drop), float("-inf"))
    return torch.multinomial(torch.softmax(lg, -1), 1, generator=gen)[:, 0]


class Bark:
    def __init__(self, path: str, device: str = "cpu"):
        with open(os.path.join(path, "config.json")) as f:
            cfg = json.load(f)
        self.path = path
        self.device = torch.device(device)
        sd = _fold_weight_norm(load_safetensors_dir(path))
        self.W = {k: v.float().to(self.device) for k, v in sd.items()}
        self.sem_hp = _hp(_SUB, cfg.get("semantic_config"))
        self.coa_hp = _hp(_SUB, cfg.get("coarse_acoustics_config"))
        self.fin_hp = _hp(_SUB, cfg.get("fine_acoustics_config"))
        gc = {}
        gp = os.path.join(path, "generation_config.json")
        if os.path.exists(gp):
            with open(gp) as f:
                gc = json.load(f)
        self.sem = _hp(_SEM, gc.get("semantic_config"))
        self.coa = _hp(_COA, gc.get("coarse_acoustics_config"))
        self.fin = _hp(_FIN, gc.get("fine_acoustics_config"))
        self.codebook_size = int(gc.get("codebook_size", 1024))
        self.sampling_rate = int(gc.get("sample_rate", 24000))
        # fine heads tied to the next codebook's embedding when the checkpoint stores only one copy
        for j in range(self.fin_hp["n_codes_total"] - self.fin_hp["n_codes_given"]):
            k = f"fine_acoustics.lm_heads.{j}.weight"
            if k not in self.W:
                self.W[k] = self.W[f"fine_acoustics.input_embeds_layers.{j + 1}.weight"]
        self.semantic = _GPT(self.W, "semantic.", self.sem_hp, True)
        self.coarse = _GPT(self.W, "coarse_acoustics.", self.coa_hp, True)
        self.fine = _GPT(self.W, "fine_acoustics.", self.fin_hp, False)
        self.codec = EncodecDecoder(self.W, _hp(_ENC, cfg.get("codec_config")), self.device, prefix="codec_model.")
        self.tokenizer = None
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            from tokenizers import Tokenizer
            self.tokenizer = Tokenizer.from_file(tj)
        self.voices: Dict[str, dict] = {}
        vp = os.path.join(path, "speaker_embeddings_path.json")
        if os.path.exists(vp):
            with open(vp) as f:
                self.voices = json.load(f)

    # ------------------------------------------------------------------ voices / text
    def history(self, voice: str) -> Optional[Dict[str, torch.Tensor]]:
        """A speaker preset: a name from speaker_embeddings_path.json or a path to an .npz holding
        semantic_prompt / coarse_prompt / fine_prompt (numeric arrays; never unpickled)."""
        if not voice:
            return None
        out = {}
        if voice in self.voices:
            ent = self.voices[voice]
            for key in ("semantic_prompt", "coarse_prompt", "fine_prompt"):
                p = ent[key]
                p = p if os.path.isabs(p) else os.path.join(self.path, self.voices.get("repo_or_path", ""), p)
                out[key] = np.load(p, allow_pickle=False)
        elif os.path.exists(voice):
            with np.load(voice, allow_pickle=False) as z:
                out = {k: z[k] for k in ("semantic_prompt", "coarse_prompt", "fine_prompt")}
        else:
            raise ValueError(f"unknown Bark voice {voice!r}")
        return {k: torch.as_tensor(np.asarray(v, dtype=np.int64), device=self.device) for k, v in out.items()}

    def tokenize(self, text: str) -> List[int]:
        if self.tokenizer is None:
            raise RuntimeError("the checkpoint has no tokenizer.json")
        return self.tokenizer.encode(text, add_special_tokens=False).ids

    # ------------------------------------------------------------------ stages
    @torch.no_grad()
    def semantic_tokens(self, ids: List[int], hist=None, max_new_tokens: Optional[int] = None,
                        gen: Optional[torch.Generator] = None) -> torch.Tensor:
        c, E = self.sem, self.W["semantic.input_embeds_layer.weight"]
        n = c["max_input_semantic_length"]
        ids = ids[:n]
        t = torch.full((n,), c["text_pad_token"], dtype=torch.long, device=self.device)
        if ids:
            t[:len(ids)] = torch.tensor(ids, device=self.device) + c["text_encoding_offset"]
        h = torch.full((n,), c["eos_token_id"], dtype=torch.long, device=self.device)
        if hist is not None:
            sp = hist["semantic_prompt"][-n:]
            h[:len(sp)] = sp
        x = torch.cat([E[t] + E[h], E[c["semantic_infer_token"]][None]], 0)[None]   # [1, n+1, H]
        eos = c["eos_token_id"]
        V = self.sem_hp["output_vocab_size"]
        allow = torch.zeros(V, dtype=torch.bool, device=self.device)
        allow[:c["semantic_vocab_size"]] = True
        allow[eos] = True
        steps = int(max_new_tokens or c["max_new_tokens"])
        self.semantic.reset(1, n + 1 + steps, self.device)
        out = []
        pos = 0
        for _ in range(steps):
            hs = self.semantic(x, pos, cache=True)
            pos += x.shape[1]
            lg = self.W["semantic.lm_head.weight"] @ hs[0, -1]
            lg = lg.masked_fill(~allow, float("-inf"))[None]
            if c["min_eos_p"]:
                if torch.softmax(lg.float(), -1)[0, eos] > c["min_eos_p"]:
                    lg = torch.full_like(lg, float("-inf")).index_fill(1, torch.tensor([eos], device=self.device), 0.0)
            tok = int(_pick(lg, c, gen)[0])
            out.append(tok)
            if tok == eos:
                break
            x = E[tok][None, None]
        return torch.tensor(out, dtype=torch.long, device=self.device)

    @torch.no_grad()
    def coarse_tokens(self, sem: torch.Tensor, hist=None, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        s, c = self.sem, self.coa
        cb = self.codebook_size
        sem = sem.clone()
        sem[sem == s["eos_token_id"]] = c["coarse_semantic_pad_token"]
        ratio = c["coarse_rate_hz"] / s["semantic_rate_hz"] * c["n_coarse_codebooks"]
        max_sem_hist = int(np.floor(c["max_coarse_history"] / ratio))
        n_valid = int((sem != c["coarse_semantic_pad_token"]).sum())
        total_len = int(round(np.floor(n_valid * ratio / c["n_coarse_codebooks"]) * c["n_coarse_codebooks"]))
        if hist is not None:
            xs = hist["semantic_prompt"]
            xc = hist["coarse_prompt"].clone()
            for k in range(1, xc.shape[0]):
                xc[k] += cb * k
            xc = xc.t().reshape(-1) + s["semantic_vocab_size"]
            n_sem = min(max_sem_hist, xs.shape[0] - xs.shape[0] % 2, int(np.floor(xc.shape[0] / ratio)))
            n_coa = int(round(n_sem * ratio))
            xs, xc = xs[-n_sem:], xc[-n_coa:][:-2]                          # (a 0 keeps all, as the reference)
        else:
            xs = torch.zeros(0, dtype=torch.long, device=self.device)
            xc = torch.zeros(0, dtype=torch.long, device=self.device)
        base = xs.shape[0]
        sem = torch.cat([xs, sem])
        n_hist = xc.shape[0]
        E = self.W["coarse_acoustics.input_embeds_layer.weight"]
        V = self.coa_hp["output_vocab_size"]
        sv = s["semantic_vocab_size"]
        ar = torch.arange(V, device=self.device)
        first = ~((ar >= sv) & (ar < sv + cb))                               # even steps: codebook 0 ids
        second = ar < sv + cb                                                # odd steps: codebook 1 ids
        generated = 0
        for _ in range(int(np.ceil(total_len / c["sliding_window_len"]))):
            idx = base + int(round(generated / ratio))
            win = sem[max(0, idx - max_sem_hist):][:c["max_coarse_input_length"]]
            win = F.pad(win, (0, c["max_coarse_input_length"] - win.shape[0]), value=c["coarse_semantic_pad_token"])
            prompt = torch.cat([win, torch.tensor([c["coarse_infer_token"]], device=self.device),
                                xc[-c["max_coarse_history"]:]])
            new = min(c["sliding_window_len"], total_len - generated)
            self.coarse.reset(1, prompt.shape[0] + new, self.device)
            x = E[prompt][None]
            pos = 0
            toks = []
            for j in range(new):
                hs = self.coarse(x, pos, cache=True)
                pos += x.shape[1]
                lg = self.W["coarse_acoustics.lm_head.weight"] @ hs[0, -1]
                lg = lg.masked_fill(first if j % 2 == 0 else second, float("-inf"))[None]
                tok = int(_pick(lg, c, gen)[0])
                toks.append(tok)
                x = E[tok][None, None]
            xc = torch.cat([xc, torch.tensor(toks, dtype=torch.long, device=self.device)])
            generated = xc.shape[0] - n_hist
        return xc[n_hist:]

    @torch.no_grad()
    def fine_tokens(self, coarse: torch.Tensor, hist=None, gen: Optional[torch.Generator] = None) -> torch.Tensor:
        s, c, f = self.sem, self.coa, self.fin
        cb = self.codebook_size
        nc, nf = c["n_coarse_codebooks"], f["n_fine_codebooks"]
        co = torch.remainder(coarse.view(-1, nc) - s["semantic_vocab_size"], cb)   # [T, nc]
        T = co.shape[0]
        x = F.pad(co, (0, nf - nc), value=cb)                                # [T, nf]
        n_hist = 0
        if hist is not None:
            fh = hist["fine_prompt"].t()[-f["max_fine_history_length"]:]
            x = torch.cat([fh, x], 0)
            n_hist = fh.shape[0]
        L, Hl = f["max_fine_input_length"], f["max_fine_history_length"]
        n_rm = 0
        if x.shape[0] < L:
            n_rm = L - x.shape[0]
            x = F.pad(x, (0, 0, 0, n_rm), value=cb)
        loops = max(0, int(np.ceil((T - (L - n_hist)) / Hl))) + 1
        temp = f["temperature"]
        for o in range(loops):
            st = min(o * Hl, x.shape[0] - L)
            fill = min(n_hist + o * Hl, x.shape[0] - Hl)
            rel = fill - st
            buf = x[st:st + L].clone()
            for k in range(nc, nf):
                emb = sum(self.W[f"fine_acoustics.input_embeds_layers.{i}.weight"][buf[:, i]] for i in range(k + 1))
                hs = self.fine(emb[None])[0]
                lg = (hs @ self.W[f"fine_acoustics.lm_heads.{k - self.fin_hp['n_codes_given']}.weight"].t())[:, :cb]
                if temp is None or temp == 1.0:
                    pred = lg[rel:].argmax(-1)
                else:
                    pr = torch.softmax(lg / temp, -1)[rel:L]
                    pred = torch.multinomial(pr, 1, generator=gen)[:, 0]
                buf[rel:, k] = pred
            x[fill:fill + (L - rel), nc:] = buf[rel:, nc:]
        x = x[n_hist:]
        if n_rm:
            x = x[:-n_rm]
        return x.t()                                                         # [nf, T]

    @torch.no_grad()
    def generate(self, text: str, voice: str = "", seed: Optional[int] = None,
                 semantic_max_new_tokens: Optional[int] = None) -> np.ndarray:
        hist = self.history(voice)
        gen = None
        if self.sem["do_sample"] or self.coa["do_sample"] or self.fin["temperature"] not in (None, 1.0):
            gen = torch.Generator(device=self.device)
            gen.manual_seed(int(seed) if seed is not None else int(torch.randint(0, 2 ** 31 - 1, (1,))))
        sem = self.semantic_tokens(self.tokenize(text), hist, semantic_max_new_tokens, gen)
        co = self.coarse_tokens(sem, hist, gen)
        fi = self.fine_tokens(co, hist, gen)
        return self.codec(fi)[0].float().cpu().numpy()
