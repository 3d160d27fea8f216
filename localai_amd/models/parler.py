"""Native Parler-TTS: the `parler-tts` TTS backend.

Reference behaviour: `backend/python/parler-tts/backend.py:71-90` -- the request's `voice` is a
natural-language *description* of the speaker (a fixed default description when empty), tokenised
into `input_ids` for the text encoder; the request's `text` is tokenised into `prompt_input_ids`;
`model.generate(input_ids=..., prompt_input_ids=...)` with the checkpoint's generation config, and
the waveform is written to `dst` at the audio codec's sampling rate.

Checkpoints in the Hugging Face layout of `parler_tts.ParlerTTSForConditionalGeneration`
(`config.json` model_type "parler_tts" with text_encoder / audio_encoder / decoder sub-configs,
`*.safetensors`, `tokenizer.json`, `generation_config.json`):

  description encoder  T5 encoder (shared with models/musicgen.py), projected to the decoder width
                       by `enc_to_dec_proj` when the widths differ; its cross-attention K/V are
                       computed once per request
  prompt               `embed_prompts` token embeddings PREPENDED to the decoder's input sequence:
                       the decoder sees [prompt tokens | audio frames] under one causal mask with
                       sinusoidal positions counted from the first prompt token
  decoder              MusicGen-style pre-LN transformer over the sum of the K codebook embeddings,
                       grouped-query self-attention (`num_key_value_heads`), K linear heads
  delay pattern        codebook k lags codebook 0 by k steps: the upper-left triangle is forced to
                       the BOS id, the lower-right one (relative to the length budget) to PAD; a
                       codebook that emits EOS stays on PAD; generation stops when every codebook
                       has finished.  Frames holding any id >= codebook_size are dropped before
                       decoding, as ParlerTTSForConditionalGeneration.generate does
  DAC codec            residual-VQ codebook lookups + 1x1 out-projections summed -> DAC decoder
                       (conv k7, upsampling blocks of Snake + transposed conv + three dilated
                       residual units (1, 3, 9), Snake, conv k7, tanh).  Weights in either the
                       `descript-audio-codec` package layout (`audio_encoder.model.decoder.model.N`,
                       weight-normalised) or the transformers DacModel layout

On a GPU the decoder runs in bf16 and each per-frame step (all layers, static KV buffers with a
position mask) is one captured hipGraph replay; sampling (temperature / top-k / multinomial with a
seeded generator, `min_new_tokens` EOS suppression) runs on the device beside it and the host reads
the "all codebooks finished" flag once every 16 frames.
"""
from __future__ import annotations

import json
import math
import os
import re
from collections import OrderedDict
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .musicgen import T5Encoder, _hp, _T5, load_safetensors_dir
from .tts import _fold_weight_norm

DEFAULT_DESCRIPTION = ("A female speaker with a slightly low-pitched voice delivers her words quite expressively, "
                       "in a very confined sounding environment with clear audio quality. She speaks very fast.")

_DEC = dict(vocab_size=1088, max_position_embeddings=4096, num_hidden_layers=24, ffn_dim=4096, num_attention_heads=16,
            num_key_value_heads=None, num_cross_attention_key_value_heads=None, activation_function="gelu",
            hidden_size=1024, scale_embedding=False, num_codebooks=9, pad_token_id=1024, bos_token_id=1025,
            eos_token_id=1024, rope_embeddings=False, layer_norm_eps=1e-5)
_GEN = dict(do_sample=True, temperature=1.0, top_k=50, max_length=2580, min_new_tokens=0,
            decoder_start_token_id=None, bos_token_id=None, pad_token_id=None, eos_token_id=None)


def is_parler_dir(path: str) -> bool:
    try:
        with open(os.path.join(path, "config.json")) as f:
            return json.load(f).get("model_type") == "parler_tts"
    except (OSError, ValueError):
        return False


def dac_weights(sd: Dict[str, torch.Tensor], prefix: str) -> Dict[str, torch.Tensor]:
    """The DAC codec's tensors under `prefix`, weight norm folded, renamed to the transformers
    DacModel layout (`quantizer.quantizers.i.*`, `decoder.conv1`, `decoder.block.b.{snake1,conv_t1,
    res_unitJ.{snake1,conv1,snake2,conv2}}`, `decoder.snake1`, `decoder.conv2`).  The
    descript-audio-codec layout (`[model.]decoder.model.N...`) is mapped onto it."""
    sub = _fold_weight_norm({k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)})
    if any(k.startswith("model.") for k in sub):
        sub = {k[len("model."):]: v for k, v in sub.items() if k.startswith("model.")}
    if not any(k.startswith("decoder.model.") for k in sub):
        return sub
    nb = len({m.group(1) for k in sub for m in [re.match(r"decoder\.model\.(\d+)\.block\.1\.weight$", k)] if m})
    out = {}
    for k, v in sub.items():
        m = re.match(r"decoder\.model\.(\d+)\.(.*)$", k)
        if not m:
            out[k] = v
            continue
        i, rest = int(m.group(1)), m.group(2)
        if i == 0:
            out["decoder.conv1." + rest] = v
        elif i <= nb:
            b = f"decoder.block.{i - 1}."
            r = re.match(r"block\.(\d+)\.(.*)$", rest)
            j, tail = int(r.group(1)), r.group(2)
            if j == 0:
                out[b + "snake1." + tail] = v
            elif j == 1:
                out[b + "conv_t1." + tail] = v
            else:
                u = re.match(r"block\.(\d+)\.(.*)$", tail)
                name = ("snake1", "conv1", "snake2", "conv2")[int(u.group(1))]
                out[b + f"res_unit{j - 1}.{name}.{u.group(2)}"] = v
        elif i == nb + 1:
            out["decoder.snake1." + rest] = v
        else:
            out["decoder.conv2." + rest] = v
    return out


def _snake(x: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    return x + (alpha + 1e-9).reciprocal() * torch.sin(alpha * x).pow(2)


class DacDecoder:
    """Codes [Q, T] -> waveform [samples] (DAC residual-VQ sum + decoder)."""

    def __init__(self, W: Dict[str, torch.Tensor], device):
        self.W = {k: v.float().to(device) for k, v in W.items()}
        self.nq = len({k.split(".")[2] for k in W if k.startswith("quantizer.quantizers.")})
        self.nb = len({k.split(".")[2] for k in W if k.startswith("decoder.block.")})
        # transposed conv kernel = 2 * stride
        self.strides = [self.W[f"decoder.block.{b}.conv_t1.weight"].shape[-1] // 2 for b in range(self.nb)]
        self.hop = int(np.prod(self.strides)) if self.strides else 1

    def latents(self, codes: torch.Tensor) -> torch.Tensor:
        W = self.W
        z = 0
        for q in range(codes.shape[0]):
            p = f"quantizer.quantizers.{q}."
            e = W[p + "codebook.weight"][codes[q]]                            # [T, d]
            z = z + e @ W[p + "out_proj.weight"][:, :, 0].t() + W[p + "out_proj.bias"]
        return z.t()[None]                                                   # [1, D, T]

    @torch.no_grad()
    def __call__(self, codes: torch.Tensor) -> torch.Tensor:
        W = self.W
        x = F.conv1d(self.latents(codes), W["decoder.conv1.weight"], W["decoder.conv1.bias"], padding=3)
        for b, s in enumerate(self.strides):
            p = f"decoder.block.{b}."
            x = _snake(x, W[p + "snake1.alpha"])
            x = F.conv_transpose1d(x, W[p + "conv_t1.weight"], W[p + "conv_t1.bias"], stride=s,
                                   padding=math.ceil(s / 2))
            for j, dil in ((1, 1), (2, 3), (3, 9)):
                r = f"{p}res_unit{j}."
                y = F.conv1d(_snake(x, W[r + "snake1.alpha"]), W[r + "conv1.weight"], W[r + "conv1.bias"],
                             dilation=dil, padding=3 * dil)
                y = F.conv1d(_snake(y, W[r + "snake2.alpha"]), W[r + "conv2.weight"], W[r + "conv2.bias"])
                crop = (x.shape[-1] - y.shape[-1]) // 2
                x = (x[..., crop:x.shape[-1] - crop] if crop > 0 else x) + y
        x = _snake(x, W["decoder.snake1.alpha"])
        x = torch.tanh(F.conv1d(x, W["decoder.conv2.weight"], W["decoder.conv2.bias"], padding=3))
        return x[0, 0]


class _Graph:
    """One captured decode step for a (length budget, description length) shape."""

    def __init__(self):
        self.graph = None
        self.tok = self.pos = self.ck = self.cv = self.kc = self.vc = self.logits = None


class ParlerTTS:
    def __init__(self, path: str, device: str = "cpu", use_graphs: Optional[bool] = None):
        with open(os.path.join(path, "config.json")) as f:
            cfg = json.load(f)
        if cfg.get("prompt_cross_attention"):
            raise ValueError("prompt_cross_attention checkpoints are not supported (the prompt must be prepended)")
        self.dec = _hp(_DEC, cfg.get("decoder"))
        if self.dec["rope_embeddings"]:
            raise ValueError("rotary-position Parler decoders are not supported (sinusoidal positions only)")
        self.t5 = _hp(_T5, cfg.get("text_encoder"))
        ac = cfg.get("audio_encoder") or {}
        self.sampling_rate = int(ac.get("sampling_rate", 44100))
        self.codebook_size = int(ac.get("codebook_size", 1024))
        self.device = torch.device(device)
        self.dt = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        sd = load_safetensors_dir(path)
        self.codec = DacDecoder(dac_weights(sd, "audio_encoder."), self.device)
        sd = {k: v for k, v in sd.items() if not k.startswith("audio_encoder.")}
        self.Wt = {k: v.float().to(self.device) for k, v in sd.items() if k.startswith("text_encoder.")}
        self.text = T5Encoder(self.Wt, self.t5)
        self.W = {k: v.to(self.device, self.dt) for k, v in sd.items() if not k.startswith("text_encoder.")}
        self.tokenizer = None
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            from tokenizers import Tokenizer
            self.tokenizer = Tokenizer.from_file(tj)
        gc = dict(_GEN)
        gp = os.path.join(path, "generation_config.json")
        if os.path.exists(gp):
            with open(gp) as f:
                gc.update({k: v for k, v in json.load(f).items() if k in _GEN and v is not None})
        self.gen = gc
        d = self.dec
        self.bos = int(gc["decoder_start_token_id"] or gc["bos_token_id"] or d["bos_token_id"])
        self.pad = int(gc["pad_token_id"] if gc["pad_token_id"] is not None else d["pad_token_id"])
        eos = gc["eos_token_id"] if gc["eos_token_id"] is not None else d["eos_token_id"]
        self.eos = int(eos[0] if isinstance(eos, list) else eos)
        H, nh = d["hidden_size"], d["num_attention_heads"]
        self.hd = H // nh
        self.nkv = int(d["num_key_value_heads"] or nh)
        self.nkv_x = int(d["num_cross_attention_key_value_heads"] or self.nkv)
        K = d["num_codebooks"]
        self._emb = torch.stack([self.W[f"decoder.model.decoder.embed_tokens.{k}.weight"] for k in range(K)])
        self._heads = torch.stack([self.W[f"decoder.lm_heads.{k}.weight"] for k in range(K)])  # [K, V, H]
        half = H // 2
        f = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000) / (half - 1)))
        self._freq = f.to(self.device)
        self.use_graphs = (self.device.type == "cuda") if use_graphs is None else use_graphs
        self._graphs: "OrderedDict[tuple, _Graph]" = OrderedDict()

    # ------------------------------------------------------------------ inputs
    def tokenize(self, text: str) -> torch.Tensor:
        if self.tokenizer is None:
            raise RuntimeError("the checkpoint has no tokenizer.json")
        return torch.tensor([self.tokenizer.encode(text).ids], device=self.device)

    def _positions(self, n: int) -> torch.Tensor:
        t = torch.arange(n, device=self.device, dtype=torch.float32)[:, None] * self._freq[None]
        e = torch.cat([torch.cos(t), torch.sin(t)], 1)
        if self.dec["hidden_size"] % 2:
            e = F.pad(e, (0, 1))
        return e.to(self.dt)

    def encode_description(self, ids: torch.Tensor) -> torch.Tensor:
        h = self.text(ids)[0]
        if "enc_to_dec_proj.weight" in self.W:
            h = F.linear(h.to(self.dt), self.W["enc_to_dec_proj.weight"], self.W["enc_to_dec_proj.bias"])
        return h.to(self.dt)                                                 # [S, H]

    def _cross_kv(self, enc: torch.Tensor):
        d, W, hd = self.dec, self.W, self.hd
        ck, cv = [], []
        for i in range(d["num_hidden_layers"]):
            pp = f"decoder.model.decoder.layers.{i}.encoder_attn."
            ck.append((enc @ W[pp + "k_proj.weight"].t()).view(-1, self.nkv_x, hd).transpose(0, 1))
            cv.append((enc @ W[pp + "v_proj.weight"].t()).view(-1, self.nkv_x, hd).transpose(0, 1))
        return torch.stack(ck), torch.stack(cv)                              # [layers, nkv, S, hd]

    # ------------------------------------------------------------------ decoder
    def _ln(self, x, name):
        return F.layer_norm(x, (x.shape[-1],), self.W[name + ".weight"], self.W[name + ".bias"], self.dec["layer_norm_eps"])

    def _attend(self, q, k, v, mask):
        """q [nh, T, hd], k/v [nkv, L, hd] (grouped), mask [T, L] additive."""
        nh = q.shape[0]
        g = nh // k.shape[0]
        if g > 1:
            k, v = k.repeat_interleave(g, 0), v.repeat_interleave(g, 0)
        s = (q @ k.transpose(-1, -2)).float() * self.hd ** -0.5
        if mask is not None:
            s = s + mask
        return (torch.softmax(s, -1).to(v.dtype) @ v)

    def _layers(self, x, kc, vc, ck, cv, self_mask, pos_idx):
        """x [T, H] at sequence rows pos_idx (tensor [T]); kc/vc [layers, nkv, L, hd] written at those rows."""
        d, W, hd, nh = self.dec, self.W, self.hd, self.dec["num_attention_heads"]
        T, H = x.shape
        act = F.gelu if d["activation_function"] == "gelu" else F.relu
        for i in range(d["num_hidden_layers"]):
            pp = f"decoder.model.decoder.layers.{i}."
            h = self._ln(x, pp + "self_attn_layer_norm")
            q = (h @ W[pp + "self_attn.q_proj.weight"].t()).view(T, nh, hd).transpose(0, 1)
            kc[i].index_copy_(1, pos_idx, (h @ W[pp + "self_attn.k_proj.weight"].t()).view(T, self.nkv, hd).transpose(0, 1))
            vc[i].index_copy_(1, pos_idx, (h @ W[pp + "self_attn.v_proj.weight"].t()).view(T, self.nkv, hd).transpose(0, 1))
            a = self._attend(q, kc[i], vc[i], self_mask)
            x = x + a.transpose(0, 1).reshape(T, H) @ W[pp + "self_attn.out_proj.weight"].t()
            h = self._ln(x, pp + "encoder_attn_layer_norm")
            q = (h @ W[pp + "encoder_attn.q_proj.weight"].t()).view(T, nh, hd).transpose(0, 1)
            a = self._attend(q, ck[i], cv[i], None)
            x = x + a.transpose(0, 1).reshape(T, H) @ W[pp + "encoder_attn.out_proj.weight"].t()
            h = self._ln(x, pp + "final_layer_norm")
            x = x + act(h @ W[pp + "fc1.weight"].t()) @ W[pp + "fc2.weight"].t()
        x = self._ln(x, "decoder.model.decoder.layer_norm")
        return torch.einsum("th,kvh->tkv", x, self._heads).float()           # [T, K, V]

    def _embed(self, tok: torch.Tensor) -> torch.Tensor:
        """tok [K] -> summed codebook embedding [1, H]."""
        K = tok.shape[0]
        x = self._emb[torch.arange(K, device=tok.device), tok].sum(0, keepdim=True)
        return x * math.sqrt(self.dec["hidden_size"]) if self.dec["scale_embedding"] else x

    def _step(self, tok, pos, kc, vc, ck, cv, pe):
        """One frame: tok [K] at sequence row pos (tensor [1]) -> logits [K, V]."""
        L = kc.shape[2]
        x = self._embed(tok) + pe.index_select(0, pos)
        mask = torch.where(torch.arange(L, device=pos.device)[None] <= pos[:, None], 0.0, float("-inf"))
        return self._layers(x, kc, vc, ck, cv, mask, pos)[0]

    def _graph_step(self, L, S, ck, cv, pe):
        key = (L, S)
        g = self._graphs.get(key)
        if g is None:
            g = _Graph()
            d = self.dec
            g.tok = torch.full((d["num_codebooks"],), self.bos, dtype=torch.long, device=self.device)
            g.pos = torch.zeros(1, dtype=torch.long, device=self.device)
            g.ck, g.cv = torch.empty_like(ck), torch.empty_like(cv)
            g.pe = pe.clone()
            shp = (d["num_hidden_layers"], self.nkv, L, self.hd)
            g.kc = torch.zeros(shp, dtype=self.dt, device=self.device)
            g.vc = torch.zeros(shp, dtype=self.dt, device=self.device)
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):                                           # warm the allocator / libraries
                    self._step(g.tok, g.pos, g.kc, g.vc, g.ck, g.cv, g.pe)
            torch.cuda.current_stream(self.device).wait_stream(s)
            g.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g.graph):
                g.logits = self._step(g.tok, g.pos, g.kc, g.vc, g.ck, g.cv, g.pe)
            self._graphs[key] = g
            while len(self._graphs) > 4:
                self._graphs.popitem(last=False)
        self._graphs.move_to_end(key)
        g.ck.copy_(ck)
        g.cv.copy_(cv)
        return g

    # ------------------------------------------------------------------ generation
    @torch.no_grad()
    def generate_codes(self, desc_ids: torch.Tensor, prompt_ids: torch.Tensor, max_new_tokens: Optional[int] = None,
                       do_sample: Optional[bool] = None, temperature: Optional[float] = None,
                       top_k: Optional[int] = None, seed: Optional[int] = None, ignore_eos: bool = False):
        """-> (seq [K, 1 + n] with the delay pattern, codes [K, frames] with special frames dropped)."""
        d, gc = self.dec, self.gen
        K, V = d["num_codebooks"], d["vocab_size"]
        do_sample = gc["do_sample"] if do_sample is None else do_sample
        temperature = float(gc["temperature"] if temperature is None else temperature)
        top_k = int(gc["top_k"] if top_k is None else top_k)
        P = prompt_ids.shape[1]
        if max_new_tokens is None:
            max_new_tokens = max(int(gc["max_length"]) - 1, K)
        n = int(max_new_tokens)
        Lseq = n + 1                                                         # audio rows incl. the start row
        L = P + Lseq
        L = -(-L // 64) * 64 if self.use_graphs else L                        # graph shapes in 64-row buckets
        enc = self.encode_description(desc_ids)
        ck, cv = self._cross_kv(enc)
        pe = self._positions(L)
        # delay pattern over seq columns t = 0..n: BOS for t <= k, PAD for t >= n - K + 2 + k
        kk = torch.arange(K, device=self.device)[:, None]
        tt = torch.arange(Lseq, device=self.device)[None, :]
        force_bos = tt <= kk
        force_pad = tt >= (Lseq - K + 1 + kk)
        seq = torch.full((K, Lseq), self.bos, dtype=torch.long, device=self.device)
        gen = None
        if do_sample:
            gen = torch.Generator(device=self.device)
            gen.manual_seed(int(seed) if seed is not None else int(torch.randint(0, 2 ** 31 - 1, (1,))))
        g = self._graph_step(L, ck.shape[2], ck, cv, pe) if self.use_graphs else None
        if g is not None:
            kc, vc = g.kc, g.vc
        else:
            shp = (d["num_hidden_layers"], self.nkv, L, self.hd)
            kc = torch.zeros(shp, dtype=self.dt, device=self.device)
            vc = torch.zeros(shp, dtype=self.dt, device=self.device)
        # prefill: the prompt embeddings + the start frame in one causal pass
        x = torch.cat([self.W["embed_prompts.weight"][prompt_ids[0]], self._embed(seq[:, 0])], 0) + pe[:P + 1]
        rows = torch.arange(P + 1, device=self.device)
        mask = torch.where(torch.arange(L, device=self.device)[None] <= rows[:, None], 0.0, float("-inf"))
        logits = self._layers(x, kc, vc, ck, cv, mask, rows)[-1]          # [K, V]
        finished = torch.zeros(K, dtype=torch.bool, device=self.device)
        min_new = int(gc["min_new_tokens"] or 0)
        steps = 0
        for s in range(Lseq - 1):
            lg = logits.float()
            if s < min_new and not ignore_eos:
                lg[:, self.eos] = float("-inf")
            if do_sample:
                lg = lg / max(temperature, 1e-5)
                if top_k and top_k < V:
                    kth = torch.topk(lg, top_k, -1).values[:, -1:]
                    lg = lg.masked_fill(lg < kth, float("-inf"))
                nxt = torch.multinomial(torch.softmax(lg, -1), 1, generator=gen)[:, 0]
            else:
                nxt = lg.argmax(-1)
            if not ignore_eos:
                nxt = torch.where(finished, torch.full_like(nxt, self.pad), nxt)
            t = s + 1
            nxt = torch.where(force_bos[:, t], torch.full_like(nxt, self.bos),
                              torch.where(force_pad[:, t], torch.full_like(nxt, self.pad), nxt))
            seq[:, t] = nxt
            steps = t
            if not ignore_eos:
                finished |= (nxt == self.eos) & ~force_bos[:, t]
                if t % 16 == 0 and bool(finished.all()):
                    break
            if t == Lseq - 1:
                break
            pos = torch.full((1,), P + t, dtype=torch.long, device=self.device)
            if g is not None:
                g.tok.copy_(nxt)
                g.pos.copy_(pos)
                g.graph.replay()
                logits = g.logits
            else:
                logits = self._step(nxt, pos, kc, vc, ck, cv, pe)
        seq = seq[:, :steps + 1]
        # un-delay: frame f of codebook k sits at column f + k + 1
        nf = seq.shape[1] - K
        if nf <= 0:
            return seq, torch.zeros(K, 0, dtype=torch.long, device=self.device)
        codes = torch.stack([seq[k, k + 1:k + 1 + nf] for k in range(K)])
        keep = (codes < self.codebook_size).all(0)
        return seq, codes[:, keep]

    @torch.no_grad()
    def generate(self, text: str, description: str = "", max_new_tokens: Optional[int] = None,
                 do_sample: Optional[bool] = None, seed: Optional[int] = None) -> np.ndarray:
        """-> float32 mono waveform [samples] at `sampling_rate`."""
        desc = self.tokenize(description or DEFAULT_DESCRIPTION)
        prompt = self.tokenize(text)
        _, codes = self.generate_codes(desc, prompt, max_new_tokens, do_sample=do_sample, seed=seed)
        if codes.shape[1] == 0:
            return np.zeros(0, dtype=np.float32)
        return self.codec(codes).float().cpu().numpy()
