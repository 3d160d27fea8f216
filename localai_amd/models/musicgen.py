"""Native MusicGen text-to-music: the `transformers-musicgen` SoundGeneration / TTS backend.

Reference behaviour: `backend/python/transformers-musicgen/backend.py:66-121` -- text (or an
unconditional request when the text is empty) -> audio codes -> waveform written to `dst`;
`duration` seconds -> int(duration * 51.2) new tokens (256 when unset, 512 for TTS),
`temperature` is the classifier-free guidance scale (3.0 when unset), `sample` toggles sampling.

Checkpoints in the Hugging Face layout (`config.json` with text_encoder / audio_encoder / decoder
sub-configs, `*.safetensors`, `tokenizer.json`), run entirely on the device:

  text encoder   T5 encoder: RMS norms, bucketed relative-position bias shared by all blocks,
                 ReLU or gated-GELU feed-forward
  decoder        pre-LN transformer over the sum of the K codebook embeddings + sinusoidal
                 positions; self-attention with a KV cache, cross-attention on the projected text
                 states (its K/V computed once); K linear heads.  Classifier-free guidance runs the
                 conditional and the unconditional row as one batch of two -- the unconditional
                 row's cross-attention contributes exactly zero (all-masked zero keys/values), so
                 it is skipped -- and mixes logits uncond + g * (cond - uncond)
  delay pattern  codebook k lags codebook 0 by k steps: positions outside each codebook's window
                 are forced to the pad id; the valid diagonal band is the code grid
  EnCodec        residual-VQ codebook sum -> SEANet decoder (causal reflect-padded convs, 2-layer
                 LSTM with a skip, ELU, transposed-conv upsamplers with right trim, residual units)
"""
from __future__ import annotations

import glob
import json
import math
import os
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .tts import _fold_weight_norm

_DEC = dict(vocab_size=2048, max_position_embeddings=2048, num_hidden_layers=24, ffn_dim=4096, num_attention_heads=16,
            activation_function="gelu", hidden_size=1024, scale_embedding=False, num_codebooks=4, audio_channels=1,
            pad_token_id=2048, bos_token_id=2048, decoder_start_token_id=None, cross_attention_hidden_size=None)
_T5 = dict(vocab_size=32128, d_model=512, d_kv=64, d_ff=2048, num_layers=6, num_heads=8,
           relative_attention_num_buckets=32, relative_attention_max_distance=128, layer_norm_epsilon=1e-6,
           feed_forward_proj="relu", eos_token_id=1)
_ENC = dict(sampling_rate=24000, audio_channels=1, hidden_size=128, num_filters=32, num_residual_layers=1,
            upsampling_ratios=[8, 5, 4, 2], norm_type="weight_norm", kernel_size=7, last_kernel_size=7,
            residual_kernel_size=3, dilation_growth_rate=2, use_causal_conv=True, pad_mode="reflect", compress=2,
            num_lstm_layers=2, trim_right_ratio=1.0, codebook_size=1024, codebook_dim=None, use_conv_shortcut=True)


def is_musicgen_dir(path: str) -> bool:
    try:
        with open(os.path.join(path, "config.json")) as f:
            return json.load(f).get("model_type") == "musicgen"
    except (OSError, ValueError):
        return False


def load_safetensors_dir(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    sd: Dict[str, torch.Tensor] = {}
    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if files:
        for fn in files:
            sd.update(load_file(fn))
        return sd
    return torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)


def _hp(defaults: dict, raw: Optional[dict]) -> dict:
    hp = dict(defaults)
    hp.update({k: v for k, v in (raw or {}).items() if k in defaults})
    return hp


def t5_bucket(rel: torch.Tensor, num_buckets: int, max_distance: int) -> torch.Tensor:
    """Bidirectional T5 relative-position bucket of (key - query)."""
    nb = num_buckets // 2
    out = (rel > 0).long() * nb
    a = rel.abs()
    exact = nb // 2
    large = exact + (torch.log(a.float().clamp_min(1) / exact) / math.log(max_distance / exact)
                     * (nb - exact)).long()
    large = large.clamp_max(nb - 1)
    return out + torch.where(a < exact, a, large)


class T5Encoder:
    def __init__(self, W: Dict[str, torch.Tensor], hp: dict, prefix: str = "text_encoder."):
        self.W, self.hp, self.p = W, hp, prefix

    def _rms(self, x, name):
        # T5LayerNorm: fp32 variance; the normalised states go back to a half-precision weight's dtype
        w = self.W[self.p + name]
        v = x.float().pow(2).mean(-1, keepdim=True)
        h = x * torch.rsqrt(v + self.hp["layer_norm_epsilon"])
        if w.dtype in (torch.float16, torch.bfloat16):
            h = h.to(w.dtype)
        return w * h

    def __call__(self, ids: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """ids [B, T] -> hidden [B, T, d_model]; mask [B, T] (1 = token)."""
        hp, W, p = self.hp, self.W, self.p
        nh, dk = hp["num_heads"], hp["d_kv"]
        x = W[p + "shared.weight"][ids] if p + "shared.weight" in W else W[p + "encoder.embed_tokens.weight"][ids]
        B, T, _ = x.shape
        pos = torch.arange(T, device=x.device)
        bucket = t5_bucket(pos[None, :] - pos[:, None], hp["relative_attention_num_buckets"],
                           hp["relative_attention_max_distance"])
        bias = W[p + "encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"][bucket]  # [T, T, nh]
        bias = bias.permute(2, 0, 1)[None]                                   # [1, nh, T, T]
        if mask is not None:
            bias = bias + (1.0 - mask[:, None, None, :].float()) * torch.finfo(torch.float32).min
        gated = hp["feed_forward_proj"].startswith("gated")
        for i in range(hp["num_layers"]):
            b = f"encoder.block.{i}.layer."
            h = self._rms(x, b + "0.layer_norm.weight")
            proj = lambda n: (h @ W[p + b + f"0.SelfAttention.{n}.weight"].t()).view(B, T, nh, dk).transpose(1, 2)  # noqa: E731
            q, k, v = proj("q"), proj("k"), proj("v")
            a = torch.softmax(q @ k.transpose(-1, -2) + bias, -1) @ v       # T5: no 1/sqrt(d) scaling
            x = x + a.transpose(1, 2).reshape(B, T, nh * dk) @ W[p + b + "0.SelfAttention.o.weight"].t()
            h = self._rms(x, b + "1.layer_norm.weight")
            ff = b + "1.DenseReluDense."
            if gated:
                u = F.gelu(h @ W[p + ff + "wi_0.weight"].t(), approximate="tanh") * (h @ W[p + ff + "wi_1.weight"].t())
            else:
                u = F.relu(h @ W[p + ff + "wi.weight"].t())
            x = x + u @ W[p + ff + "wo.weight"].t()
        return self._rms(x, "encoder.final_layer_norm.weight")


def _pad1d(x: torch.Tensor, left: int, right: int, mode: str) -> torch.Tensor:
    if mode != "reflect":
        return F.pad(x, (left, right), mode=mode if mode != "zero" else "constant")
    n = x.shape[-1]
    extra = max(left, right) - n + 1 if n <= max(left, right) else 0
    if extra:
        x = F.pad(x, (0, extra))
    y = F.pad(x, (left, right), mode="reflect")
    return y[..., :y.shape[-1] - extra] if extra else y


class EncodecDecoder:
    """Codes [K, T] -> waveform [channels, samples] (EnCodec residual-VQ + SEANet decoder)."""

    def __init__(self, W: Dict[str, torch.Tensor], hp: dict, device, prefix: str = "audio_encoder."):
        self.W, self.hp, self.p = W, hp, prefix
        self.lstm = None
        nf, ratios = hp["num_filters"], hp["upsampling_ratios"]
        scale = 2 ** len(ratios)
        dim = scale * nf
        # layer plan of decoder.layers.*: ("conv", idx, k, stride, dil) / ("lstm", idx) / ("elu",) /
        # ("convt", idx, k, stride) / ("res", idx, dim, dils)
        plan = [("conv", 0, hp["kernel_size"], 1, 1), ("lstm", 1)]
        i = 2
        for r in ratios:
            cur = scale * nf
            plan += [("elu",), ("convt", i + 1, 2 * r, r)]
            i += 2
            for j in range(hp["num_residual_layers"]):
                plan.append(("res", i, cur // 2, (hp["dilation_growth_rate"] ** j, 1)))
                i += 1
            scale //= 2
        plan += [("elu",), ("conv", i + 1, hp["last_kernel_size"], 1, 1)]
        self.plan = plan
        lp = f"{prefix}decoder.layers.1.lstm."
        self.lstm = torch.nn.LSTM(dim, dim, hp["num_lstm_layers"]).to(device)
        self.lstm.load_state_dict({k[len(lp):]: v for k, v in W.items() if k.startswith(lp)})
        self.lstm.flatten_parameters()

    def _conv(self, x, name, k, stride=1, dil=1):
        hp = self.hp
        keff = (k - 1) * dil + 1
        ptot = keff - stride
        n = x.shape[-1]
        frames = math.ceil((n - keff + ptot) / stride + 1) - 1
        extra = frames * stride + keff - ptot - n
        if hp["use_causal_conv"]:
            x = _pad1d(x, ptot, extra, hp["pad_mode"])
        else:
            pr = ptot // 2
            x = _pad1d(x, ptot - pr, pr + extra, hp["pad_mode"])
        y = F.conv1d(x, self.W[name + ".weight"], self.W.get(name + ".bias"), stride=stride, dilation=dil)
        if hp["norm_type"] == "time_group_norm":
            y = F.group_norm(y, 1, self.W[name.replace(".conv", ".norm") + ".weight"],
                             self.W[name.replace(".conv", ".norm") + ".bias"])
        return y

    def _convt(self, x, name, k, stride):
        hp = self.hp
        y = F.conv_transpose1d(x, self.W[name + ".weight"], self.W.get(name + ".bias"), stride=stride)
        if hp["norm_type"] == "time_group_norm":
            y = F.group_norm(y, 1, self.W[name.replace(".conv", ".norm") + ".weight"],
                             self.W[name.replace(".conv", ".norm") + ".bias"])
        ptot = k - stride
        pr = math.ceil(ptot * hp["trim_right_ratio"]) if hp["use_causal_conv"] else ptot // 2
        return y[..., ptot - pr:y.shape[-1] - pr]

    @torch.no_grad()
    def __call__(self, codes: torch.Tensor) -> torch.Tensor:
        """codes [Q, T] (Q <= quantizers) -> [audio_channels, samples]."""
        hp, W, p = self.hp, self.W, self.p
        x = sum(W[f"{p}quantizer.layers.{q}.codebook.embed"][codes[q]] for q in range(codes.shape[0]))  # [T, D]
        x = x.t()[None]                                                      # [1, D, T]
        dp = p + "decoder.layers."
        for st in self.plan:
            if st[0] == "conv":
                x = self._conv(x, f"{dp}{st[1]}.conv", st[2], st[3], st[4])
            elif st[0] == "lstm":
                y = x.permute(2, 0, 1)
                x = (self.lstm(y)[0] + y).permute(1, 2, 0)
            elif st[0] == "elu":
                x = F.elu(x)
            elif st[0] == "convt":
                x = self._convt(x, f"{dp}{st[1]}.conv", st[2], st[3])
            else:  # residual unit: ELU, conv(k, dil), ELU, conv(1) + shortcut
                _, idx, dim, dils = st
                y = self._conv(F.elu(x), f"{dp}{idx}.block.1.conv", hp["residual_kernel_size"], 1, dils[0])
                y = self._conv(F.elu(y), f"{dp}{idx}.block.3.conv", 1, 1, dils[1])
                sc = self._conv(x, f"{dp}{idx}.shortcut.conv", 1) if hp["use_conv_shortcut"] else x
                x = sc + y
        return x[0]


class MusicGen:
    def __init__(self, path: str, device: str = "cpu"):
        with open(os.path.join(path, "config.json")) as f:
            cfg = json.load(f)
        self.dec = _hp(_DEC, cfg.get("decoder"))
        self.t5 = _hp(_T5, cfg.get("text_encoder"))
        self.enc = _hp(_ENC, cfg.get("audio_encoder"))
        self.device = torch.device(device)
        sd = _fold_weight_norm(load_safetensors_dir(path))
        self.W = {k: v.float().to(self.device) for k, v in sd.items()}
        self.text = T5Encoder(self.W, self.t5)
        self.codec = EncodecDecoder(self.W, self.enc, self.device)
        self.sampling_rate = int(self.enc["sampling_rate"])
        self.tokenizer = None
        tj = os.path.join(path, "tokenizer.json")
        if os.path.exists(tj):
            from tokenizers import Tokenizer
            self.tokenizer = Tokenizer.from_file(tj)
        gc = {}
        gp = os.path.join(path, "generation_config.json")
        if os.path.exists(gp):
            with open(gp) as f:
                gc = json.load(f)
        self.top_k = int(gc.get("top_k") or 250)
        self.pad = int(self.dec["pad_token_id"])
        self.start = int(gc.get("decoder_start_token_id") or self.dec["decoder_start_token_id"] or self.pad)
        H = self.dec["hidden_size"]
        half = H // 2
        f = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000) / (half - 1)))
        self._freq = f.to(self.device)

    def _positions(self, start: int, n: int) -> torch.Tensor:
        t = torch.arange(start, start + n, device=self.device, dtype=torch.float32)[:, None] * self._freq[None]
        e = torch.cat([torch.cos(t), torch.sin(t)], 1)
        if self.dec["hidden_size"] % 2:
            e = F.pad(e, (0, 1))
        return e

    def encode_text(self, text: str):
        if not text:
            return None
        if self.tokenizer is None:
            raise RuntimeError("the checkpoint has no tokenizer.json")
        ids = self.tokenizer.encode(text).ids
        return torch.tensor([ids], device=self.device)

    def _cond(self, ids: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """T5 states projected to the decoder width (None: unconditional)."""
        if ids is None:
            return None
        h = self.text(ids)
        if "enc_to_dec_proj.weight" in self.W:
            h = F.linear(h, self.W["enc_to_dec_proj.weight"], self.W["enc_to_dec_proj.bias"])
        return h[0]                                                          # [S, H]

    @torch.no_grad()
    def generate_codes(self, ids: Optional[torch.Tensor], max_new_tokens: int, guidance_scale: float = 3.0,
                       do_sample: bool = True, top_k: Optional[int] = None, temperature: float = 1.0,
                       seed: Optional[int] = None) -> torch.Tensor:
        """-> codes [K, frames] (frames = max_new_tokens + 1 - K; stereo: + 1 - K/2)."""
        d, W = self.dec, self.W
        K, H, nh = d["num_codebooks"], d["hidden_size"], d["num_attention_heads"]
        hd = H // nh
        L = max_new_tokens + 1
        pad = self.pad
        # delay pattern: codebook k lags by k steps (stereo: the left/right pair of each level shares
        # a lag); positions outside a codebook's window are forced to the start/pad id
        kc = K // 2 if d["audio_channels"] == 2 else K
        kk = (torch.arange(K) // (K // kc))[:, None]
        tt = torch.arange(L)[None, :]
        forced = (tt <= kk) | (tt >= L - kc + 1 + kk)
        forced = forced.to(self.device)
        enc = self._cond(ids)
        cfg = guidance_scale is not None and guidance_scale > 1 and enc is not None
        B = 2 if cfg else 1                                                  # row 0 conditional, row 1 not
        cross = []
        if enc is not None:
            for i in range(d["num_hidden_layers"]):
                pp = f"decoder.model.decoder.layers.{i}.encoder_attn."
                ck = (enc @ W[pp + "k_proj.weight"].t()).view(-1, nh, hd).transpose(0, 1)
                cv = (enc @ W[pp + "v_proj.weight"].t()).view(-1, nh, hd).transpose(0, 1)
                cross.append((ck, cv))
        kc = [torch.zeros(B, nh, L, hd, device=self.device) for _ in range(d["num_hidden_layers"])]
        vc = [torch.zeros_like(kc[0]) for _ in range(d["num_hidden_layers"])]
        gen = None
        if do_sample:
            gen = torch.Generator(device=self.device)
            gen.manual_seed(int(seed) if seed is not None else int(torch.randint(0, 2 ** 31 - 1, (1,))))
        seq = torch.full((K, L), self.start, dtype=torch.long, device=self.device)
        tk = top_k or self.top_k
        act = F.gelu if d["activation_function"] == "gelu" else F.relu
        for s in range(L - 1):
            tok = seq[:, s]                                                  # [K]
            x = sum(W[f"decoder.model.decoder.embed_tokens.{k}.weight"][tok[k]] for k in range(K))
            if d["scale_embedding"]:
                x = x * math.sqrt(H)
            x = (x + self._positions(s, 1)[0]).expand(B, H).contiguous()     # [B, H]
            for i in range(d["num_hidden_layers"]):
                pp = f"decoder.model.decoder.layers.{i}."
                h = F.layer_norm(x, (H,), W[pp + "self_attn_layer_norm.weight"], W[pp + "self_attn_layer_norm.bias"])
                q = (h @ W[pp + "self_attn.q_proj.weight"].t()).view(B, nh, 1, hd)
                kc[i][:, :, s] = (h @ W[pp + "self_attn.k_proj.weight"].t()).view(B, nh, hd)
                vc[i][:, :, s] = (h @ W[pp + "self_attn.v_proj.weight"].t()).view(B, nh, hd)
                a = torch.softmax((q @ kc[i][:, :, :s + 1].transpose(-1, -2)) * hd ** -0.5, -1) @ vc[i][:, :, :s + 1]
                x = x + a.reshape(B, H) @ W[pp + "self_attn.out_proj.weight"].t()
                if cross:
                    h = F.layer_norm(x[:1], (H,), W[pp + "encoder_attn_layer_norm.weight"],
                                     W[pp + "encoder_attn_layer_norm.bias"])
                    q = (h @ W[pp + "encoder_attn.q_proj.weight"].t()).view(nh, 1, hd)
                    ck, cv = cross[i]
                    a = torch.softmax((q @ ck.transpose(-1, -2)) * hd ** -0.5, -1) @ cv
                    upd = a.reshape(1, H) @ W[pp + "encoder_attn.out_proj.weight"].t()
                    x = torch.cat([x[:1] + upd, x[1:]], 0)                   # row 1 (unconditional): + 0
                h = F.layer_norm(x, (H,), W[pp + "final_layer_norm.weight"], W[pp + "final_layer_norm.bias"])
                x = x + act(h @ W[pp + "fc1.weight"].t()) @ W[pp + "fc2.weight"].t()
            x = F.layer_norm(x, (H,), W["decoder.model.decoder.layer_norm.weight"],
                             W["decoder.model.decoder.layer_norm.bias"])
            logits = torch.stack([x @ W[f"decoder.lm_heads.{k}.weight"].t() for k in range(K)], 1)  # [B, K, V]
            lg = logits[1] + (logits[0] - logits[1]) * guidance_scale if cfg else logits[0]
            if do_sample:
                lg = lg / max(temperature, 1e-5)
                if tk and tk < lg.shape[-1]:
                    kth = torch.topk(lg, tk, -1).values[:, -1:]
                    lg = lg.masked_fill(lg < kth, float("-inf"))
                nxt = torch.multinomial(torch.softmax(lg, -1), 1, generator=gen)[:, 0]
            else:
                nxt = lg.argmax(-1)
            seq[:, s + 1] = torch.where(forced[:, s + 1], torch.full_like(nxt, self.start), nxt)
        keep = ~forced                                                       # the band of real codes
        return torch.stack([seq[k][keep[k]] for k in range(K)])

    @torch.no_grad()
    def generate(self, text: str, max_new_tokens: int = 256, guidance_scale: float = 3.0, do_sample: bool = True,
                 seed: Optional[int] = None) -> np.ndarray:
        """-> float32 waveform [samples] (mono) or [channels, samples]."""
        codes = self.generate_codes(self.encode_text(text), max_new_tokens, guidance_scale, do_sample, seed=seed)
        if self.dec["audio_channels"] == 2:
            wav = torch.cat([self.codec(codes[0::2]), self.codec(codes[1::2])], 0)
            return wav.float().cpu().numpy()
        return self.codec(codes)[0].float().cpu().numpy()
