"""Native VITS text-to-speech: the `piper` / `vits` / `mms-tts` TTS backends.

Reference behaviour: `backend/go/tts/piper.go:30-49` (text -> wav file at `dst`, one voice per
model), `backend/python/coqui/backend.py:67` / `transformers` TTS (VITS checkpoints), routed by
`core/backend/tts.go` (piper is the default TTS backend).  Piper voices are VITS networks; this
module runs VITS checkpoints in the Hugging Face layout (`config.json`, `vocab.json`,
`tokenizer_config.json`, `model.safetensors` or `pytorch_model.bin`, e.g. facebook/mms-tts-*),
entirely on the device:

  text encoder   transformer with windowed relative-position attention (bias and value terms
                 gathered per offset, no pad/reshape skew), conv feed-forward, post-LayerNorm
  durations      stochastic (reversed spline/affine flows over noise) or deterministic predictor
  expansion      per-token frame counts -> repeat_interleave of the prior mean / log-sd
  flow           reversed residual-coupling layers (gated WaveNet), channel flips
  vocoder        HiFi-GAN: transposed-conv upsamplers + multi-receptive-field residual blocks

Weight-normalised convolutions are folded to plain weights once at load.  Noise is drawn from a
CPU generator in a fixed order (duration noise, then prior noise), so a seed gives the same
waveform on every device.  Checkpoints load with safetensors or `torch.load(weights_only=True)`.
"""
from __future__ import annotations

import json
import math
import os
import re
import wave
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

_DEFAULTS = dict(
    vocab_size=38, hidden_size=192, num_hidden_layers=6, num_attention_heads=2, window_size=4, ffn_dim=768,
    ffn_kernel_size=3, flow_size=192, hidden_act="relu", layer_norm_eps=1e-5, use_stochastic_duration_prediction=True,
    num_speakers=1, speaker_embedding_size=0, upsample_initial_channel=512, upsample_rates=[8, 8, 2, 2],
    upsample_kernel_sizes=[16, 16, 4, 4], resblock_kernel_sizes=[3, 7, 11],
    resblock_dilation_sizes=[[1, 3, 5], [1, 3, 5], [1, 3, 5]], leaky_relu_slope=0.1, depth_separable_channels=2,
    depth_separable_num_layers=3, duration_predictor_flow_bins=10, duration_predictor_tail_bound=5.0,
    duration_predictor_kernel_size=3, duration_predictor_num_flows=4, duration_predictor_filter_channels=256,
    prior_encoder_num_flows=4, prior_encoder_num_wavenet_layers=4, wavenet_kernel_size=5, wavenet_dilation_rate=1,
    speaking_rate=1.0, noise_scale=0.667, noise_scale_duration=0.8, sampling_rate=16000)


def is_vits_dir(path: str) -> bool:
    try:
        with open(os.path.join(path, "config.json")) as f:
            return json.load(f).get("model_type") == "vits"
    except (OSError, ValueError):
        return False


def _load_state(path: str) -> Dict[str, torch.Tensor]:
    st = os.path.join(path, "model.safetensors")
    if os.path.exists(st):
        from safetensors.torch import load_file
        return load_file(st)
    return torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)


def _fold_weight_norm(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """weight = g * v / |v| (norm over every dim but 0), for both the legacy `weight_g/weight_v`
    and the parametrization `parametrizations.weight.original0/1` spellings."""
    out = {}
    pairs = {}
    for k, v in sd.items():
        m = re.match(r"(.*)\.(weight_g|weight_v|parametrizations\.weight\.original0|parametrizations\.weight\.original1)$", k)
        if m:
            pairs.setdefault(m.group(1), {})["g" if m.group(2) in ("weight_g", "parametrizations.weight.original0")
                                            else "v"] = v
        else:
            out[k] = v
    for base, gv in pairs.items():
        g, v = gv["g"].float(), gv["v"].float()
        norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape([-1] + [1] * (v.dim() - 1))
        out[base + ".weight"] = g * v / norm
    return out


class VitsTokenizer:
    """Characters -> ids from vocab.json (mms-tts style): optional lower-casing that keeps
    multi-character vocabulary entries, out-of-vocabulary characters dropped when normalising,
    and a blank (id 0) between every pair of symbols when `add_blank`."""

    def __init__(self, path: str):
        with open(os.path.join(path, "vocab.json"), encoding="utf-8") as f:
            self.vocab: Dict[str, int] = json.load(f)
        cfg = {}
        p = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(p):
            with open(p, encoding="utf-8") as f:
                cfg = json.load(f)
        self.add_blank = bool(cfg.get("add_blank", True))
        self.normalize = bool(cfg.get("normalize", True))
        self.unk = self.vocab.get(cfg.get("unk_token", "<unk>"), 0)
        self._multi = sorted((w for w in self.vocab if len(w) > 1), key=len, reverse=True)

    def __call__(self, text: str) -> List[int]:
        if self.normalize:
            out, i = [], 0
            while i < len(text):
                for w in self._multi:
                    if text.startswith(w, i):
                        out.append(w)
                        i += len(w)
                        break
                else:
                    out.append(text[i].lower())
                    i += 1
            syms = [s for s in out if s in self.vocab]
            while syms and syms[0] == " ":
                syms.pop(0)
            while syms and syms[-1] == " ":
                syms.pop()
        else:
            syms = list(text)
        ids = [self.vocab.get(s, self.unk) for s in syms]
        if self.add_blank:
            inter = [0] * (2 * len(ids) + 1)
            inter[1::2] = ids
            ids = inter
        return ids


def _rq_spline_inverse(y, uw, uh, ud, tail: float, min_w: float = 1e-3, min_h: float = 1e-3, min_d: float = 1e-3):
    """Inverse of the monotone rational-quadratic spline on [-tail, tail] (identity outside).
    y [...], uw/uh [..., B], ud [..., B-1] (inner knot derivatives, unconstrained)."""
    B = uw.shape[-1]
    inside = (y >= -tail) & (y <= tail)
    edge = math.log(math.exp(1 - min_d) - 1)
    ud = F.pad(ud, (1, 1), value=edge)

    def knots(u, mn):
        w = mn + (1 - mn * B) * torch.softmax(u, -1)
        c = F.pad(torch.cumsum(w, -1), (1, 0))
        c = 2 * tail * c - tail
        c[..., 0], c[..., -1] = -tail, tail
        return c, c[..., 1:] - c[..., :-1]

    cw, w = knots(uw, min_w)
    ch, h = knots(uh, min_h)
    d = min_d + F.softplus(ud)
    loc = ch.clone()
    loc[..., -1] += 1e-6
    k = (torch.sum(y[..., None] >= loc, -1) - 1).clamp(0, B - 1)[..., None]
    g = lambda t: t.gather(-1, k)[..., 0]  # noqa: E731
    x0, wk, y0, hk = g(cw), g(w), g(ch), g(h)
    dk, dk1 = g(d), d[..., 1:].gather(-1, k)[..., 0]
    s = hk / wk
    t1 = dk + dk1 - 2 * s
    r = (y - y0) * t1
    a = hk * (s - dk) + r
    b = hk * dk - r
    c = -s * (y - y0)
    root = (2 * c) / (-b - torch.sqrt(torch.clamp_min(b * b - 4 * a * c, 0)))
    return torch.where(inside, root * wk + x0, y)


class VitsVoice:
    def __init__(self, path: str, device: str = "cpu"):
        with open(os.path.join(path, "config.json")) as f:
            raw = json.load(f)
        self.hp = dict(_DEFAULTS)
        self.hp.update({k: v for k, v in raw.items() if k in _DEFAULTS})
        self.device = torch.device(device)
        self.tok = VitsTokenizer(path)
        sd = _fold_weight_norm(_load_state(path))
        self.W = {k: v.float().to(self.device) for k, v in sd.items()}
        self.sampling_rate = int(self.hp["sampling_rate"])

    # ------------------------------------------------------------------ building blocks
    def _conv(self, x, name, pad=0, dil=1, groups=1):
        return F.conv1d(x, self.W[name + ".weight"], self.W.get(name + ".bias"), padding=pad, dilation=dil,
                        groups=groups)

    def _ln_c(self, x, name, eps=1e-5):
        """LayerNorm over channels of a [B, C, T] tensor."""
        return F.layer_norm(x.transpose(1, 2), (x.shape[1],), self.W[name + ".weight"], self.W[name + ".bias"],
                            eps).transpose(1, 2)

    def _text_encoder(self, ids: torch.Tensor):
        hp, W = self.hp, self.W
        H, nh, win = hp["hidden_size"], hp["num_attention_heads"], hp["window_size"]
        hd = H // nh
        x = W["text_encoder.embed_tokens.weight"][ids] * math.sqrt(H)      # [T, H]
        T = x.shape[0]
        pos = torch.arange(T, device=x.device)
        rel = pos[None, :] - pos[:, None]                                   # j - i
        near = rel.abs() <= (win or 0)
        ridx = (rel + (win or 0)).clamp(0, 2 * (win or 0))
        act = {"relu": F.relu, "gelu": F.gelu}.get(hp["hidden_act"], F.relu)
        k_ff = hp["ffn_kernel_size"]
        for i in range(hp["num_hidden_layers"]):
            p = f"text_encoder.encoder.layers.{i}."
            lin = lambda t, n: F.linear(t, W[p + f"attention.{n}.weight"], W.get(p + f"attention.{n}.bias"))  # noqa: E731
            q = (lin(x, "q_proj") * hd ** -0.5).view(T, nh, hd).transpose(0, 1)   # [nh, T, hd]
            k = lin(x, "k_proj").view(T, nh, hd).transpose(0, 1)
            v = lin(x, "v_proj").view(T, nh, hd).transpose(0, 1)
            s = q @ k.transpose(1, 2)
            if win:
                ek, ev = W[p + "attention.emb_rel_k"][0], W[p + "attention.emb_rel_v"][0]   # [2w+1, hd]
                rk = q @ ek.t()                                             # [nh, T, 2w+1]
                s = s + torch.where(near, rk.gather(2, ridx.expand(nh, T, T)), torch.zeros((), device=x.device))
            pr = torch.softmax(s, -1)
            o = pr @ v
            if win:
                # sum_j p[i, j] * ev[j - i + w] over the window: scatter the probabilities per offset
                pw = torch.zeros(nh, T, 2 * win + 1, device=x.device)
                pw.scatter_add_(2, ridx.expand(nh, T, T), torch.where(near, pr, torch.zeros((), device=x.device)))
                o = o + pw @ ev
            o = lin(o.transpose(0, 1).reshape(T, H), "out_proj")
            x = F.layer_norm(x + o, (H,), W[p + "layer_norm.weight"], W[p + "layer_norm.bias"], hp["layer_norm_eps"])
            y = x.t()[None]                                                 # [1, H, T]
            pad = ((k_ff - 1) // 2, k_ff // 2)
            y = act(self._conv(F.pad(y, pad), p + "feed_forward.conv_1"))
            y = self._conv(F.pad(y, pad), p + "feed_forward.conv_2")
            x = F.layer_norm(x + y[0].t(), (H,), W[p + "final_layer_norm.weight"], W[p + "final_layer_norm.bias"],
                             hp["layer_norm_eps"])
        stats = self._conv(x.t()[None], "text_encoder.project")           # [1, 2*flow, T]
        fs = hp["flow_size"]
        return x.t()[None], stats[:, :fs], stats[:, fs:]

    def _dds(self, x, prefix, cond=None):
        hp = self.hp
        k = hp["duration_predictor_kernel_size"]
        C = x.shape[1]
        if cond is not None:
            x = x + cond
        for i in range(hp["depth_separable_num_layers"]):
            d = k ** i
            y = self._conv(x, f"{prefix}.convs_dilated.{i}", pad=(k * d - d) // 2, dil=d, groups=C)
            y = F.gelu(self._ln_c(y, f"{prefix}.norms_1.{i}"))
            y = self._conv(y, f"{prefix}.convs_pointwise.{i}")
            y = F.gelu(self._ln_c(y, f"{prefix}.norms_2.{i}"))
            x = x + y
        return x

    def _log_durations(self, h, g, gen):
        hp, W = self.hp, self.W
        if not hp["use_stochastic_duration_prediction"]:
            x = h if g is None else h + self._conv(g, "duration_predictor.cond")
            k = hp["duration_predictor_kernel_size"]
            eps = hp["layer_norm_eps"]
            x = self._ln_c(torch.relu(self._conv(x, "duration_predictor.conv_1", pad=k // 2)), "duration_predictor.norm_1", eps)
            x = self._ln_c(torch.relu(self._conv(x, "duration_predictor.conv_2", pad=k // 2)), "duration_predictor.norm_2", eps)
            return self._conv(x, "duration_predictor.proj")
        p = "duration_predictor"
        x = self._conv(h, p + ".conv_pre")
        if g is not None:
            x = x + self._conv(g, p + ".cond")
        x = self._conv(self._dds(x, p + ".conv_dds"), p + ".conv_proj")
        T = h.shape[2]
        z = torch.randn(1, 2, T, generator=gen).to(h.device) * hp["noise_scale_duration"]
        nf = hp["duration_predictor_num_flows"]
        bins, tail = hp["duration_predictor_flow_bins"], hp["duration_predictor_tail_bound"]
        C = hp["hidden_size"]
        # reversed flow stack: conv flows nf .. 2 (flow 1 is skipped at inference), then the affine
        for f in list(range(nf, 1, -1)) + [0]:
            z = torch.flip(z, [1])
            fp = f"{p}.flows.{f}"
            if f == 0:
                z = (z - W[fp + ".translate"]) * torch.exp(-W[fp + ".log_scale"])
                continue
            a, b = z[:, :1], z[:, 1:]
            y = self._conv(a, fp + ".conv_pre")
            y = self._conv(self._dds(y, fp + ".conv_dds", cond=x), fp + ".conv_proj")   # [1, 3B-1, T]
            y = y.reshape(1, 1, 3 * bins - 1, T).permute(0, 1, 3, 2)
            b = _rq_spline_inverse(b, y[..., :bins] / math.sqrt(C), y[..., bins:2 * bins] / math.sqrt(C),
                                   y[..., 2 * bins:], tail)
            z = torch.cat([a, b], 1)
        return z[:, :1]

    def _wavenet(self, x, prefix, g):
        hp = self.hp
        H, L = hp["hidden_size"], hp["prior_encoder_num_wavenet_layers"]
        k, dr = hp["wavenet_kernel_size"], hp["wavenet_dilation_rate"]
        gc = self._conv(g, prefix + ".cond_layer") if g is not None else None
        out = torch.zeros_like(x)
        for i in range(L):
            d = dr ** i
            a = self._conv(x, f"{prefix}.in_layers.{i}", pad=(k * d - d) // 2, dil=d)
            if gc is not None:
                a = a + gc[:, 2 * H * i:2 * H * (i + 1)]
            a = torch.tanh(a[:, :H]) * torch.sigmoid(a[:, H:])
            rs = self._conv(a, f"{prefix}.res_skip_layers.{i}")
            if i < L - 1:
                x = x + rs[:, :H]
                out = out + rs[:, H:]
            else:
                out = out + rs
        return out

    def _flow_reverse(self, z, g):
        hp = self.hp
        half = hp["flow_size"] // 2
        for f in reversed(range(hp["prior_encoder_num_flows"])):
            z = torch.flip(z, [1])
            p = f"flow.flows.{f}"
            a, b = z[:, :half], z[:, half:]
            m = self._conv(self._wavenet(self._conv(a, p + ".conv_pre"), p + ".wavenet", g), p + ".conv_post")
            z = torch.cat([a, b - m], 1)
        return z

    def _vocoder(self, z, g):
        hp = self.hp
        x = self._conv(z, "decoder.conv_pre", pad=3)
        if g is not None:
            x = x + self._conv(g, "decoder.cond")
        nk = len(hp["resblock_kernel_sizes"])
        slope = hp["leaky_relu_slope"]
        for i, (r, k) in enumerate(zip(hp["upsample_rates"], hp["upsample_kernel_sizes"])):
            x = F.leaky_relu(x, slope)
            x = F.conv_transpose1d(x, self.W[f"decoder.upsampler.{i}.weight"], self.W.get(f"decoder.upsampler.{i}.bias"),
                                   stride=r, padding=(k - r) // 2)
            acc = None
            for j, (rk, dils) in enumerate(zip(hp["resblock_kernel_sizes"], hp["resblock_dilation_sizes"])):
                p = f"decoder.resblocks.{i * nk + j}"
                y = x
                for m, d in enumerate(dils):
                    t = self._conv(F.leaky_relu(y, slope), f"{p}.convs1.{m}", pad=(rk * d - d) // 2, dil=d)
                    t = self._conv(F.leaky_relu(t, slope), f"{p}.convs2.{m}", pad=(rk - 1) // 2)
                    y = y + t
                acc = y if acc is None else acc + y
            x = acc / nk
        x = self._conv(F.leaky_relu(x), "decoder.conv_post", pad=3)   # final slope: the 0.01 default
        return torch.tanh(x)

    # ------------------------------------------------------------------ API
    @torch.no_grad()
    def synthesize(self, text: str, speaker_id: Optional[int] = None, speaking_rate: Optional[float] = None,
                   seed: Optional[int] = None, ids: Optional[List[int]] = None) -> np.ndarray:
        """text -> float32 waveform in [-1, 1] at `sampling_rate`."""
        hp = self.hp
        ids = self.tok(text) if ids is None else ids
        if not ids:
            return np.zeros(0, dtype=np.float32)
        gen = torch.Generator()
        gen.manual_seed(int(seed) if seed is not None else int(torch.randint(0, 2 ** 31 - 1, (1,))))
        t = torch.tensor(ids, dtype=torch.long, device=self.device)
        g = None
        if hp["num_speakers"] > 1:
            sid = int(speaker_id or 0)
            if not 0 <= sid < hp["num_speakers"]:
                raise ValueError(f"speaker id must be in 0..{hp['num_speakers'] - 1}")
            g = self.W["embed_speaker.weight"][sid].view(1, -1, 1)
        h, m, logs = self._text_encoder(t)
        logw = self._log_durations(h, g, gen)
        rate = speaking_rate if speaking_rate else hp["speaking_rate"]
        dur = torch.ceil(torch.exp(logw) * (1.0 / rate))[0, 0].long()                # frames per token
        if int(dur.sum()) == 0:
            m = torch.zeros(1, m.shape[1], 1, device=self.device)
            logs = torch.zeros_like(m)
        else:
            m = torch.repeat_interleave(m, dur, dim=2)
            logs = torch.repeat_interleave(logs, dur, dim=2)
        # prior noise filled into a frame-major [T, C] buffer viewed as [C, T] (the layout, and so
        # the draw order, of the HF reference's randn_like on its transposed prior)
        eps = torch.empty(1, m.shape[2], m.shape[1]).transpose(1, 2).normal_(generator=gen).to(self.device)
        z = m + eps * torch.exp(logs) * hp["noise_scale"]
        wav = self._vocoder(self._flow_reverse(z, g), g)
        return wav[0, 0].float().cpu().numpy()


def write_wav(path: str, audio: np.ndarray, sampling_rate: int) -> None:
    """16-bit PCM; audio [samples] (mono) or [channels, samples] (interleaved on write)."""
    ch = 1 if audio.ndim == 1 else audio.shape[0]
    pcm = (np.clip(audio if audio.ndim == 1 else audio.T, -1.0, 1.0) * 32767.0).astype("<i2")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with wave.open(path, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(2)
        w.setframerate(int(sampling_rate))
        w.writeframes(pcm.tobytes())
