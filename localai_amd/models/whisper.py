"""Whisper speech-to-text on the engine's device (the reference's `whisper` backend).

Reference behaviour: `backend/go/transcribe/whisper/whisper.go:27-104` converts the upload to
16 kHz mono PCM with ffmpeg (`pkg/utils/ffmpeg.go:18`), runs whisper.cpp over the samples
(language from the request or "auto", optional translate) and returns whisper.cpp's segments
(id, text, start / end as Go durations, token ids) plus their concatenated text.

Model files are whisper.cpp's GGML binaries (`ggml-base.en.bin`, ...): magic 'ggml', eleven int32
hyper-parameters, the mel filterbank, the byte-level vocabulary, then (n_dims, name length,
type, ne[], name, data) tensor records with the OpenAI checkpoint's tensor names [external:
whisper.cpp models/convert-pt-to-ggml.py, whisper_model_load].  Quantised files (q4_0 ... q8_0)
are dequantised at load.

Compute: the log-mel front end (STFT n_fft 400 / hop 160, Hann, log10, 8-decade floor,
(x + 4) / 4), the conv stem + pre-LN transformer encoder over 30-s windows, and the decoder with
self-attention KV caches and per-window cross-attention K/V, greedily decoded with timestamp
tokens (whisper.cpp / OpenAI rules: a window opens with a timestamp <= 1 s, timestamps come in
pairs and never decrease, a timestamp wins when the timestamps' total probability beats the best
text token, no <|notimestamps|>); text between a timestamp pair is one segment with its start /
end, and a window that ends on a lone timestamp seeks the next window to it.  `timestamps=False`
keeps the single-segment-per-window mode.  The GEMMs run through torch.matmul (hipBLASLt on the GPU, bf16 weights); whisper
is a side workload next to the LLM path, whose hot ops are the hand-written kernels.
"""
from __future__ import annotations

import io
import math
import os
import struct
import subprocess
import wave
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as Fn

from ..gguf import dequantize, type_nbytes

GGML_MAGIC = 0x67676D6C
SAMPLE_RATE = 16000
N_FFT, HOP = 400, 160
CHUNK_S = 30
N_SAMPLES = CHUNK_S * SAMPLE_RATE
N_FRAMES = N_SAMPLES // HOP

LANGUAGES = ["en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
             "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
             "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
             "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
             "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
             "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su", "yue"]


@dataclass
class WhisperHParams:
    n_vocab: int
    n_audio_ctx: int
    n_audio_state: int
    n_audio_head: int
    n_audio_layer: int
    n_text_ctx: int
    n_text_state: int
    n_text_head: int
    n_text_layer: int
    n_mels: int
    ftype: int

    FIELDS = ("n_vocab", "n_audio_ctx", "n_audio_state", "n_audio_head", "n_audio_layer", "n_text_ctx",
              "n_text_state", "n_text_head", "n_text_layer", "n_mels", "ftype")


def is_whisper_ggml(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            return struct.unpack("<I", f.read(4))[0] == GGML_MAGIC
    except (OSError, struct.error):
        return False


def read_ggml(path: str):
    """-> (hparams, mel filters [n_mel, n_fft] f32, vocabulary bytes, {name: f32 array (torch order)})."""
    with open(path, "rb") as fh:
        mm = fh.read()  # whisper files are at most ~3 GB (large, f16): read whole
    off = 0

    def i32(n=1):
        nonlocal off
        v = struct.unpack_from(f"<{n}i", mm, off)
        off += 4 * n
        return v if n > 1 else v[0]

    if struct.unpack_from("<I", mm, 0)[0] != GGML_MAGIC:
        raise ValueError(f"{path}: not a whisper.cpp GGML model")
    off = 4
    hp = WhisperHParams(*i32(11))
    n_mel, n_fft = i32(2)
    filters = np.frombuffer(mm, dtype=np.float32, count=n_mel * n_fft, offset=off).reshape(n_mel, n_fft).copy()
    off += 4 * n_mel * n_fft
    n_words = i32()
    words: List[bytes] = []
    for _ in range(n_words):
        ln = i32()
        words.append(bytes(mm[off:off + ln]))
        off += ln
    tensors: Dict[str, np.ndarray] = {}
    size = len(mm)
    while off + 12 <= size:
        n_dims, name_len, ttype = i32(3)
        ne = [i32() for _ in range(n_dims)]
        name = bytes(mm[off:off + name_len]).decode()
        off += name_len
        n = int(np.prod(ne))
        nb = type_nbytes(ttype, n)
        raw = np.frombuffer(mm, dtype=np.uint8, count=nb, offset=off)
        off += nb
        shape = tuple(reversed(ne))
        tensors[name] = dequantize(raw, ttype, shape).reshape(shape).astype(np.float32)
    return hp, filters, words, tensors


@dataclass
class Segment:
    id: int
    start_ns: int
    end_ns: int
    text: str
    tokens: List[int]


class WhisperModel:
    def __init__(self, path: str, device="cpu"):
        self.path = path
        self.device = torch.device(device)
        hp, filters, words, t = read_ggml(path)
        self.hp, self.words = hp, words
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.filters = torch.from_numpy(filters).to(self.device)
        self.w = {k: torch.from_numpy(v).to(self.device) for k, v in t.items()}
        for k, v in list(self.w.items()):  # matmul weights in the compute dtype, the rest fp32
            if v.dim() == 2 and k.endswith(".weight") and "embedding" not in k:
                self.w[k] = v.to(self.dtype)
        self.tok_emb = self.w["decoder.token_embedding.weight"].to(self.dtype)
        # special tokens (whisper.cpp whisper_vocab): languages are reserved even in .en models
        self.multilingual = hp.n_vocab >= 51865
        self.n_lang = 100 if hp.n_vocab >= 51866 else 99
        self.eot = 50256 + int(self.multilingual)
        self.sot = self.eot + 1
        self.tok_translate = self.sot + 1 + self.n_lang
        self.tok_transcribe = self.tok_translate + 1
        self.no_timestamps = self.tok_translate + 5
        self.timestamp_begin = self.tok_translate + 6

    # ------------------------------------------------------------------ front end
    def log_mel(self, audio: torch.Tensor) -> torch.Tensor:
        """[n_mels, N_FRAMES] log-mel of one 30-s window (zero padded)."""
        a = torch.zeros(N_SAMPLES, dtype=torch.float32, device=self.device)
        a[:audio.shape[0]] = audio[:N_SAMPLES].to(self.device)
        win = torch.hann_window(N_FFT, device=self.device)
        st = torch.stft(a, N_FFT, HOP, window=win, return_complex=True)
        mag = st[..., :-1].abs() ** 2
        mel = self.filters @ mag
        lg = torch.clamp(mel, min=1e-10).log10()
        lg = torch.maximum(lg, lg.max() - 8.0)
        return (lg + 4.0) / 4.0

    # ------------------------------------------------------------------ transformer pieces
    def _lin(self, x, name, bias=True):
        y = x.to(self.dtype) @ self.w[name + ".weight"].t()
        b = self.w.get(name + ".bias") if bias else None
        y = y.float()
        return y + b if b is not None else y

    def _ln(self, x, name):
        return Fn.layer_norm(x, (x.shape[-1],), self.w[name + ".weight"], self.w[name + ".bias"], 1e-5)

    @staticmethod
    def _attend(q, k, v, n_head, causal_from: Optional[int] = None):
        """q [Tq, D], k / v [Tk, D] -> [Tq, D]; causal_from: absolute position of q row 0."""
        Tq, D = q.shape
        dh = D // n_head
        qh = q.view(Tq, n_head, dh).transpose(0, 1)
        kh = k.view(-1, n_head, dh).transpose(0, 1)
        vh = v.view(-1, n_head, dh).transpose(0, 1)
        s = (qh @ kh.transpose(1, 2)) / math.sqrt(dh)
        if causal_from is not None:
            Tk = kh.shape[1]
            qpos = torch.arange(causal_from, causal_from + Tq, device=q.device).view(-1, 1)
            s = s.masked_fill(torch.arange(Tk, device=q.device).view(1, -1) > qpos, float("-inf"))
        return (torch.softmax(s.float(), -1) @ vh.float()).transpose(0, 1).reshape(Tq, D)

    def _mlp(self, x, p):
        return self._lin(Fn.gelu(self._lin(x, p + "mlp.0")), p + "mlp.2")

    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        hp, w = self.hp, self.w
        x = mel.unsqueeze(0).float()
        x = Fn.gelu(Fn.conv1d(x, w["encoder.conv1.weight"].float(), w["encoder.conv1.bias"].view(-1), padding=1))
        x = Fn.gelu(Fn.conv1d(x, w["encoder.conv2.weight"].float(), w["encoder.conv2.bias"].view(-1), stride=2,
                              padding=1))
        x = x[0].t() + w["encoder.positional_embedding"][: x.shape[-1]]
        for i in range(hp.n_audio_layer):
            p = f"encoder.blocks.{i}."
            h = self._ln(x, p + "attn_ln")
            x = x + self._lin(self._attend(self._lin(h, p + "attn.query"), self._lin(h, p + "attn.key", bias=False),
                                           self._lin(h, p + "attn.value"), hp.n_audio_head), p + "attn.out")
            x = x + self._mlp(self._ln(x, p + "mlp_ln"), p)
        return self._ln(x, "encoder.ln_post")

    def _decoder(self, enc: torch.Tensor):
        """Greedy-decoding closure over one window's encoder output (cross K/V computed once)."""
        hp = self.hp
        cross = [(self._lin(enc, f"decoder.blocks.{i}.cross_attn.key", bias=False),
                  self._lin(enc, f"decoder.blocks.{i}.cross_attn.value")) for i in range(hp.n_text_layer)]
        cache: List[Tuple[torch.Tensor, torch.Tensor]] = [None] * hp.n_text_layer  # type: ignore
        pos = [0]

        def step(tokens: List[int]) -> torch.Tensor:
            T, p0 = len(tokens), pos[0]
            ids = torch.tensor(tokens, device=self.device)
            x = self.tok_emb[ids].float() + self.w["decoder.positional_embedding"][p0:p0 + T]
            for i in range(hp.n_text_layer):
                p = f"decoder.blocks.{i}."
                h = self._ln(x, p + "attn_ln")
                k, v = self._lin(h, p + "attn.key", bias=False), self._lin(h, p + "attn.value")
                if cache[i] is not None:
                    k, v = torch.cat([cache[i][0], k]), torch.cat([cache[i][1], v])
                cache[i] = (k, v)
                x = x + self._lin(self._attend(self._lin(h, p + "attn.query"), k, v, hp.n_text_head, causal_from=p0),
                                  p + "attn.out")
                h = self._ln(x, p + "cross_attn_ln")
                x = x + self._lin(self._attend(self._lin(h, p + "cross_attn.query"), cross[i][0], cross[i][1],
                                               hp.n_text_head), p + "cross_attn.out")
                x = x + self._mlp(self._ln(x, p + "mlp_ln"), p)
            pos[0] += T
            x = self._ln(x[-1:], "decoder.ln")
            return (x.to(self.dtype) @ self.tok_emb.t()).float()[0]
        return step

    def detect_language(self, enc: torch.Tensor) -> int:
        logits = self._decoder(enc)([self.sot])
        lang = logits[self.sot + 1:self.sot + 1 + self.n_lang]
        return int(torch.argmax(lang))

    def decode_window(self, enc: torch.Tensor, lang_id: Optional[int], translate: bool, max_tokens: int) -> List[int]:
        prompt = [self.sot]
        if self.multilingual:
            prompt += [self.sot + 1 + (lang_id or 0), self.tok_translate if translate else self.tok_transcribe]
        prompt.append(self.no_timestamps)
        step = self._decoder(enc)
        logits = step(prompt)
        out: List[int] = []
        limit = min(max_tokens, self.hp.n_text_ctx // 2)
        for _ in range(limit):
            logits[self.eot + 1:] = float("-inf")  # special and timestamp tokens (no-timestamp mode)
            if not out:
                logits[self.eot] = float("-inf")      # SuppressBlank: no empty transcript ...
                if self.words and len(self.words) > 220:
                    logits[220] = float("-inf")        # ... and no leading lone space
            t = int(torch.argmax(logits))
            if t == self.eot:
                break
            out.append(t)
            logits = step([t])
        return out

    TS_STEP = 0.02          # seconds per timestamp token
    MAX_INITIAL_TS = 1.0    # the first timestamp of a window is at most this (seconds)

    def _timestamp_rules(self, logits: torch.Tensor, out: List[int]) -> None:
        """In-place logit masks of timestamp decoding (OpenAI ApplyTimestampRules / whisper.cpp
        whisper_process_logits)."""
        tb, eot = self.timestamp_begin, self.eot
        logits[self.no_timestamps] = float("-inf")
        logits[eot + 1:tb] = float("-inf")                       # other specials
        if not out:
            logits[:tb] = float("-inf")                           # a window opens with a timestamp ...
            logits[tb + int(round(self.MAX_INITIAL_TS / self.TS_STEP)) + 1:] = float("-inf")  # ... <= 1 s
            return
        last_ts = out[-1] >= tb
        prev_ts = len(out) < 2 or out[-2] >= tb
        if last_ts:
            if prev_ts:
                logits[tb:] = float("-inf")                       # a pair is complete: text next
            else:
                logits[:eot] = float("-inf")                      # close the pair (or end)
        ts = [t for t in out if t >= tb]
        if ts:
            # never decrease; a segment has nonzero length; after a closing timestamp the next one
            # may repeat it (the next segment's start)
            floor = ts[-1] if (last_ts and not prev_ts) else ts[-1] + 1
            logits[tb:floor] = float("-inf")
        lp = torch.log_softmax(logits.float(), -1)
        if torch.logsumexp(lp[tb:], 0) > lp[:tb].max():
            logits[:tb] = float("-inf")                           # timestamps together beat any text token

    def decode_window_ts(self, enc: torch.Tensor, lang_id: Optional[int], translate: bool,
                         max_tokens: int) -> List[int]:
        prompt = [self.sot]
        if self.multilingual:
            prompt += [self.sot + 1 + (lang_id or 0), self.tok_translate if translate else self.tok_transcribe]
        step = self._decoder(enc)
        logits = step(prompt)
        out: List[int] = []
        for _ in range(min(max_tokens, self.hp.n_text_ctx // 2)):
            self._timestamp_rules(logits, out)
            t = int(torch.argmax(logits))
            if t == self.eot:
                break
            out.append(t)
            logits = step([t])
        return out

    def split_segments(self, toks: List[int], t0: float, dur: float):
        """Window tokens -> ([(start_s, end_s, text tokens)], seek_s): text between timestamps is a
        segment (absolute times from the window start t0); a trailing lone timestamp closing a
        segment moves the next window to it, otherwise the whole window was consumed."""
        tb = self.timestamp_begin
        segs, start, text = [], None, []
        for t in toks:
            if t >= tb:
                ts = (t - tb) * self.TS_STEP
                if start is not None and text:
                    segs.append((t0 + start, t0 + min(ts, dur), text))
                    text, start = [], None
                else:
                    start = ts
            else:
                if start is None:
                    start = 0.0
                text.append(t)
        if text:
            segs.append((t0 + start, t0 + dur, text))
        seek = dur
        if len(toks) >= 2 and toks[-1] >= tb and toks[-2] < tb:
            last = (toks[-1] - tb) * self.TS_STEP
            if 0 < last < dur:
                seek = last
        return segs, seek

    def shutdown(self):
        self.w.clear()

    def text(self, tokens: List[int]) -> str:
        return b"".join(self.words[t] for t in tokens if 0 <= t < len(self.words)).decode("utf-8", errors="replace")

    @torch.no_grad()
    def transcribe(self, audio: np.ndarray, language: str = "", translate: bool = False,
                   max_tokens_per_window: int = 224, timestamps: bool = True) -> Tuple[List[Segment], str]:
        x = torch.from_numpy(np.asarray(audio, dtype=np.float32))
        segs: List[Segment] = []
        lang_id = None
        if self.multilingual and language and language != "auto":
            if language not in LANGUAGES[:self.n_lang]:
                raise ValueError(f"unsupported language {language!r}")
            lang_id = LANGUAGES.index(language)
        if not timestamps:
            n = max(1, math.ceil(x.shape[0] / N_SAMPLES))
            for wi in range(n):
                chunk = x[wi * N_SAMPLES:(wi + 1) * N_SAMPLES]
                if chunk.numel() == 0:
                    break
                enc = self.encode(self.log_mel(chunk))
                if self.multilingual and lang_id is None:
                    lang_id = self.detect_language(enc)
                toks = self.decode_window(enc, lang_id, translate, max_tokens_per_window)
                start = wi * CHUNK_S * 10 ** 9
                end = start + int(chunk.numel() / SAMPLE_RATE * 1e9)
                segs.append(Segment(wi, start, end, self.text(toks), toks))
            return segs, "".join(s.text for s in segs)
        seek = 0                                                   # samples
        total = max(1, x.shape[0])
        while seek < total:
            chunk = x[seek:seek + N_SAMPLES]
            if chunk.numel() < HOP:                                # less than one frame left
                break
            enc = self.encode(self.log_mel(chunk))
            if self.multilingual and lang_id is None:
                lang_id = self.detect_language(enc)
            toks = self.decode_window_ts(enc, lang_id, translate, max_tokens_per_window)
            dur = chunk.numel() / SAMPLE_RATE
            parts, adv = self.split_segments(toks, seek / SAMPLE_RATE, dur)
            for s0, s1, tt in parts:
                segs.append(Segment(len(segs), int(round(s0 * 1e9)), int(round(max(s1, s0) * 1e9)), self.text(tt), tt))
            seek += max(HOP, int(round(adv * SAMPLE_RATE)))
        return segs, "".join(s.text for s in segs)


def load_audio(path: str) -> np.ndarray:
    """16 kHz mono float32 samples.  Like the reference (ffmpeg -ar 16000 -ac 1 pcm_s16le) when an
    ffmpeg binary exists; otherwise WAV files are read directly (8/16/32-bit PCM, any rate,
    channels averaged, polyphase-resampled to 16 kHz)."""
    try:
        r = subprocess.run(["ffmpeg", "-nostdin", "-loglevel", "error", "-i", path, "-f", "s16le", "-ar",
                            str(SAMPLE_RATE), "-ac", "1", "-acodec", "pcm_s16le", "-"], capture_output=True, timeout=600)
        if r.returncode == 0 and r.stdout:
            return np.frombuffer(r.stdout, dtype=np.int16).astype(np.float32) / 32768.0
    except (OSError, subprocess.TimeoutExpired):
        pass
    with open(path, "rb") as f:
        data = f.read()
    try:
        w = wave.open(io.BytesIO(data), "rb")
    except (wave.Error, EOFError) as e:
        raise ValueError(f"unsupported audio (no ffmpeg on this host; WAV expected): {e}") from e
    with w:
        ch, sw, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        a = np.frombuffer(raw, dtype="<i2").astype(np.float32) / 32768.0
    elif sw == 4:
        a = np.frombuffer(raw, dtype="<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        a = (np.frombuffer(raw, dtype=np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported WAV sample width {sw}")
    if ch > 1:
        a = a.reshape(-1, ch).mean(1)
    if rate != SAMPLE_RATE:
        from scipy.signal import resample_poly
        g = math.gcd(rate, SAMPLE_RATE)
        a = resample_poly(a, SAMPLE_RATE // g, rate // g).astype(np.float32)
    return a


def mel_filters(n_mels: int = 80, sr: int = SAMPLE_RATE, n_fft: int = N_FFT) -> np.ndarray:
    """Slaney-style mel filterbank [n_mels, n_fft // 2 + 1] (what whisper's mel_filters.npz holds),
    used by the synthetic model writer."""
    def hz_to_mel(f):
        f = np.asarray(f, dtype=np.float64)
        m = f / (200.0 / 3)
        log_t = f >= 1000.0
        return np.where(log_t, 15.0 + np.log(np.maximum(f, 1e-10) / 1000.0) / (np.log(6.4) / 27.0), m)

    def mel_to_hz(m):
        m = np.asarray(m, dtype=np.float64)
        f = m * (200.0 / 3)
        return np.where(m >= 15.0, 1000.0 * np.exp((np.log(6.4) / 27.0) * (m - 15.0)), f)

    fft_f = np.linspace(0, sr / 2, n_fft // 2 + 1)
    mel_pts = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2), n_mels + 2))
    fb = np.zeros((n_mels, n_fft // 2 + 1))
    for i in range(n_mels):
        lo, c, hi = mel_pts[i], mel_pts[i + 1], mel_pts[i + 2]
        up = (fft_f - lo) / max(c - lo, 1e-10)
        down = (hi - fft_f) / max(hi - c, 1e-10)
        fb[i] = np.maximum(0, np.minimum(up, down)) * (2.0 / (hi - lo))
    return fb.astype(np.float32)


def write_ggml(path: str, hp: WhisperHParams, filters: np.ndarray, words: List[bytes],
               tensors: Dict[str, np.ndarray]):
    """Write a whisper.cpp GGML model (the convert-pt-to-ggml.py layout): 2-D+ weights as F16
    (biases, norms and positional embeddings F32), conv biases as [n, 1]."""
    with open(path, "wb") as f:
        f.write(struct.pack("<I", GGML_MAGIC))
        f.write(struct.pack("<11i", *[getattr(hp, k) for k in WhisperHParams.FIELDS]))
        f.write(struct.pack("<2i", *filters.shape))
        f.write(filters.astype(np.float32).tobytes())
        f.write(struct.pack("<i", len(words)))
        for wd in words:
            f.write(struct.pack("<i", len(wd)))
            f.write(wd)
        for name, data in tensors.items():
            if name in ("encoder.conv1.bias", "encoder.conv2.bias"):
                data = data.reshape(-1, 1)
            f16 = data.ndim >= 2 and "positional_embedding" not in name and not name.endswith(".bias") \
                and hp.ftype == 1
            arr = data.astype(np.float16 if f16 else np.float32)
            nb = name.encode()
            f.write(struct.pack("<3i", arr.ndim, len(nb), 1 if f16 else 0))
            f.write(struct.pack(f"<{arr.ndim}i", *reversed(arr.shape)))
            f.write(nb)
            f.write(np.ascontiguousarray(arr).tobytes())
