"""Piper voices: `<voice>.onnx` + `<voice>.onnx.json`, the default `piper` TTS backend.

Reference: backend/go/tts/piper.go:20-24 (the model must end in `.onnx`; go-piper's TextToWav
phonemises the text, runs the voice through onnxruntime and writes a wav to `dst`),
core/backend/tts.go:28 (piper when no backend is named), gallery/piper.yaml and
embedded/models/rhasspy-voice-en-us-amy.yaml (the voice files).

Here the graph runs on utils/onnx_runtime.OnnxRunner (PyTorch ops, CPU or the GPU), so no ONNX
runtime is needed.  The voice's JSON config supplies the rest of piper's contract:

  ids      BOS "^", PAD "_", then every phoneme followed by PAD, then EOS "$" (phoneme_id_map;
           phoneme_map rewrites phonemes first; unknown phonemes are skipped)
  inputs   input [1, T] int64, input_lengths [1], scales [noise_scale, length_scale, noise_w]
           (inference.*), sid [1] for multi-speaker voices
  output   [.., samples] float audio; peak-normalised like piper before 16-bit PCM
  text     one utterance per sentence, joined with 0.2 s of silence

Phonemes: voices with phoneme_type "text" read the text's characters (NFD, lower-cased), exactly
as piper does.  "espeak" voices (every rhasspy voice in the gallery) get their phonemes from
models/g2p_en.py, a rule-based English front end that writes espeak-ng's en-us IPA (lexicon +
letter-to-sound rules + stress), folded onto the voice's phoneme_id_map; espeak-ng itself is not
in this image.  Text that already holds IPA letters is read as phonemes as given; voices whose
espeak voice is not English read the text's characters.  Parity with real piper voices is
unpinned (no voice files, espeak-ng or onnxruntime here); the graph executor itself is checked
against transformers' VITS exported to ONNX (tests/test_piper.py).
"""
from __future__ import annotations

import json
import os
import re
import unicodedata
from typing import Dict, List, Optional

import numpy as np
import torch

PAD, BOS, EOS = "_", "^", "$"
SENTENCE_SILENCE = 0.2
_SENT = re.compile(r"(?<=[.!?])\s+")
_IPA_INPUT = re.compile("[\u0250-\u02af\u02c8\u02cc\u02d0\u00e6\u00f0\u03b8\u014b]")   # IPA letters / marks


def config_path(onnx_path: str) -> Optional[str]:
    for p in (onnx_path + ".json", os.path.splitext(onnx_path)[0] + ".json"):
        if os.path.exists(p):
            return p
    return None


def is_piper_voice(path: str) -> bool:
    return path.endswith(".onnx") and os.path.isfile(path) and config_path(path) is not None


class PiperVoice:
    def __init__(self, path: str, device: str = "cpu"):
        from ..utils.onnx_runtime import OnnxRunner
        cp = config_path(path)
        if cp is None:
            raise ValueError(f"piper voice {path}: no {os.path.basename(path)}.json next to it")
        with open(cp, encoding="utf-8") as f:
            cfg = json.load(f)
        self.cfg = cfg
        self.sampling_rate = int((cfg.get("audio") or {}).get("sample_rate", 22050))
        inf = cfg.get("inference") or {}
        self.noise_scale = float(inf.get("noise_scale", 0.667))
        self.length_scale = float(inf.get("length_scale", 1.0))
        self.noise_w = float(inf.get("noise_w", 0.8))
        self.id_map: Dict[str, List[int]] = cfg.get("phoneme_id_map") or {}
        if not self.id_map:
            raise ValueError(f"piper voice {path}: phoneme_id_map missing from {cp}")
        self.phoneme_map: Dict[str, List[str]] = cfg.get("phoneme_map") or {}
        self.phoneme_type = cfg.get("phoneme_type", "espeak")
        self.num_speakers = int(cfg.get("num_speakers", 1))
        self.speaker_id_map: Dict[str, int] = cfg.get("speaker_id_map") or {}
        self.generator = torch.Generator()
        self.runner = OnnxRunner(path, device, generator=self.generator)

    # ------------------------------------------------------------------ text -> ids
    def _g2p(self) -> bool:
        """English espeak voice: phonemise with the en-us front end."""
        if self.phoneme_type != "espeak":
            return False
        lang = str(((self.cfg.get("espeak") or {}).get("voice")) or "en-us").lower()
        return lang.startswith("en")

    def phonemes(self, text: str) -> List[List[str]]:
        from . import g2p_en
        out = []
        g2p = self._g2p()
        for sent in _SENT.split(text.strip()):
            if not sent:
                continue
            if g2p and not _IPA_INPUT.search(sent):
                sent = g2p_en.phonemize(sent)
            s = unicodedata.normalize("NFD", sent)
            if self.phoneme_type == "text":
                s = s.lower()
            ph: List[str] = []
            for c in s:
                ph += self.phoneme_map.get(c, [c])
            if g2p:
                ph = g2p_en.fold(ph, self.id_map)
            out.append(ph)
        return out

    def ids(self, phonemes: List[str]) -> List[int]:
        m = self.id_map
        ids = list(m[BOS]) + list(m.get(PAD, []))
        for p in phonemes:
            if p in m:
                ids += m[p]
                ids += m.get(PAD, [])
        return ids + list(m[EOS])

    def speaker(self, voice: str) -> Optional[int]:
        if self.num_speakers <= 1:
            return None
        v = (voice or "").strip()
        if v in self.speaker_id_map:
            return int(self.speaker_id_map[v])
        return int(v) if v.isdigit() else 0

    # ------------------------------------------------------------------ synthesis
    @torch.no_grad()
    def _utterance(self, ids: List[int], sid: Optional[int], length_scale: float) -> np.ndarray:
        names = set(self.runner.input_names)
        feeds = {"input": torch.tensor([ids], dtype=torch.int64)}
        if "input_lengths" in names:
            feeds["input_lengths"] = torch.tensor([len(ids)], dtype=torch.int64)
        if "scales" in names:
            feeds["scales"] = torch.tensor([self.noise_scale, length_scale, self.noise_w], dtype=torch.float32)
        if "sid" in names:
            feeds["sid"] = torch.tensor([sid or 0], dtype=torch.int64)
        out = next(iter(self.runner.run(feeds).values()))
        return out.reshape(-1).float().cpu().numpy()

    def synthesize(self, text: str, speaker_id: Optional[int] = None, speaking_rate: Optional[float] = None,
                   seed: int = 0) -> np.ndarray:
        """Float audio in [-1, 1] at self.sampling_rate (piper's peak normalisation)."""
        self.generator.manual_seed(seed)
        ls = self.length_scale / speaking_rate if speaking_rate else self.length_scale
        gap = np.zeros(int(SENTENCE_SILENCE * self.sampling_rate), dtype=np.float32)
        parts: List[np.ndarray] = []
        for ph in self.phonemes(text):
            if parts:
                parts.append(gap)
            parts.append(self._utterance(self.ids(ph), speaker_id, ls))
        if not parts:
            return np.zeros(0, dtype=np.float32)
        audio = np.concatenate(parts)
        peak = max(0.01, float(np.abs(audio).max()))
        return (audio / peak).astype(np.float32)
