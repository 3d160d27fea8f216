"""Text-to-speech / sound-generation backend servicers (backend.proto LoadModel + TTS /
SoundGeneration) over the native audio models.

  piper / vits / mms-tts     VITS voices (models/tts.py; piper .onnx voices: models/piper.py)
                                                                 -- backend/go/tts/piper.go:30-49
  transformers-musicgen      MusicGen (models/musicgen.py)      -- backend/python/transformers-musicgen/backend.py:66,121
  bark                       Bark (models/bark.py)              -- backend/python/bark/backend.py:44
  parler-tts                 Parler-TTS (models/parler.py)      -- backend/python/parler-tts/backend.py:71-90

TTS writes a 16-bit PCM wav to `request.dst` and answers `Result(success=True)`, as the
reference backends do.  `voice` selects a speaker id of a multi-speaker VITS voice (a number) or
a Bark history prompt name, or a Parler-TTS speaker description; `language` is accepted and ignored (the voice fixes the language).
"""
from __future__ import annotations

import asyncio
import os
import threading

from . import backend_pb as pb


class _AudioBase:
    kind = "audio"

    def __init__(self, device: str = ""):
        self.device = device
        self.model = None
        self.state = pb.StatusResponse.UNINITIALIZED
        self._lock = threading.Lock()

    def _dev(self) -> str:
        if self.device:
            return self.device
        import torch
        return "cuda:0" if torch.cuda.is_available() else "cpu"

    async def Health(self, request, context=None):
        return pb.Reply(message=b"OK")

    async def Status(self, request, context=None):
        return pb.StatusResponse(state=self.state)

    def shutdown(self):
        self.model, self.state = None, pb.StatusResponse.UNINITIALIZED

    def _load(self, path: str):
        raise NotImplementedError

    async def LoadModel(self, request, context=None):
        path = request.ModelFile or request.Model
        try:
            m = await asyncio.get_running_loop().run_in_executor(None, self._load, path)
        except Exception as e:  # noqa: BLE001 - reported to the caller like the reference
            return pb.Result(success=False, message=f"{self.kind}: could not load {path}: {e}")
        self.model, self.state = m, pb.StatusResponse.READY
        return pb.Result(success=True, message="Model loaded successfully")

    async def TTS(self, request, context=None):
        return pb.Result(success=False, message=f"TTS is not supported by the {self.kind} backend")

    async def SoundGeneration(self, request, context=None):
        return pb.Result(success=False, message=f"SoundGeneration is not supported by the {self.kind} backend")

    async def _run(self, fn, *a):
        try:
            await asyncio.get_running_loop().run_in_executor(None, fn, *a)
        except Exception as e:  # noqa: BLE001
            return pb.Result(success=False, message=f"{self.kind}: {e}")
        return pb.Result(success=True, message="Media generated")


class VitsServicer(_AudioBase):
    """piper / vits / mms-tts voices."""
    kind = "vits"

    def _load(self, path):
        from ..models.tts import VitsVoice, is_vits_dir
        if path.endswith(".onnx"):  # a piper voice: <voice>.onnx + <voice>.onnx.json (models/piper.py)
            from ..models.piper import PiperVoice
            return PiperVoice(path, self._dev())
        if not is_vits_dir(path):
            raise ValueError("not a VITS checkpoint directory (config.json model_type 'vits')")
        return VitsVoice(path, self._dev())

    def _tts(self, request):
        from ..models.tts import write_wav
        v = self.model
        if v is None:
            raise RuntimeError("no model loaded")
        sid = int(request.voice) if request.voice.strip().isdigit() else None
        if hasattr(v, "speaker"):  # piper: speaker names from the voice's speaker_id_map
            sid = v.speaker(request.voice)
        with self._lock:
            audio = v.synthesize(request.text, speaker_id=sid)
        write_wav(request.dst, audio, v.sampling_rate)

    async def TTS(self, request, context=None):
        return await self._run(self._tts, request)


class MusicgenServicer(_AudioBase):
    """transformers-musicgen: SoundGeneration (and the older TTS entry point)."""
    kind = "transformers-musicgen"

    def _load(self, path):
        from ..models.musicgen import MusicGen, is_musicgen_dir
        if not is_musicgen_dir(path):
            raise ValueError("not a MusicGen checkpoint directory (config.json model_type 'musicgen')")
        return MusicGen(path, self._dev())

    def _sound(self, request, tts: bool):
        from ..models.tts import write_wav
        m = self.model
        if m is None:
            raise RuntimeError("no model loaded")
        if tts:
            tokens, guidance, sample = 512, 3.0, True     # backend.py TTS: 10 s, generation defaults
        else:
            tokens = int(request.duration * 51.2) if request.HasField("duration") else 256
            guidance = request.temperature if request.HasField("temperature") else 3.0
            sample = request.sample if request.HasField("sample") else True
        with self._lock:
            audio = m.generate(request.text, max_new_tokens=max(tokens, m.dec["num_codebooks"]),
                               guidance_scale=guidance, do_sample=sample)
        write_wav(request.dst, audio, m.sampling_rate)

    async def SoundGeneration(self, request, context=None):
        if request.HasField("src"):
            return pb.Result(success=False, message="audio-prompted generation (src) is not supported")
        return await self._run(self._sound, request, False)

    async def TTS(self, request, context=None):
        return await self._run(self._sound, request, True)


class BarkServicer(_AudioBase):
    """bark: TTS with an optional speaker preset (`voice`)."""
    kind = "bark"

    def _load(self, path):
        from ..models.bark import Bark, is_bark_dir
        if not is_bark_dir(path):
            raise ValueError("not a Bark checkpoint directory (config.json model_type 'bark')")
        return Bark(path, self._dev())

    def _tts(self, request):
        from ..models.tts import write_wav
        m = self.model
        if m is None:
            raise RuntimeError("no model loaded")
        with self._lock:
            audio = m.generate(request.text, voice=request.voice)
        write_wav(request.dst, audio, m.sampling_rate)

    async def TTS(self, request, context=None):
        return await self._run(self._tts, request)


class ParlerServicer(_AudioBase):
    """parler-tts: TTS where `voice` is the natural-language speaker description."""
    kind = "parler-tts"

    def _load(self, path):
        from ..models.parler import ParlerTTS, is_parler_dir
        if not is_parler_dir(path):
            raise ValueError("not a Parler-TTS checkpoint directory (config.json model_type 'parler_tts')")
        return ParlerTTS(path, self._dev())

    def _tts(self, request):
        from ..models.tts import write_wav
        m = self.model
        if m is None:
            raise RuntimeError("no model loaded")
        with self._lock:
            audio = m.generate(request.text, description=request.voice)
        write_wav(request.dst, audio, m.sampling_rate)

    async def TTS(self, request, context=None):
        return await self._run(self._tts, request)
