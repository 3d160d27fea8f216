"""Speech-to-text (the reference's whisper backend, backend/go/transcribe/whisper/whisper.go): the
whisper.cpp GGML format, the log-mel front end, greedy decoding, the AudioTranscription RPC and
POST /v1/audio/transcriptions end to end, on a random-init model (no checkpoints offline: the
transcript text itself is meaningless, its determinism and plumbing are what is checked)."""
import asyncio
import io
import wave

import numpy as np
import pytest
import torch

from localai_amd.models import synth
from localai_amd.models.whisper import (N_FRAMES, WhisperModel, is_whisper_ggml, load_audio, read_ggml)


@pytest.fixture(scope="module")
def wpath(tmp_path_factory):
    return synth.write_whisper(str(tmp_path_factory.mktemp("wh") / "ggml-tiny-random.bin"))


def _wav(path, seconds=2.0, rate=8000, channels=2):
    t = np.arange(int(seconds * rate)) / rate
    x = (0.3 * np.sin(2 * np.pi * 330 * t) * 32767).astype(np.int16)
    with wave.open(path, "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(np.repeat(x[:, None], channels, 1).tobytes())
    return path


def test_ggml_format_roundtrip(wpath):
    assert is_whisper_ggml(wpath)
    hp, filters, words, t = read_ggml(wpath)
    assert hp.n_vocab == 51865 and hp.n_mels == 80 and filters.shape == (80, 201)
    assert len(words) == 50256 and t["encoder.conv1.weight"].shape == (64, 80, 3)
    assert t["decoder.token_embedding.weight"].shape == (51865, 64) and t["encoder.conv1.bias"].shape == (64, 1)


def test_audio_loading_resamples_and_mixes(tmp_path):
    a = load_audio(_wav(str(tmp_path / "a.wav"), seconds=1.5, rate=8000, channels=2))
    assert a.dtype == np.float32 and abs(a.shape[0] - 24000) <= 2 and 0.2 < np.abs(a).max() < 0.35


def test_log_mel_and_transcribe_deterministic(wpath, tmp_path):
    m = WhisperModel(wpath, "cpu")
    audio = load_audio(_wav(str(tmp_path / "b.wav")))
    mel = m.log_mel(torch.from_numpy(audio))
    assert mel.shape == (80, N_FRAMES) and float(mel.max()) <= 2.0 and float(mel.max() - mel.min()) <= 2.0 + 1e-5
    # no-timestamp mode: one segment per 30-s window
    s1, text1 = m.transcribe(audio, max_tokens_per_window=12, timestamps=False)
    s2, text2 = m.transcribe(audio, max_tokens_per_window=12, timestamps=False)
    assert text1 == text2 and len(s1) == 1 and s1[0].tokens == s2[0].tokens and len(s1[0].tokens) >= 1
    assert s1[0].start_ns == 0 and s1[0].end_ns == 2 * 10 ** 9
    assert all(t < m.eot for t in s1[0].tokens)
    # explicit language and the translate task take other prompt tokens
    s3, _ = m.transcribe(audio, language="de", translate=True, max_tokens_per_window=12, timestamps=False)
    assert len(s3) == 1
    with pytest.raises(ValueError):
        m.transcribe(audio, language="xx")
    # > 30 s of audio: one segment per window
    long = np.concatenate([audio] * 16)
    s4, _ = m.transcribe(long, max_tokens_per_window=4, timestamps=False)
    assert [s.id for s in s4] == [0, 1] and s4[1].start_ns == 30 * 10 ** 9
    # timestamp mode (the default, as whisper.cpp): segments in order, inside the audio, text only
    for a, cap in ((audio, 24), (long, 16)):
        segs, text = m.transcribe(a, max_tokens_per_window=cap)
        again, _ = m.transcribe(a, max_tokens_per_window=cap)
        assert [s.tokens for s in segs] == [s.tokens for s in again]
        assert segs and [s.id for s in segs] == list(range(len(segs))) and text == "".join(s.text for s in segs)
        dur = int(a.shape[0] / 16000 * 1e9) + 1
        for x, y in zip(segs, segs[1:]):
            assert x.start_ns <= y.start_ns
        assert all(0 <= s.start_ns <= s.end_ns <= dur and all(t < m.eot for t in s.tokens) for s in segs)


def test_timestamp_rules_and_segments(wpath):
    """The decoding rules on synthetic logits and the segment split on synthetic token streams."""
    m = WhisperModel(wpath, "cpu")
    tb, V = m.timestamp_begin, m.hp.n_vocab
    lg = torch.zeros(V)
    m._timestamp_rules(lg, [])
    allowed = torch.isfinite(lg).nonzero().flatten().tolist()
    assert allowed == list(range(tb, tb + 51))                     # first token: a timestamp <= 1.00 s
    lg = torch.zeros(V)
    m._timestamp_rules(lg, [tb + 10, 300])
    # text after an opening timestamp: the closing one must be later (nonzero-length segment)
    assert torch.isinf(lg[tb:tb + 11]).all() and torch.isfinite(lg[tb + 11]) and torch.isinf(lg[m.no_timestamps])
    lg = torch.zeros(V)
    m._timestamp_rules(lg, [tb + 10, 300, tb + 40])               # pair open after text: close it
    assert torch.isinf(lg[:m.eot]).all() and torch.isfinite(lg[tb + 40])
    lg = torch.zeros(V)
    m._timestamp_rules(lg, [tb + 10, 300, tb + 40, tb + 40])      # pair complete: text next
    assert torch.isinf(lg[tb:]).all() and torch.isfinite(lg[300])
    lg = torch.full((V,), -5.0)
    lg[tb:] = 0.0                                                  # timestamps' mass beats any text token
    m._timestamp_rules(lg, [tb, 300])
    assert torch.isinf(lg[:tb]).all()
    # "<|0.00|> a b <|1.00|><|1.00|> c <|2.50|>" in a window starting at 30 s
    segs, seek = m.split_segments([tb, 11, 12, tb + 50, tb + 50, 13, tb + 125], 30.0, 30.0)
    assert [(a, b, t) for a, b, t in segs] == [(30.0, 31.0, [11, 12]), (31.0, 32.5, [13])]
    assert seek == pytest.approx(2.5)                              # ended on a lone timestamp: seek to it
    segs, seek = m.split_segments([tb, 11, tb + 50, tb + 50, 12], 0.0, 7.0)
    assert segs[-1] == (1.0, 7.0, [12]) and seek == 7.0            # unterminated: runs to the window end


def test_transcription_endpoint(wpath, tmp_path):
    import os
    import shutil
    from fastapi.testclient import TestClient
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    mdir.mkdir()
    shutil.copy(wpath, mdir / "ggml-tiny.bin")
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    ac.engine_mode = "inprocess"
    st = AppState(ac)
    bc = BackendConfig({"name": "whisper-1", "backend": "whisper", "parameters": {"model": "ggml-tiny.bin"}})
    bc.set_defaults()
    st.configs.add(bc)
    app = create_app(st)
    wav = open(_wav(str(tmp_path / "c.wav")), "rb").read()
    with TestClient(app) as c:
        r = c.post("/v1/audio/transcriptions", data={"model": "whisper-1", "language": "en"},
                   files={"file": ("c.wav", wav, "audio/wav")})
        assert r.status_code == 200, r.text
        j = r.json()
        assert j["segments"] and j["text"] == "".join(s["text"] for s in j["segments"])
        assert all(s["end"] <= 2 * 10 ** 9 + 1 and s["start"] <= s["end"] for s in j["segments"])
        assert [s["id"] for s in j["segments"]] == list(range(len(j["segments"])))


@pytest.mark.gpu
def test_whisper_on_gpu_matches_cpu(wpath, tmp_path):
    """The same model on the GPU (bf16 GEMMs through hipBLASLt): log-mel identical to fp32 tolerance,
    encoder output close, and a transcript produced through the AudioTranscription RPC."""
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    cpu, gpu = WhisperModel(wpath, "cpu"), WhisperModel(wpath, "cuda:0")
    audio = load_audio(_wav(str(tmp_path / "g.wav")))
    x = torch.from_numpy(audio)
    m0, m1 = cpu.log_mel(x), gpu.log_mel(x).cpu()
    assert (m0 - m1).abs().max().item() < 1e-3
    e0, e1 = cpu.encode(m0), gpu.encode(m1.cuda()).cpu()
    assert (e0 - e1).abs().max().item() < 0.1 * max(1.0, e0.abs().max().item())
    sv = EngineServicer(device="cuda:0")
    res = asyncio.run(sv.LoadModel(pb.ModelOptions(ModelFile=wpath, Model=wpath)))
    assert res.success, res.message
    out = asyncio.run(sv.AudioTranscription(pb.TranscriptRequest(dst=str(tmp_path / "g.wav"), language="en")))
    assert out.segments and out.text == "".join(s.text for s in out.segments)
