"""Native VITS text-to-speech (models/tts.py) and the piper / vits TTS backends.

Oracle: transformers' VitsModel (importable here) with the same random weights, saved in the
Hugging Face layout and loaded by our loader (weight-norm folding included); the same seed gives
the same waveform (stochastic and deterministic duration predictors, single- and multi-speaker).
"""
import json
import os
import wave

import numpy as np
import pytest
import torch

from localai_amd.models.tts import VitsTokenizer, VitsVoice, is_vits_dir, write_wav

transformers = pytest.importorskip("transformers")

VOCAB = "_ abcdefghijklmnopqrstuvwxyz'"


def make_voice(path, stochastic=True, speakers=1, seed=0):
    from transformers import VitsConfig, VitsModel
    cfg = VitsConfig(vocab_size=len(VOCAB), hidden_size=16, num_hidden_layers=2, num_attention_heads=2, window_size=2,
                     ffn_dim=24, flow_size=8, upsample_initial_channel=16, upsample_rates=[4, 2],
                     upsample_kernel_sizes=[8, 4], resblock_kernel_sizes=[3, 5], resblock_dilation_sizes=[[1, 3], [1, 3]],
                     duration_predictor_filter_channels=12, prior_encoder_num_wavenet_layers=2,
                     use_stochastic_duration_prediction=stochastic, num_speakers=speakers,
                     speaker_embedding_size=6 if speakers > 1 else 0, sampling_rate=8000)
    torch.manual_seed(seed)
    m = VitsModel(cfg).eval()
    m.save_pretrained(str(path))
    with open(os.path.join(path, "vocab.json"), "w") as f:
        json.dump({c: i for i, c in enumerate(VOCAB)}, f)
    with open(os.path.join(path, "tokenizer_config.json"), "w") as f:
        json.dump({"add_blank": True, "normalize": True, "pad_token": "_", "unk_token": "_"}, f)
    return m


@pytest.mark.parametrize("stochastic,speakers", [(True, 1), (False, 3), (True, 2)])
def test_vits_matches_transformers(tmp_path, stochastic, speakers):
    m = make_voice(tmp_path, stochastic, speakers)
    v = VitsVoice(str(tmp_path), "cpu")
    from transformers import VitsTokenizer as HFTok
    text = "Hello, World's voice!"
    ids = v.tok(text)
    assert ids == HFTok(vocab_file=str(tmp_path / "vocab.json"), add_blank=True, normalize=True,
                        phonemize=False, pad_token="_", unk_token="_")(text)["input_ids"]
    sid = 1 if speakers > 1 else None
    torch.manual_seed(11)
    with torch.no_grad():
        ref = m(torch.tensor([ids]), speaker_id=sid).waveform[0].numpy()
    out = v.synthesize(text, speaker_id=sid, seed=11)
    assert out.shape == ref.shape
    assert np.abs(out - ref).max() < 1e-4


def test_weight_norm_folding_legacy_names(tmp_path):
    """`weight_g` / `weight_v` (older checkpoints) fold to the same weights as the parametrization spelling."""
    from safetensors.torch import load_file, save_file
    make_voice(tmp_path)
    a = VitsVoice(str(tmp_path), "cpu")
    sd = load_file(str(tmp_path / "model.safetensors"))
    legacy = {}
    for k, t in sd.items():
        k = k.replace("parametrizations.weight.original0", "weight_g").replace("parametrizations.weight.original1",
                                                                              "weight_v")
        legacy[k] = t
    os.remove(tmp_path / "model.safetensors")
    torch.save(legacy, tmp_path / "pytorch_model.bin")
    b = VitsVoice(str(tmp_path), "cpu")
    assert a.W.keys() == b.W.keys()
    assert all(torch.equal(a.W[k], b.W[k]) for k in a.W)
    assert np.array_equal(a.synthesize("abc", seed=3), b.synthesize("abc", seed=3))


def test_tokenizer_and_wav(tmp_path):
    make_voice(tmp_path)
    tok = VitsTokenizer(str(tmp_path))
    assert tok("  AB? ") == [0, VOCAB.index("a"), 0, VOCAB.index("b"), 0]
    assert is_vits_dir(str(tmp_path)) and not is_vits_dir(str(tmp_path / "nope"))
    dst = tmp_path / "o" / "x.wav"
    write_wav(str(dst), np.array([0.0, 0.5, -1.5], dtype=np.float32), 8000)
    with wave.open(str(dst)) as w:
        assert (w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()) == (8000, 1, 2, 3)
        assert list(np.frombuffer(w.readframes(3), "<i2")) == [0, 16383, -32767]


def test_tts_endpoints(tmp_path):
    """/tts with no backend named (piper by default, core/backend/tts.go), /v1/audio/speech and the
    ElevenLabs route through the piper/vits backends; the answer is a wav of the voice's rate."""
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    make_voice(mdir / "voice-tiny", speakers=2)
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    bc = BackendConfig({"name": "speaker", "backend": "vits", "parameters": {"model": "voice-tiny"}})
    bc.set_defaults()
    st.configs.add(bc)
    import io
    with TestClient(create_app(st)) as c:
        for r in (c.post("/tts", json={"model": "voice-tiny", "input": "hello there"}),
                  c.post("/v1/audio/speech", json={"model": "speaker", "input": "hi", "voice": "1"}),
                  c.post("/v1/text-to-speech/1", json={"model_id": "speaker", "text": "hey"})):
            assert r.status_code == 200, r.text
            with wave.open(io.BytesIO(r.content)) as w:
                assert w.getframerate() == 8000 and w.getnframes() > 0
        assert {"piper", "vits"} <= set(c.get("/system").json()["backends"])
        r = c.post("/v1/audio/speech", json={"model": "speaker", "input": "hi", "voice": "7"})
        assert r.status_code == 500 and "speaker id" in r.text


@pytest.mark.gpu
def test_vits_on_gpu_matches_cpu(tmp_path):
    make_voice(tmp_path)
    a = VitsVoice(str(tmp_path), "cpu").synthesize("the quick brown fox", seed=5)
    b = VitsVoice(str(tmp_path), "cuda:0").synthesize("the quick brown fox", seed=5)
    assert a.shape == b.shape and np.abs(a - b).max() < 1e-2
