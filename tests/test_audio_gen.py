"""Native MusicGen (models/musicgen.py) and Bark (models/bark.py), and their backends.

Oracles: transformers' MusicgenForConditionalGeneration and BarkModel (importable here) with the
same random weights saved in the Hugging Face layout.  Greedy decoding makes every stage
deterministic, so the T5 states, the delay-pattern code grid, Bark's semantic / coarse / fine
tokens and the EnCodec waveforms are compared exactly (to fp32 rounding)."""
import io
import json
import os
import wave

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from localai_amd.models.bark import Bark  # noqa: E402
from localai_amd.models.musicgen import MusicGen, t5_bucket  # noqa: E402


def make_musicgen(path, channels=1, gated=False):
    from transformers import (EncodecConfig, MusicgenConfig, MusicgenDecoderConfig, MusicgenForConditionalGeneration,
                              T5Config)
    t5 = T5Config(vocab_size=50, d_model=24, d_kv=8, d_ff=32, num_layers=2, num_heads=3,
                  feed_forward_proj="gated-gelu" if gated else "relu")
    ec = EncodecConfig(hidden_size=16, num_filters=4, upsampling_ratios=[4, 2], codebook_size=32, sampling_rate=8000,
                       target_bandwidths=[40.0])
    K = 4 if channels == 1 else 8
    dc = MusicgenDecoderConfig(vocab_size=32, hidden_size=32, num_hidden_layers=2, ffn_dim=48, num_attention_heads=4,
                               num_codebooks=K, audio_channels=channels, pad_token_id=32, bos_token_id=32,
                               decoder_start_token_id=32, max_position_embeddings=128)
    cfg = MusicgenConfig(text_encoder=t5.to_dict(), audio_encoder=ec.to_dict(), decoder=dc.to_dict())
    torch.manual_seed(0)
    m = MusicgenForConditionalGeneration(cfg).eval()
    with torch.no_grad():
        for layer in m.audio_encoder.quantizer.layers:
            layer.codebook.embed.normal_()
    m.save_pretrained(str(path))
    return m


def make_tokenizer(path, words):
    from tokenizers import Tokenizer
    from tokenizers.models import WordLevel
    from tokenizers.pre_tokenizers import Whitespace
    vocab = {"[PAD]": 0, "[UNK]": 1}
    vocab.update({w: i + 2 for i, w in enumerate(words)})
    tok = Tokenizer(WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = Whitespace()
    tok.save(os.path.join(path, "tokenizer.json"))
    return vocab


def test_t5_bucket_matches_reference():
    from transformers.models.t5.modeling_t5 import T5Attention
    rel = torch.arange(-300, 300)[None, :] - torch.zeros(1, 1, dtype=torch.long)
    ref = T5Attention._relative_position_bucket(rel, bidirectional=True, num_buckets=32, max_distance=128)
    assert torch.equal(t5_bucket(rel, 32, 128), ref)


@pytest.mark.parametrize("channels,gated", [(1, False), (2, True)])
def test_musicgen_matches_transformers(tmp_path, channels, gated):
    m = make_musicgen(tmp_path, channels, gated)
    mg = MusicGen(str(tmp_path), "cpu")
    ids = torch.tensor([[5, 7, 9, 11, 1]])
    with torch.no_grad():
        ref_h = m.text_encoder(input_ids=ids).last_hidden_state
        ref = m.generate(input_ids=ids, attention_mask=torch.ones_like(ids), do_sample=False, guidance_scale=3.0,
                         max_new_tokens=14)
    assert (mg.text(ids) - ref_h).abs().max() < 1e-5
    codes = mg.generate_codes(ids, 14, 3.0, do_sample=False)
    assert codes.shape == (mg.dec["num_codebooks"], 15 - 4)
    if channels == 1:
        wav = mg.codec(codes)
    else:
        wav = torch.cat([mg.codec(codes[0::2]), mg.codec(codes[1::2])], 0)
    assert wav.shape == ref[0].shape
    assert (wav - ref[0]).abs().max() < 1e-5


def test_musicgen_unconditional_and_sampling(tmp_path):
    make_musicgen(tmp_path)
    make_tokenizer(str(tmp_path), ["lofi", "beat"])
    mg = MusicGen(str(tmp_path), "cpu")
    a = mg.generate("", max_new_tokens=10, do_sample=True, seed=1)
    b = mg.generate("lofi beat", max_new_tokens=10, do_sample=True, seed=1)
    c = mg.generate("lofi beat", max_new_tokens=10, do_sample=True, seed=1)
    assert a.ndim == 1 and a.shape == b.shape and np.array_equal(b, c) and np.isfinite(b).all()


def make_bark(path):
    from transformers import BarkCoarseConfig, BarkConfig, BarkFineConfig, BarkModel, BarkSemanticConfig, EncodecConfig
    sub = dict(block_size=1024, num_layers=2, num_heads=2, hidden_size=16)
    cfg = BarkConfig(
        semantic_config=BarkSemanticConfig(input_vocab_size=129600, output_vocab_size=10048, **sub).to_dict(),
        coarse_acoustics_config=BarkCoarseConfig(input_vocab_size=12096, output_vocab_size=12096, **sub).to_dict(),
        fine_acoustics_config=BarkFineConfig(input_vocab_size=1056, output_vocab_size=1056, n_codes_total=8,
                                             n_codes_given=1, **sub).to_dict(),
        codec_config=EncodecConfig(hidden_size=16, num_filters=4, upsampling_ratios=[4, 2], codebook_size=1024,
                                   sampling_rate=8000, target_bandwidths=[80.0]).to_dict())
    torch.manual_seed(0)
    m = BarkModel(cfg).eval()
    with torch.no_grad():
        for layer in m.codec_model.quantizer.layers:
            layer.codebook.embed.normal_()
    m.save_pretrained(str(path))
    return m


def test_bark_matches_transformers(tmp_path):
    from transformers.models.bark.generation_configuration_bark import (BarkCoarseGenerationConfig,
                                                                         BarkFineGenerationConfig,
                                                                         BarkSemanticGenerationConfig)
    m = make_bark(tmp_path)
    b = Bark(str(tmp_path), "cpu")
    sg, cg, fg = BarkSemanticGenerationConfig(max_new_tokens=20), BarkCoarseGenerationConfig(), BarkFineGenerationConfig()
    ids = [101, 2000, 3000, 4000]
    with torch.no_grad():
        s_ref = m.semantic.generate(torch.tensor([ids + [0] * (256 - len(ids))]), semantic_generation_config=sg,
                                    attention_mask=torch.tensor([[1] * len(ids) + [0] * (256 - len(ids))]))
        c_ref = m.coarse_acoustics.generate(s_ref.clone(), semantic_generation_config=sg, coarse_generation_config=cg,
                                            codebook_size=1024)
        f_ref = m.fine_acoustics.generate(c_ref.clone(), semantic_generation_config=sg, coarse_generation_config=cg,
                                          fine_generation_config=fg, codebook_size=1024)
        a_ref = m.codec_decode(f_ref)
    s = b.semantic_tokens(ids, None, 20)
    assert torch.equal(s, s_ref[0])
    c = b.coarse_tokens(s)
    assert torch.equal(c, c_ref[0])
    f = b.fine_tokens(c)
    assert torch.equal(f, f_ref[0])
    assert (b.codec(f) - a_ref).abs().max() < 1e-5


def test_bark_voice_preset_history(tmp_path):
    """A speaker preset (semantic / coarse / fine prompts, .npz read without pickle) conditions all
    three stages; the reference's history handling (trim + 2-token alignment) matches."""
    from transformers.models.bark.generation_configuration_bark import (BarkCoarseGenerationConfig,
                                                                         BarkFineGenerationConfig,
                                                                         BarkSemanticGenerationConfig)
    m = make_bark(tmp_path)
    rng = np.random.default_rng(0)
    prompts = {"semantic_prompt": rng.integers(0, 10000, 90), "coarse_prompt": rng.integers(0, 1024, (2, 270)),
               "fine_prompt": rng.integers(0, 1024, (8, 270))}
    np.savez(tmp_path / "spk.npz", **prompts)
    b = Bark(str(tmp_path), "cpu")
    hist = b.history(str(tmp_path / "spk.npz"))
    th = {k: torch.as_tensor(v) for k, v in prompts.items()}
    sg, cg, fg = BarkSemanticGenerationConfig(max_new_tokens=12), BarkCoarseGenerationConfig(), BarkFineGenerationConfig()
    ids = [7, 8, 9]
    with torch.no_grad():
        s_ref = m.semantic.generate(torch.tensor([ids + [0] * 253]), semantic_generation_config=sg, history_prompt=th,
                                    attention_mask=torch.tensor([[1] * 3 + [0] * 253]))
        c_ref = m.coarse_acoustics.generate(s_ref.clone(), semantic_generation_config=sg, coarse_generation_config=cg,
                                            codebook_size=1024, history_prompt=th)
        f_ref = m.fine_acoustics.generate(c_ref.clone(), semantic_generation_config=sg, coarse_generation_config=cg,
                                          fine_generation_config=fg, codebook_size=1024, history_prompt=th)
    s = b.semantic_tokens(ids, hist, 12)
    c = b.coarse_tokens(s, hist)
    f = b.fine_tokens(c, hist)
    assert torch.equal(s, s_ref[0]) and torch.equal(c, c_ref[0]) and torch.equal(f, f_ref[0])


def _state(tmp_path, configs):
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.state import AppState
    ac = ApplicationConfig(models_path=str(tmp_path / "models"), upload_dir=str(tmp_path / "up"),
                           config_dir=str(tmp_path / "cfg"), image_dir=str(tmp_path / "img"),
                           audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    for c in configs:
        bc = BackendConfig(c)
        bc.set_defaults()
        st.configs.add(bc)
    return st


def test_sound_generation_and_bark_endpoints(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.gateway.app import create_app
    make_musicgen(tmp_path / "models" / "mg")
    make_tokenizer(str(tmp_path / "models" / "mg"), ["lofi", "beat"])
    make_bark(tmp_path / "models" / "bk")
    make_tokenizer(str(tmp_path / "models" / "bk"), ["hello", "world"])
    st = _state(tmp_path, [{"name": "music", "backend": "transformers-musicgen", "parameters": {"model": "mg"}},
                           {"name": "speech", "backend": "bark", "parameters": {"model": "bk"}}])
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/sound-generation", json={"model_id": "music", "text": "lofi beat", "duration_seconds": 0.3})
        assert r.status_code == 200, r.text
        with wave.open(io.BytesIO(r.content)) as w:
            assert w.getframerate() == 8000 and w.getnframes() > 0
        r = c.post("/tts", json={"model": "speech", "input": "hello world"})
        assert r.status_code == 200, r.text
        with wave.open(io.BytesIO(r.content)) as w:
            assert w.getframerate() == 24000
        assert {"bark", "transformers-musicgen"} <= set(c.get("/system").json()["backends"])
        r = c.post("/tts", json={"model": "speech", "input": "hi", "voice": "nope"})
        assert r.status_code == 500 and "unknown Bark voice" in r.text


@pytest.mark.gpu
def test_musicgen_and_bark_on_gpu_match_cpu(tmp_path):
    make_musicgen(tmp_path / "mg")
    make_bark(tmp_path / "bk")
    ids = torch.tensor([[5, 7, 9, 11, 1]])
    a = MusicGen(str(tmp_path / "mg"), "cpu").generate_codes(ids, 12, 3.0, do_sample=False)
    g = MusicGen(str(tmp_path / "mg"), "cuda:0").generate_codes(ids.cuda(), 12, 3.0, do_sample=False)
    assert torch.equal(a, g.cpu())
    bc, bg = Bark(str(tmp_path / "bk"), "cpu"), Bark(str(tmp_path / "bk"), "cuda:0")
    s = bc.semantic_tokens([3, 4, 5], None, 10)
    assert torch.equal(s, bg.semantic_tokens([3, 4, 5], None, 10).cpu())
    f = bc.fine_tokens(bc.coarse_tokens(s))
    wc, wg = bc.codec(f), bg.codec(f.cuda()).cpu()
    assert (wc - wg).abs().max() < 1e-3
