"""Native Parler-TTS (models/parler.py) and the `parler-tts` backend.

parler_tts is not importable here, so the oracles are its building blocks from transformers with
the same random weights: T5EncoderModel (description encoder), MusicgenForCausalLM (the Parler
decoder is MusicGen's decoder with the prompt embeddings prepended to its input sequence: it is run
teacher-forced on [embed_prompts(prompt) | codebook-embedding sums] with the full-length sinusoidal
table) and DacModel (the codec; the checkpoint stores it in the descript-audio-codec layout with
weight norm, which the loader maps back).  The generation loop's delay pattern / EOS bookkeeping is
checked against its rules directly; parity of the sampled path with parler_tts.generate is unpinned."""
import io
import json
import os
import wave

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from localai_amd.models.parler import ParlerTTS, dac_weights, is_parler_dir  # noqa: E402

CB, V, K = 32, 40, 3          # codebook size, decoder vocab (codes + specials), codebooks
PAD, BOS = 32, 33


def _to_dac_layout(sd, nb):
    """transformers DacModel names -> descript-audio-codec names with weight norm split."""
    out = {}
    g = torch.Generator().manual_seed(5)
    for k, v in sd.items():
        n = k
        if k.startswith("decoder."):
            r = k[len("decoder."):]
            if r.startswith("conv1."):
                n = "decoder.model.0." + r[len("conv1."):]
            elif r.startswith("snake1."):
                n = f"decoder.model.{nb + 1}." + r[len("snake1."):]
            elif r.startswith("conv2."):
                n = f"decoder.model.{nb + 2}." + r[len("conv2."):]
            else:
                parts = r.split(".")                      # block.b.<mod>.(...)
                b, mod, rest = int(parts[1]), parts[2], parts[3:]
                base = f"decoder.model.{b + 1}.block."
                if mod == "snake1":
                    n = base + "0." + ".".join(rest)
                elif mod == "conv_t1":
                    n = base + "1." + ".".join(rest)
                else:
                    j = int(mod[len("res_unit"):])
                    sub = {"snake1": 0, "conv1": 1, "snake2": 2, "conv2": 3}[rest[0]]
                    n = base + f"{j + 1}.block.{sub}." + ".".join(rest[1:])
        if n.endswith(".weight") and v.dim() == 3:
            norm = v.reshape(v.shape[0], -1).norm(dim=1).reshape(-1, 1, 1)
            scale = torch.rand(v.shape[0], 1, 1, generator=g) + 0.5
            out["model." + n[:-len("weight")] + "weight_g"] = norm
            out["model." + n[:-len("weight")] + "weight_v"] = v * scale
        else:
            out["model." + n] = v
    return out


def make_parler(path, dac_layout="dac", gen=None):
    """Random Parler-TTS checkpoint; returns the transformers oracles (t5, decoder, dac, embed_prompts, proj)."""
    from safetensors.torch import save_file
    from transformers import (DacConfig, DacModel, MusicgenDecoderConfig, MusicgenForCausalLM, T5Config,
                              T5EncoderModel)

    from localai_amd.models.synth import _t5_byte_tokenizer
    os.makedirs(path, exist_ok=True)
    n_t5 = _t5_byte_tokenizer(str(path))
    torch.manual_seed(0)
    t5c = T5Config(vocab_size=n_t5, d_model=24, d_kv=8, d_ff=32, num_layers=2, num_heads=3,
                   feed_forward_proj="gated-gelu")
    t5 = T5EncoderModel(t5c).eval()
    dc = MusicgenDecoderConfig(vocab_size=V, hidden_size=32, num_hidden_layers=2, ffn_dim=48, num_attention_heads=4,
                               num_codebooks=K, pad_token_id=PAD, bos_token_id=BOS, max_position_embeddings=256)
    dec = MusicgenForCausalLM(dc).eval()
    ac = DacConfig(encoder_hidden_size=8, downsampling_ratios=[2, 4], decoder_hidden_size=32, upsampling_ratios=[4, 2],
                   n_codebooks=K, codebook_size=CB, codebook_dim=4, hidden_size=16, sampling_rate=16000)
    dac = DacModel(ac).eval()
    emb_prompts = torch.randn(n_t5, 32) * 0.5
    proj_w, proj_b = torch.randn(32, 24) * 0.2, torch.randn(32) * 0.1
    sd = {"text_encoder." + k: v for k, v in t5.state_dict().items()}
    sd.update({"decoder." + k: v for k, v in dec.state_dict().items()})
    dsd = dac.state_dict()
    if dac_layout == "dac":
        dsd = _to_dac_layout(dsd, len(ac.upsampling_ratios))
    sd.update({"audio_encoder." + k: v for k, v in dsd.items()})
    sd.update({"embed_prompts.weight": emb_prompts, "enc_to_dec_proj.weight": proj_w, "enc_to_dec_proj.bias": proj_b})
    save_file({k: v.detach().clone().contiguous() for k, v in sd.items()}, os.path.join(path, "model.safetensors"))
    cfg = {"model_type": "parler_tts", "vocab_size": n_t5, "text_encoder": t5c.to_dict(),
           "audio_encoder": {"model_type": "dac_on_the_hub", "codebook_size": CB, "num_codebooks": K,
                             "latent_dim": 16, "sampling_rate": 16000},
           "decoder": dict(dc.to_dict(), model_type="parler_tts_decoder", eos_token_id=PAD)}
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(cfg, f)
    g = {"do_sample": True, "max_length": 40, "min_new_tokens": 4, "decoder_start_token_id": BOS,
         "bos_token_id": BOS, "pad_token_id": PAD, "eos_token_id": PAD}
    g.update(gen or {})
    with open(os.path.join(path, "generation_config.json"), "w") as f:
        json.dump(g, f)
    return t5, dec, dac, emb_prompts, (proj_w, proj_b)


@pytest.mark.parametrize("layout", ["dac", "hf"])
def test_dac_decoder_matches_transformers(tmp_path, layout):
    _, _, dac, _, _ = make_parler(tmp_path, layout)
    from safetensors.torch import load_file
    from localai_amd.models.parler import DacDecoder
    codec = DacDecoder(dac_weights(load_file(str(tmp_path / "model.safetensors")), "audio_encoder."), "cpu")
    codes = torch.randint(0, CB, (K, 7))
    with torch.no_grad():
        ref = dac.decode(audio_codes=codes[None]).audio_values.reshape(-1)
    wav = codec(codes)
    assert codec.hop == 8 and wav.shape == ref.shape
    assert (wav - ref).abs().max() < 1e-5


def test_parler_decoder_matches_musicgen_teacher_forced(tmp_path):
    t5, dec, _, emb_prompts, (pw, pb_) = make_parler(tmp_path)
    assert is_parler_dir(str(tmp_path))
    m = ParlerTTS(str(tmp_path), "cpu")
    desc = m.tokenize("a calm voice")
    prompt = m.tokenize("hello there")
    with torch.no_grad():
        enc_ref = t5(input_ids=desc).last_hidden_state[0] @ pw.t() + pb_
    assert (m.encode_description(desc) - enc_ref).abs().max() < 1e-5
    n = 14
    seq, codes = m.generate_codes(desc, prompt, n, do_sample=False, ignore_eos=True)
    assert seq.shape == (K, n + 1)
    # delay pattern: BOS upper-left triangle, PAD lower-right triangle of the n + 1 columns
    for k in range(K):
        assert (seq[k, :k + 1] == BOS).all() and (seq[k, n + 1 - K + 1 + k:] == PAD).all()
    # teacher-forced oracle over [prompt | frames 0..n-1]
    audio = sum(dec.model.decoder.embed_tokens[k](seq[k, :-1]) for k in range(K))
    x = torch.cat([emb_prompts[prompt[0]], audio], 0)[None]
    S = x.shape[1]
    table = dec.model.decoder.embed_positions.weights[:S]
    dec.model.decoder.embed_positions.forward = lambda input, past_key_values_length=0: table
    with torch.no_grad():
        logits = dec(inputs_embeds=x, encoder_hidden_states=enc_ref[None]).logits.reshape(K, S, -1)
    P = prompt.shape[1]
    pred = logits[:, P:].argmax(-1)                                                      # predicts seq[:, 1:]
    kk = torch.arange(K)[:, None]
    tt = torch.arange(1, n + 1)[None]
    free = ~((tt <= kk) | (tt >= n + 1 - K + 1 + kk))
    assert free.sum() > 20 and torch.equal(pred[free], seq[:, 1:][free])
    # un-delayed frames: codebook k's frame f at column f + k + 1
    nf = n + 1 - K
    grid = torch.stack([seq[k, k + 1:k + 1 + nf] for k in range(K)])
    assert torch.equal(codes, grid[:, (grid < CB).all(0)])


def test_parler_eos_and_sampling(tmp_path):
    make_parler(tmp_path)
    m = ParlerTTS(str(tmp_path), "cpu")
    desc, prompt = m.tokenize("x"), m.tokenize("y z")
    # bias the heads so codebook 0 says EOS as soon as min_new_tokens allows
    m._heads[0, :, :] = 0
    with torch.no_grad():
        m.W["decoder.model.decoder.layer_norm.bias"].fill_(1.0)
        m._heads[0, PAD, :] = 1.0
    seq, codes = m.generate_codes(desc, prompt, 30, do_sample=False)
    assert (seq[0, 1:5] != PAD).all()                         # min_new_tokens = 4 suppresses EOS
    assert seq[0, 5] == PAD and (seq[0, 5:] == PAD).all()     # finished codebook stays on PAD
    assert codes.shape[1] <= 4 and (codes < CB).all()
    a = m.generate("hello", "calm", max_new_tokens=12, do_sample=True, seed=3)
    b = m.generate("hello", "calm", max_new_tokens=12, do_sample=True, seed=3)
    assert np.array_equal(a, b)


def test_parler_backend_tts_endpoint(tmp_path):
    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    make_parler(tmp_path / "models" / "pt", gen={"max_length": 24})
    ac = ApplicationConfig(models_path=str(tmp_path / "models"), upload_dir=str(tmp_path / "up"),
                           config_dir=str(tmp_path / "cfg"), image_dir=str(tmp_path / "img"),
                           audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    bc = BackendConfig({"name": "parler", "backend": "parler-tts", "parameters": {"model": "pt"}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/tts", json={"model": "parler", "input": "hello world", "voice": "a deep male voice"})
        assert r.status_code == 200, r.text
        with wave.open(io.BytesIO(r.content)) as w:
            assert w.getframerate() == 16000
        assert "parler-tts" in c.get("/system").json()["backends"]


@pytest.mark.gpu
def test_parler_graph_decode_on_gpu(tmp_path):
    make_parler(tmp_path)
    c = ParlerTTS(str(tmp_path), "cpu")
    g = ParlerTTS(str(tmp_path), "cuda:0")
    e = ParlerTTS(str(tmp_path), "cuda:0", use_graphs=False)
    assert g.use_graphs
    desc, prompt = c.tokenize("a calm voice"), c.tokenize("hello there")
    sc, _ = c.generate_codes(desc, prompt, 20, do_sample=False, ignore_eos=True)
    sg, _ = g.generate_codes(desc.cuda(), prompt.cuda(), 20, do_sample=False, ignore_eos=True)
    se, _ = e.generate_codes(desc.cuda(), prompt.cuda(), 20, do_sample=False, ignore_eos=True)
    assert torch.equal(sg.cpu(), se.cpu())                    # graph replay == eager on the device
    assert (sg.cpu() == sc).float().mean() > 0.8              # bf16 device vs fp32 host (greedy drift)
    a = g.generate("hello", "calm", max_new_tokens=16, seed=4)
    b = g.generate("hello", "calm", max_new_tokens=16, seed=4)
    assert np.array_equal(a, b) and np.isfinite(a).all()
