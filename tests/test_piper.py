"""Piper `.onnx` voices (models/piper.py) on the ONNX graph executor (utils/onnx_runtime.py).

Oracle: transformers' VitsModel exported to ONNX with torch's TorchScript exporter (the way
piper exports its voices), noise scales 0 so the waveform is deterministic; our executor must
reproduce it for prompt lengths other than the traced one (dynamic shapes through the duration
predictor).  Real piper voices (espeak phonemes, onnxruntime) are not available here: parity
with them is unpinned.
"""
import io
import json
import wave

import numpy as np
import pytest
import torch

from localai_amd.utils.onnx_proto import Node, encode_model, load_model
from localai_amd.utils.onnx_runtime import OnnxRunner

pytest.importorskip("transformers")


def _run(nodes, inits, inputs, outputs, feeds, opset=15):
    return OnnxRunner(load_model(encode_model(nodes, inits, inputs, outputs, opset=opset))).run(feeds)


def test_proto_roundtrip_tensors_and_attributes():
    w = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    i = np.array([-1, 5], dtype=np.int64)
    n = Node("Conv", ["x", "w"], ["y"], {"pads": [1, 1], "group": 1, "alpha": 0.5, "mode": "reflect",
                                         "value": np.array(3, dtype=np.int64)})
    m = load_model(encode_model([n], {"w": w, "i": i}, ["x"], ["y"], opset=17))
    assert m.opset == 17 and m.graph.inputs == ["x"] and m.graph.outputs == ["y"]
    assert np.array_equal(m.graph.initializers["w"], w) and np.array_equal(m.graph.initializers["i"], i)
    a = m.graph.nodes[0].attrs
    assert a["pads"] == [1, 1] and a["group"] == 1 and abs(a["alpha"] - 0.5) < 1e-7 and a["mode"] == b"reflect"
    assert a["value"].shape == () and int(a["value"]) == 3


def test_ops_against_torch():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 9, generator=g)
    w = torch.randn(6, 2, 3, generator=g)
    b = torch.randn(6, generator=g)
    out = _run([Node("Conv", ["x", "w", "b"], ["y"], {"pads": [2, 1], "dilations": [2], "group": 2, "strides": [1],
                                                     "kernel_shape": [3]})],
               {"w": w.numpy(), "b": b.numpy()}, ["x"], ["y"], {"x": x})["y"]
    ref = torch.nn.functional.conv1d(torch.nn.functional.pad(x, (2, 1)), w, b, dilation=2, groups=2)
    assert torch.allclose(out, ref, atol=1e-5)
    wt = torch.randn(4, 3, 4, generator=g)
    out = _run([Node("ConvTranspose", ["x", "w"], ["y"], {"strides": [2], "pads": [1, 1]})],
               {"w": wt.numpy()}, ["x"], ["y"], {"x": x})["y"]
    assert torch.allclose(out, torch.nn.functional.conv_transpose1d(x, wt, stride=2, padding=1), atol=1e-5)
    # shape arithmetic: Shape -> Gather (scalar) -> Unsqueeze -> Concat -> Reshape (0 = copy)
    nodes = [Node("Shape", ["x"], ["s"]), Node("Gather", ["s", "i1"], ["d1"], {"axis": 0}),
             Node("Unsqueeze", ["d1", "a0"], ["u"]), Node("Concat", ["z", "u", "m1"], ["shp"], {"axis": 0}),
             Node("Reshape", ["x", "shp"], ["y"])]
    y = _run(nodes, {"i1": np.array(1, np.int64), "a0": np.array([0], np.int64), "z": np.array([0], np.int64),
                     "m1": np.array([-1], np.int64)}, ["x"], ["y"], {"x": x})["y"]
    assert y.shape == (2, 4, 9)
    # Slice with negative step, CumSum exclusive+reverse, Pad reflect, Where / NonZero / GatherND / ScatterND
    v = torch.arange(10.0).reshape(2, 5)
    y = _run([Node("Slice", ["v", "st", "en", "ax", "sp"], ["y"])],
             {"st": np.array([-1], np.int64), "en": np.array([-100], np.int64), "ax": np.array([1], np.int64),
              "sp": np.array([-2], np.int64)}, ["v"], ["y"], {"v": v})["y"]
    assert torch.equal(y, v.flip(1)[:, ::2])
    y = _run([Node("CumSum", ["v", "ax"], ["y"], {"exclusive": 1, "reverse": 1})],
             {"ax": np.array(1, np.int64)}, ["v"], ["y"], {"v": v})["y"]
    assert torch.equal(y, v.flip(1).cumsum(1).flip(1) - v)
    y = _run([Node("Pad", ["v", "p"], ["y"], {"mode": "reflect"})],
             {"p": np.array([0, 0, 2, 0, 0, 1], np.int64)}, ["v"], ["y"], {"v": v.unsqueeze(0)})["y"]
    assert torch.equal(y, torch.nn.functional.pad(v.unsqueeze(0), (2, 1), mode="reflect"))
    c = torch.tensor([[True, False, True], [False, True, False]])
    r = _run([Node("NonZero", ["c"], ["nz"]), Node("Transpose", ["nz"], ["idx"], {"perm": [1, 0]}),
              Node("GatherND", ["d", "idx"], ["g"]), Node("ScatterND", ["d", "idx", "g2"], ["s"]),
              Node("Where", ["c", "d", "zero"], ["wh"])],
             {"zero": np.zeros((), np.float32), "g2": -np.ones(3, np.float32)}, ["c", "d"], ["g", "s", "wh"],
             {"c": c, "d": torch.arange(6.0).reshape(2, 3)})
    assert r["g"].tolist() == [0.0, 2.0, 4.0]
    assert r["s"].tolist() == [[-1.0, 1.0, -1.0], [3.0, -1.0, 5.0]]
    assert r["wh"].tolist() == [[0.0, 0.0, 2.0], [0.0, 4.0, 0.0]]
    with pytest.raises(NotImplementedError):
        OnnxRunner(load_model(encode_model([Node("Loop", ["x"], ["y"])], {}, ["x"], ["y"])))


@pytest.fixture(scope="module")
def voice(tmp_path_factory):
    from localai_amd.models import synth
    d = tmp_path_factory.mktemp("piper")
    path = str(d / "en-test-x_low.onnx")
    m = synth.write_piper_voice(path, seed=3)
    return path, m


def test_piper_voice_matches_transformers_vits(voice):
    from localai_amd.models.piper import PiperVoice, is_piper_voice
    path, m = voice
    assert is_piper_voice(path)
    v = PiperVoice(path, "cpu")
    for text in ("hello world", "a quick test of the voice, with more phonemes than the trace"):
        (ph,) = v.phonemes(text)
        ids = v.ids(ph)
        sym = json.load(open(path + ".json"))["phoneme_id_map"]
        assert ids[:2] == sym["^"] + sym["_"] and ids[-1] == sym["$"][0] and ids[3] == sym["_"][0]
        with torch.no_grad():
            ref = m(input_ids=torch.tensor([ids])).waveform[0].numpy()
        raw = v._utterance(ids, None, 1.0)
        assert raw.shape == ref.shape
        assert np.abs(raw - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())
    # two sentences: joined with 0.2 s of silence, peak-normalised
    a = v.synthesize("hello. world!")
    n1 = v._utterance(v.ids(v.phonemes("hello.")[0]), None, 1.0).shape[0]
    gap = int(0.2 * v.sampling_rate)
    assert np.all(a[n1:n1 + gap] == 0) and abs(np.abs(a).max() - 1.0) < 1e-6


def test_piper_tts_endpoint(voice, tmp_path):
    """/tts with no backend named -> piper (core/backend/tts.go) on a `.onnx` voice in the models dir."""
    import shutil

    from fastapi.testclient import TestClient

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    path, _ = voice
    mdir = tmp_path / "models"
    mdir.mkdir()
    shutil.copy(path, mdir / "en-test-x_low.onnx")
    shutil.copy(path + ".json", mdir / "en-test-x_low.onnx.json")
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    with TestClient(create_app(AppState(ac))) as c:
        r = c.post("/tts", json={"model": "en-test-x_low.onnx", "input": "Hi, this is a test."})
        assert r.status_code == 200, r.text
        with wave.open(io.BytesIO(r.content)) as w:
            assert w.getframerate() == 8000 and w.getnframes() > 0


@pytest.mark.gpu
def test_piper_voice_on_gpu_matches_cpu(voice):
    from localai_amd.models.piper import PiperVoice
    path, _ = voice
    a = PiperVoice(path, "cpu").synthesize("the quick brown fox")
    b = PiperVoice(path, "cuda:0").synthesize("the quick brown fox")
    assert a.shape == b.shape and np.abs(a - b).max() < 1e-3


# the symbol inventory of piper's espeak-ng voices (the keys of their phoneme_id_map)
_ESPEAK_SYMBOLS = set("_^$ !'(),-.:;?abcdefhijklmnopqrstuvwxyzæçðøħŋœǀǁǂǃɐɑɒɓɔɕɖɗɘəɚɛɜɞɟɠɡɢɣɤɥɦɧɨɪɫɬɭɮɯɰɱɲɳɴɵɶɸɹɺɻɽɾʀʁʂʃʄʈʉʊʋʌʍʎʏʐʑʒʔʕʘʙʛʜʝʟʡʢʲˈˌːˑ˞βθχᵻⱱ0123456789\"#↓↑")


def test_g2p_english_espeak_style():
    """espeak-type piper voices (reference backend/go/tts/piper.go:20-49 phonemises through
    espeak-ng) get en-us IPA from the rule-based front end: dictionary readings of common words,
    letter-to-sound rules with stress and the en-us flap, numbers read out, and every emitted
    phoneme inside the espeak voices' inventory.  Parity with espeak-ng itself is unpinned."""
    from localai_amd.models.g2p_en import fold, phonemize
    assert phonemize("Hello world!") == "həlˈoʊ wˈɜːld!"
    assert phonemize("This is a test.") == "ðɪs ɪz ɐ tˈɛst."
    rules = {"cat": "kˈæt", "phone": "fˈoʊn", "sing": "sˈɪŋ", "nation": "nˈeɪʃən", "school": "skˈuːl",
             "night": "nˈaɪt", "jumped": "dʒˈʌmpt", "fishes": "fˈɪʃɪz", "better": "bˈɛɾɚ", "dogs": "dˈɑːɡz",
             "information": "ɪnfɚmˈeɪʃən", "21": "twˈɛnti wˈʌn"}
    for w, ipa in rules.items():
        assert phonemize(w) == ipa, (w, phonemize(w))
    text = ("The quick brown fox jumps over the lazy dog. She sells 42 sea shells by the sea shore; "
            "LocalAI serves OpenAI-compatible requests & streams tokens (quickly)!")
    ipa = phonemize(text)
    assert set(ipa) <= _ESPEAK_SYMBOLS, set(ipa) - _ESPEAK_SYMBOLS
    # a voice without r-coloured schwa or length marks gets them folded onto what it has
    small = {"ə": [1], "ɹ": [2], "t": [3], "ˈ": [4], "b": [5], "ɛ": [6], "ɾ": [7]}
    assert fold(list("bˈɛɾɚ"), small) == ["b", "ˈ", "ɛ", "ɾ", "ə", "ɹ"]
    assert fold(list("tːɾ"), {"t": [1]}) == ["t", "t"]


def test_piper_espeak_voice_uses_g2p(voice):
    from localai_amd.models.g2p_en import fold, phonemize
    from localai_amd.models.piper import PiperVoice
    path, _ = voice
    v = PiperVoice(path, "cpu")
    v.phoneme_type = "espeak"
    (ph,) = v.phonemes("hello world")
    assert ph == fold(list(phonemize("hello world")), v.id_map)
    (raw,) = v.phonemes("həlˈoʊ")   # IPA input is read as given
    assert raw == fold(list("həlˈoʊ"), v.id_map)
    v.cfg["espeak"] = {"voice": "de"}   # not English: characters as before
    (de,) = v.phonemes("hallo")
    assert de == list("hallo")
