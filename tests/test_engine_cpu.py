"""LLM engine on CPU (torch reference ops): greedy decoding vs. the fp32 oracle, sampling
params, stop words, max tokens, abort, continuous batching consistency, model families
(llama / mixtral MoE / phi2), embeddings.  The same engine drives the HIP kernels on GPU."""
import math
import threading

import numpy as np
import pytest
import torch

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.models import synth


def _engine(path, **kw):
    return LLMEngine(EngineConfig(model_path=path, device="cpu", context_size=kw.pop("ctx", 512),
                                  max_num_seqs=kw.pop("seqs", 8), use_graphs=False, **kw))


@pytest.fixture(scope="module")
def eng(tiny_model_path):
    return _engine(tiny_model_path)


def test_greedy_matches_fp32_reference(eng):
    prompt = "The quick brown fox"
    ids = eng.tokenize(prompt)
    res = eng.generate(prompt, SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
    assert res["completion_tokens"] == 4
    # teacher-forced comparison: the engine's greedy tokens are (near-)argmaxes of the oracle
    out_ids = eng.tokenize(prompt + res["text"])[len(ids):]
    seq = list(ids)
    for t in out_ids[:3]:
        ref = eng.model.reference_logits(seq)[-1]
        top = torch.topk(ref, 2)
        assert t == int(top.indices[0]) or float(top.values[0] - ref[t]) < 0.05
        seq.append(t)


def test_max_tokens_and_usage(eng):
    r = eng.generate("abc", SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    assert r["finish_reason"] == "length" and r["completion_tokens"] == 3 and r["prompt_tokens"] > 0


def test_stop_word_truncates(eng):
    base = eng.generate("stop test", SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))["text"]
    if len(base) < 3:
        pytest.skip("degenerate continuation")
    stop = base[1:3]
    r = eng.generate("stop test", SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True, stop=[stop]))
    assert r["finish_reason"] == "stop"
    assert stop not in r["text"] and base.startswith(r["text"])


def test_seeded_sampling_is_reproducible(eng):
    p = SamplingParams(max_tokens=6, temperature=1.0, top_k=20, top_p=0.9, seed=1234, ignore_eos=True)
    a = eng.generate("seed", p)["text"]
    b = eng.generate("seed", SamplingParams(max_tokens=6, temperature=1.0, top_k=20, top_p=0.9, seed=1234,
                                            ignore_eos=True))["text"]
    assert a == b


def test_batched_equals_sequential(tiny_model_path):
    e = _engine(tiny_model_path)
    prompts = ["alpha beta", "gamma", "delta epsilon zeta", "eta"]
    sp = dict(max_tokens=5, temperature=0.0, ignore_eos=True)
    seq = [e.generate(p, SamplingParams(**sp))["text"] for p in prompts]
    e2 = _engine(tiny_model_path, prefix_cache=False)
    outs = {}
    done = threading.Event()

    def mk(i):
        buf = bytearray()

        def cb(ev):
            buf.extend(ev.text)
            if ev.finished:
                outs[i] = buf.decode("utf-8", "replace")
                if len(outs) == len(prompts):
                    done.set()
        return cb
    for i, p in enumerate(prompts):
        e2.add_request(p, SamplingParams(**sp), mk(i))
    while not done.is_set():
        e2.step()
    same = sum(outs[i] == seq[i] for i in range(len(prompts)))
    assert same >= len(prompts) - 1  # bf16 batch-order ties may flip one random-model token


def test_abort_frees_sequence(eng):
    got = []
    rid = eng.add_request("abort me", SamplingParams(max_tokens=50, ignore_eos=True), got.append)
    eng.step()
    eng.abort(rid)
    for _ in range(5):
        eng.step()
    assert got and got[-1].finished
    assert not eng.has_work()


def test_embeddings_shape_and_determinism(eng):
    a = eng.embed(["hello world"])[0]
    b = eng.embed(["hello world"])[0]
    assert len(a) == eng.model.hp.n_embd
    assert max(abs(x - y) for x, y in zip(a, b)) < 1e-5


@pytest.mark.parametrize("preset", ["tiny-mixtral", "tiny-phi2", "tiny-llama-q8", "tiny-qwen2", "tiny-phi3",
                                    "tiny-gemma", "tiny-gemma2", "tiny-command-r", "tiny-starcoder2",
                                    "tiny-qwen2moe", "tiny-deepseek2"])
def test_model_families_generate(preset, tmp_path):
    p = str(tmp_path / f"{preset}.gguf")
    synth.write_model(p, preset, exact=True)
    e = _engine(p)
    r = e.generate("hello", SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
    assert r["completion_tokens"] == 3
    ids = e.tokenize("hello")
    ref = e.model.reference_logits(ids)[-1]
    assert torch.isfinite(ref).all()
    # the engine's first greedy token is the oracle's argmax (or within a rounding tie of it)
    first = e.tokenize("hello" + r["text"])[len(ids)] if r["text"] else None
    if first is not None:
        top = torch.topk(ref, 2)
        assert first == int(top.indices[0]) or float(top.values[0] - ref[first]) < 0.05


def test_new_family_hparams(tmp_path):
    """GGUF metadata -> HParams for the Qwen2 / Phi-3 / Gemma layouts."""
    from localai_amd.gguf import GGUFReader
    from localai_amd.models.hparams import HParams
    got = {}
    for preset in ("tiny-qwen2", "tiny-phi3", "tiny-gemma"):
        p = str(tmp_path / f"{preset}.gguf")
        synth.write_model(p, preset)
        got[preset] = HParams.from_gguf(GGUFReader(p))
    q, ph, g = got["tiny-qwen2"], got["tiny-phi3"], got["tiny-gemma"]
    assert q.rope_mode == 1 and q.act == "swiglu" and q.norm_eps == pytest.approx(1e-6)
    assert ph.head_dim == 96 and ph.rope_mode == 1 and ph.act == "swiglu"
    assert g.head_dim == 256 and g.q_dim == 512 and g.act == "geglu" and g.tied_embeddings
    assert g.embed_scale == pytest.approx(16.0)
    p2 = str(tmp_path / "g2.gguf")
    synth.write_model(p2, "tiny-gemma2")
    g2 = HParams.from_gguf(GGUFReader(p2))
    assert (g2.attn_softcap, g2.final_softcap, g2.sliding_window) == (50.0, 30.0, 24) and g2.act == "geglu"


def test_gemma2_window_and_softcap_engine_matches_oracle(tmp_path):
    """A prompt longer than the sliding window: the engine's chunked paged attention (softcap,
    window on layer 0, post norms, final-logit softcap) reproduces the oracle's last-token logits."""
    p = str(tmp_path / "g2.gguf")
    synth.write_model(p, "tiny-gemma2", exact=True)
    e = _engine(p)
    prompt = "the quick brown fox jumps over the lazy dog " * 4
    ids = e.tokenize(prompt)
    assert len(ids) > 24
    ref = e.model.reference_logits(ids)[-1]
    r = e.generate(prompt, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True))
    full = e.tokenize(prompt + r["text"])
    first = full[len(ids)] if r["text"] and full[:len(ids)] == ids else None
    assert torch.isfinite(ref).all() and float(ref.abs().max()) <= 30.0 + 1e-4
    if first is not None:
        top = torch.topk(ref, 2)
        assert first == int(top.indices[0]) or float(top.values[0] - ref[first]) < 0.05


def _png(color, size=40):
    import io
    from PIL import Image
    img = Image.new("RGB", (size, size + 8), color)
    for x in range(0, size, 3):
        img.putpixel((x, x % size), (255 - color[0], 30, 200))
    b = io.BytesIO()
    img.save(b, format="PNG")
    return b.getvalue()


def test_llava_image_prompt(tiny_model_path, tmp_path):
    import base64
    from localai_amd.gguf import GGUFReader
    n_embd = int(GGUFReader(tiny_model_path).kv["llama.embedding_length"])
    mm = synth.write_mmproj(str(tmp_path / "mmproj.gguf"), out_dim=n_embd, dim=64, n_layer=2, heads=4, ffn=128,
                            image_size=28, patch=14)
    e = _engine(tiny_model_path, mmproj=mm)
    assert e.clip is not None and e.clip.n_patches == 4
    sp = dict(max_tokens=4, temperature=0.0, ignore_eos=True)
    out = {}

    def run(images, prompt="[img-0]What is in the image?"):
        got = {}

        def cb(ev):
            if ev.finished:
                got.update(n_prompt=ev.prompt_tokens, n=ev.completion_tokens, err=ev.error)
        e.add_request(prompt, SamplingParams(**sp), cb, images=images)
        while not got:
            e.step()
        return got
    text_only = len(e.tokenize("What is in the image?"))
    a = run([base64.b64encode(_png((200, 10, 10))).decode()])
    assert a["err"] == "" and a["n"] == 4
    assert a["n_prompt"] == text_only + 4            # 2x2 patches spliced in front of the text
    b = run([_png((10, 200, 10))], prompt="What is in the image?")  # unreferenced image goes first
    assert b["n_prompt"] == text_only + 4
    emb = e.clip.embed_image(_png((1, 2, 3)))
    assert emb.shape == (4, n_embd) and torch.isfinite(emb).all()


def test_llava16_anyres_layout(tiny_model_path, tmp_path):
    from localai_amd.gguf import GGUFReader
    n_embd = int(GGUFReader(tiny_model_path).kv["llama.embedding_length"])
    mm = synth.write_mmproj(str(tmp_path / "mmproj16.gguf"), out_dim=n_embd, dim=64, n_layer=1, heads=4, ffn=128,
                            image_size=28, patch=14, pinpoints=[28, 56, 56, 28, 56, 56])
    from localai_amd.models.clip import ClipVision
    cv = ClipVision(mm, torch.device("cpu"))
    tiles, layout = cv.preprocess(_png((90, 90, 90), size=50))
    assert layout is not None and tiles.shape[0] == 1 + layout[0] * layout[1]
    emb = cv.embed_image(_png((90, 90, 90), size=50))
    assert emb.shape[1] == n_embd and emb.shape[0] > 4 and torch.isfinite(emb).all()


def _siglip_reference(mm_path, pix):
    """Plain fp32 SigLIP tower + mlp projector straight from the GGUF tensors (no class token,
    post-LayerNorm, exact GELU) -- the oracle for ClipVision's moondream2 path."""
    import torch.nn.functional as F

    from localai_amd.gguf import GGUFReader, dequantize
    r = GGUFReader(mm_path)
    kv = r.kv

    def t(n):
        x = r.tensors[n]
        return torch.from_numpy(np.ascontiguousarray(dequantize(x.data, x.ggml_type, x.shape).reshape(x.shape),
                                                     dtype=np.float32))
    D, P, H = int(kv["clip.vision.embedding_length"]), int(kv["clip.vision.patch_size"]), \
        int(kv["clip.vision.attention.head_count"])
    x = F.conv2d(pix.float(), t("v.patch_embd.weight"), t("v.patch_embd.bias"), stride=P)
    h = x.flatten(2).transpose(1, 2) + t("v.position_embd.weight")
    n, L, _ = h.shape
    for i in range(int(kv["clip.vision.block_count"])):
        b = f"v.blk.{i}."
        a = F.layer_norm(h, (D,), t(b + "ln1.weight"), t(b + "ln1.bias"), 1e-5)
        q, k, v = (F.linear(a, t(b + f"attn_{c}.weight"), t(b + f"attn_{c}.bias")).view(n, L, H, D // H)
                   .transpose(1, 2) for c in "qkv")
        att = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(D // H), -1) @ v
        h = h + F.linear(att.transpose(1, 2).reshape(n, L, D), t(b + "attn_out.weight"), t(b + "attn_out.bias"))
        a = F.layer_norm(h, (D,), t(b + "ln2.weight"), t(b + "ln2.bias"), 1e-5)
        f1w, f2w = t(b + "ffn_down.weight"), t(b + "ffn_up.weight")
        f1b, f2b = t(b + "ffn_down.bias"), t(b + "ffn_up.bias")
        if f1w.shape[1] != D:
            f1w, f2w, f1b, f2b = f2w, f1w, f2b, f1b
        h = h + F.linear(F.gelu(F.linear(a, f1w, f1b)), f2w, f2b)
    h = F.layer_norm(h, (D,), t("v.post_ln.weight"), t("v.post_ln.bias"), 1e-5)
    y = F.gelu(F.linear(h, t("mm.0.weight"), t("mm.0.bias")))
    return F.linear(y, t("mm.2.weight"), t("mm.2.bias"))


def test_moondream_siglip_tower(tmp_path):
    """moondream2 layout (gallery/moondream.yaml): a phi2 text model with a SigLIP mmproj that has
    no class token -- every patch becomes a prompt embedding; the tower matches an fp32 oracle."""
    from localai_amd.gguf import GGUFReader
    from localai_amd.models.clip import ClipVision
    txt = str(tmp_path / "moondream-text.gguf")
    synth.write_model(txt, "tiny-phi2", exact=True)
    n_embd = int(GGUFReader(txt).kv["phi2.embedding_length"])
    mm = synth.write_mmproj(str(tmp_path / "moondream-mmproj.gguf"), out_dim=n_embd, dim=64, n_layer=2, heads=4,
                            ffn=128, image_size=42, patch=14, siglip=True)
    cv = ClipVision(mm, torch.device("cpu"))
    assert cv.cls is None and cv.n_patches == 9
    tiles, layout = cv.preprocess(_png((30, 160, 60), size=60))
    assert layout is None and tiles.shape == (1, 3, 42, 42)
    got = cv.encode_tiles(tiles)
    ref = _siglip_reference(mm, tiles)
    assert got.shape == ref.shape == (1, 9, n_embd)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 3e-2, err  # bf16 GEMM operands vs fp32
    e = _engine(txt, mmproj=mm)
    got_ev = {}

    def cb(ev):
        if ev.finished:
            got_ev.update(n_prompt=ev.prompt_tokens, n=ev.completion_tokens, err=ev.error)
    prompt = "[img-0]\nQuestion: What is this?\n\nAnswer:"
    e.add_request(prompt, SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True), cb,
                  images=[_png((30, 160, 60), size=60)])
    while not got_ev:
        e.step()
    assert got_ev["err"] == "" and got_ev["n"] == 3
    assert got_ev["n_prompt"] == len(e.tokenize(prompt.replace("[img-0]", ""))) + 9


def test_engine_trace_timeline(tiny_model_path, tmp_path, monkeypatch):
    """LOCALAI_AMD_TRACE: Chrome-trace timeline with prefill/decode steps, sequence counters and
    per-request spans tagged with the correlation ID."""
    import json

    from localai_amd.utils import trace
    out = tmp_path / "trace.json"
    monkeypatch.setenv("LOCALAI_AMD_TRACE", str(out))
    trace.reset_for_tests()
    try:
        e = _engine(tiny_model_path)
        res = e.generate("trace me", SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True,
                                                     correlation_id="cid-42"))
        assert res["completion_tokens"] == 3
        e.shutdown()
    finally:
        trace.reset_for_tests()
    doc = json.loads(out.read_text())
    names = [ev["name"] for ev in doc["traceEvents"]]
    assert "prefill" in names and "decode" in names and "sequences" in names
    req = [ev for ev in doc["traceEvents"] if ev["name"] == "request"]
    assert len(req) == 1 and req[0]["args"]["correlation_id"] == "cid-42"
    assert req[0]["args"]["completion_tokens"] == 3 and req[0]["dur"] > 0
    assert any(ev["name"] == "first_token" and ev["args"]["correlation_id"] == "cid-42" for ev in doc["traceEvents"])


def test_prefill_tuning_step_packs_one_full_chunk(tiny_model_path):
    """warmup()'s TunableOp pass must hit the exact full-chunk GEMM shape M = max_batched_tokens
    (hipBLASLt solutions are tuned per exact M): one prefill forward of that many tokens, then
    an idle engine with its serving counters untouched."""
    e = _engine(tiny_model_path, seqs=16, max_batched_tokens=1024, ctx=256)
    seen = []
    fwd = e.model.forward

    def spy(fb, kv):
        if not fb.decode:
            seen.append(int(fb.tokens.numel()))
        return fwd(fb, kv)

    e.model.forward = spy
    before = dict(e.metrics)
    e._tune_prefill()
    assert seen == [1024]
    assert not e.requests and e.metrics == before
    out = e.generate("hello", SamplingParams(max_tokens=3, temperature=0.0))
    assert out["completion_tokens"] == 3


def test_batched_vision_tower_matches_single(tiny_model_path, tmp_path):
    """Images of requests arriving in one step share vision-tower batches; embeddings equal the
    one-image-at-a-time path, also across anyres layouts with different tile counts."""
    from localai_amd.gguf import GGUFReader
    from localai_amd.models.clip import ClipVision
    n_embd = int(GGUFReader(tiny_model_path).kv["llama.embedding_length"])
    mm = synth.write_mmproj(str(tmp_path / "mm16.gguf"), out_dim=n_embd, dim=64, n_layer=1, heads=4, ffn=128,
                            image_size=28, patch=14, pinpoints=[28, 56, 56, 28, 56, 56])
    cv = ClipVision(mm, torch.device("cpu"))
    cv.TILE_BATCH = 3  # force several tower launches across image boundaries
    imgs = [_png((10, 20, 30), size=50), _png((200, 10, 10), size=20), _png((5, 99, 7), size=70)]
    batched = cv.embed_images(imgs)
    for im, b in zip(imgs, batched):
        single = cv.embed_image(im)
        assert b.shape == single.shape and torch.allclose(b, single, atol=1e-5)
    e = _engine(tiny_model_path, mmproj=mm)
    got = {}

    def cb_for(i):
        def cb(ev):
            if ev.finished:
                got[i] = (ev.prompt_tokens, ev.completion_tokens, ev.error)
        return cb
    for i, im in enumerate(imgs):  # all queued before the next step: one batched encode
        e.add_request(f"[img-0]request {i}", SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True),
                      cb_for(i), images=[im])
    while len(got) < 3:
        e.step()
    for i, im in enumerate(imgs):
        n_img = cv.embed_image(im).shape[0]
        assert got[i][2] == "" and got[i][1] == 2
        assert got[i][0] == n_img + len(e.tokenize(f"request {i}"))


def test_get_metrics_reports_the_active_slot(eng):
    """GetMetrics = the reference's get_active_slot() view (grpc-server.cpp:2434-2457): a request
    in flight is reported with its id, prompt and generated-token count; idle -> zeros."""
    import asyncio
    import json as _json

    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    sv = EngineServicer(device="cpu")
    sv.engine = eng
    idle = asyncio.run(sv.GetMetrics(pb.MetricsRequest()))
    assert idle.slot_id == 0 and idle.tokens_generated == 0 and idle.prompt_json_for_slot == ""
    ids = eng.tokenize("metrics probe")
    rid = eng.add_request(ids, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True), lambda ev: None)
    for _ in range(4):
        eng.step()
    m = asyncio.run(sv.GetMetrics(pb.MetricsRequest()))
    assert m.slot_id == rid
    assert 0 < m.tokens_generated <= 6
    assert m.prompt_tokens_processed == len(ids)
    # the prompt as a JSON string (grpc-server.cpp:2441 slot->prompt.dump()); ids are detokenised
    assert _json.loads(m.prompt_json_for_slot) == eng.tokenizer.decode(ids)
    while eng.has_work():
        eng.step()
    assert asyncio.run(sv.GetMetrics(pb.MetricsRequest())).slot_id == 0
    eng.add_request("metrics text probe", SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True),
                    lambda ev: None)
    eng.step()
    assert _json.loads(asyncio.run(sv.GetMetrics(pb.MetricsRequest())).prompt_json_for_slot) == "metrics text probe"
    while eng.has_work():
        eng.step()


def test_penalties_keep_device_sampling_within_the_ring(tiny_model_path):
    """Penalty windows up to PEN_CAP stay on the device (multi-step graphs); longer ones, mirostat
    v1 and grammars fall back to host-driven sampling."""
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine, Request
    from localai_amd.engine.sampling_params import SamplingParams
    eng = LLMEngine(EngineConfig(model_path=tiny_model_path, device="cpu", context_size=512, max_num_seqs=2,
                                 use_graphs=False))

    def need(**kw):
        return eng._needs_host_sampling(Request(0, [1], SamplingParams(**kw), lambda e: None))
    assert not need(repeat_penalty=1.3, repeat_last_n=64)
    assert not need(frequency_penalty=0.5, presence_penalty=0.5, repeat_last_n=256)
    assert need(repeat_penalty=1.3, repeat_last_n=257)
    assert need(repeat_penalty=1.3, repeat_last_n=-1)  # whole context (512 > 256)
    assert not need(repeat_last_n=-1)                   # no penalty asked
    assert need(mirostat=1)


def test_penalty_ring_push_cpu():
    import torch

    from localai_amd import ops
    hist = torch.full((2, 4), -1, dtype=torch.int32)
    cnt = torch.tensor([0, 3], dtype=torch.int32)
    hl = torch.zeros(2, dtype=torch.int32)
    cap = torch.tensor([4, 3], dtype=torch.int32)
    hist[1, :3] = torch.tensor([7, 8, 9])
    for t in (5, 6):
        ops.penalty_push(torch.tensor([t, t], dtype=torch.int32), hist, cnt, hl, cap)
    assert hist[0].tolist() == [5, 6, -1, -1] and hl.tolist() == [2, 3]
    assert sorted(hist[1, :3].tolist()) == [5, 6, 9]   # the two oldest (7, 8) dropped out of the window


def test_admission_window_closes_once_a_prefill_chunk_waits(tiny_model_path, monkeypatch):
    """Burst admission: an idle engine waits for arrivals to pause (or the window to end), but
    stops waiting as soon as the queued prompts fill half a prefill chunk (admission_close_tokens,
    default max_batched_tokens / 2); 0 restores the plain window."""
    import time
    monkeypatch.delenv("LOCALAI_AMD_ADMIT_TOKENS", raising=False)
    e = _engine(tiny_model_path, seqs=16, max_batched_tokens=64, admission_window_ms=400.0,
                admission_quiet_ms=50.0)
    e.admit_log = []
    sp = SamplingParams(max_tokens=1, temperature=0.0)
    stop = threading.Event()

    def trickle():  # one arrival every 10 ms: the quiet gap never comes
        while not stop.is_set():
            e.add_request("hello there general kenobi " * 2, sp, lambda ev: None)
            time.sleep(0.01)
    th = threading.Thread(target=trickle)
    th.start()
    try:
        time.sleep(0.02)
        t0 = time.perf_counter()
        e._admit_burst()
        early = time.perf_counter() - t0
        assert e._inbox_tokens() >= 32 and early < 0.3   # half of max_batched_tokens
        e.cfg.admission_close_tokens = 0
        t0 = time.perf_counter()
        e._admit_burst()
        assert time.perf_counter() - t0 >= 0.35  # the full window
    finally:
        stop.set()
        th.join()
    assert len(e.admit_log) == 2


@pytest.mark.parametrize("first_ms", [60000.0, 0.0])   # (a CPU prefill under a loaded test run is slow)
def test_burst_prefill_first_policy(tiny_model_path, monkeypatch, first_ms):
    """EngineConfig.prefill_first_ms: while a burst's prompts are still being prefilled (several
    chunks under a small token budget) and every decodable row holds only its first token, steps
    are prefill-only; the rows then decode together.  0 restores mixed prefill + decode steps.
    Greedy outputs are the same either way."""
    monkeypatch.delenv("LOCALAI_AMD_PREFILL_FIRST_MS", raising=False)
    e = _engine(tiny_model_path, seqs=8, max_batched_tokens=24, prefill_first_ms=first_ms, prefix_cache=False)
    kinds = []
    run_p, run_d = e._run_prefill, e._run_decode

    def rp(plan):
        kinds.append("p")
        return run_p(plan)

    def rd(plan, K):
        kinds.append("d")
        return run_d(plan, K)
    e._run_prefill, e._run_decode = rp, rd
    prompts = [f"prompt number {i} with a few more words in it" for i in range(6)]
    sp = dict(max_tokens=4, temperature=0.0, ignore_eos=True)
    outs, done = {}, threading.Event()

    def mk(i):
        buf = bytearray()

        def cb(ev):
            buf.extend(ev.text)
            if ev.finished:
                outs[i] = buf.decode("utf-8", "replace")
                if len(outs) == len(prompts):
                    done.set()
        return cb
    for i, p in enumerate(prompts):
        e.add_request(p, SamplingParams(**sp), mk(i))
    while not done.is_set():
        e.step()
    n_p = kinds.count("p")
    assert n_p >= 3  # the burst needs several prefill chunks
    last_p = len(kinds) - 1 - kinds[::-1].index("p")
    decode_during_prefill = "d" in kinds[:last_p]
    assert decode_during_prefill == (first_ms == 0.0)
    ref = {i: e.generate(p, SamplingParams(**sp))["text"] for i, p in enumerate(prompts)}
    assert sum(outs[i] == ref[i] for i in ref) >= len(ref) - 1  # bf16 batch-order ties may flip one token
