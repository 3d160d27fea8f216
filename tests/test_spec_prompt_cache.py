"""n-gram speculative decoding (exactly the greedy output, fewer forward passes) and the
persistent prompt cache (prompt_cache_path: KV prefix blocks saved, restored into a fresh
engine's prefix cache), on the CPU engine."""
import os

import pytest

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.engine.speculative import ngram_draft


def _engine(path, **kw):
    return LLMEngine(EngineConfig(model_path=path, device="cpu", context_size=512, max_num_seqs=4,
                                  use_graphs=False, block_size=16, **kw))


def test_ngram_draft_lookup():
    assert ngram_draft([1, 2, 3, 9, 1, 2, 3], 3) == [9, 1, 2]       # 3-gram match
    assert ngram_draft([5, 6, 7, 5, 6], 2) == [7, 5]                # 2-gram match
    assert ngram_draft([4, 8, 1, 4], 4) == [8, 1, 4]                # 1-gram, truncated at the end
    assert ngram_draft([1, 2, 3], 4) == []                          # no earlier occurrence
    assert ngram_draft([1, 2, 1, 2, 1], 2) == [2, 1]                # latest match wins
    assert ngram_draft([3, 3], 0) == []


def test_speculative_greedy_output_is_exact(tiny_model_path, monkeypatch):
    """Whatever the drafts are (right, wrong, partly right), the output is the greedy output; right
    drafts cut forward passes."""
    import localai_amd.engine.llm_engine as le
    eng = _engine(tiny_model_path)
    prompt = "one two three four one two three four one two three four one two"
    n_prompt = len(eng.tokenize(prompt))
    truth, evs = [], []

    def cb(ev):
        if ev.token >= 0:
            truth.append(ev.token)
        if ev.finished:
            evs.append(ev)

    eng.add_request(prompt, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True), cb)
    while not evs:
        eng.step()
    base = eng.generate(prompt, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True))
    calls = [0]

    def oracle(seq, k, **kw):  # alternately the true continuation and a wrong guess
        calls[0] += 1
        done = len(seq) - n_prompt
        nxt = truth[done:done + k]
        if calls[0] % 2 == 0 and nxt:
            nxt = nxt[:1] + [(nxt[1] + 1) if len(nxt) > 1 else nxt[0]]
        return list(nxt)

    monkeypatch.setattr(le, "ngram_draft", oracle)
    steps0 = eng.metrics["steps"]
    spec = eng.generate(prompt, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True, n_draft=4))
    assert spec["completion_tokens"] == 24
    assert spec["text"] == base["text"]
    assert eng.metrics["spec_steps"] > 0 and eng.metrics["spec_accepted"] > 0
    assert eng.metrics["steps"] - steps0 < 24  # accepted drafts saved forward passes
    # the real n-gram drafter runs end to end too (exact output whatever it proposes)
    monkeypatch.setattr(le, "ngram_draft", ngram_draft)
    again = eng.generate(prompt, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True, n_draft=4))
    assert again["text"] == base["text"]


def test_prompt_cache_persists_and_restores(tiny_model_path, tmp_path):
    path = str(tmp_path / "cache" / "prompt.safetensors")
    prompt = " ".join(f"w{i}" for i in range(60))
    p = dict(max_tokens=4, temperature=0.0, ignore_eos=True, prompt_cache_path=path)
    e1 = _engine(tiny_model_path)
    r1 = e1.generate(prompt, SamplingParams(**p))
    e1._pcache.flush()  # the file is written by a background thread, off the engine loop
    assert os.path.exists(path)
    # the same prompt again: the file already holds that prefix, so nothing is rewritten
    mt = os.path.getmtime(path)
    e1.generate(prompt, SamplingParams(**p))
    e1._pcache.flush()
    assert os.path.getmtime(path) == mt
    # a fresh engine (empty prefix cache) restores the blocks and reuses them
    e2 = _engine(tiny_model_path)
    bm = e2.sched.blocks()
    assert bm.hit_tokens == 0
    r2 = e2.generate(prompt, SamplingParams(**p, prompt_cache_ro=True))
    assert bm.hit_tokens >= 16, bm.hit_tokens
    assert r2["text"] == r1["text"]
    # a foreign / corrupt file is ignored, not fatal
    bad = tmp_path / "bad.safetensors"
    bad.write_bytes(b"not a cache")
    e3 = _engine(tiny_model_path)
    r3 = e3.generate(prompt, SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True,
                                            prompt_cache_path=str(bad), prompt_cache_ro=True))
    assert r3["completion_tokens"] == 2


@pytest.mark.parametrize("ro", [False, True])
def test_prompt_cache_read_only_never_writes(tiny_model_path, tmp_path, ro):
    path = str(tmp_path / f"pc_{ro}.safetensors")
    e = _engine(tiny_model_path)
    e.generate("a b c d e f g h i j k l m n o p q r s t u v w x y z",
               SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True, prompt_cache_path=path,
                              prompt_cache_ro=ro))
    e._pcache.flush()
    assert os.path.exists(path) is (not ro)


def test_draft_model_speculation_is_exact(tiny_model_path, tmp_path):
    """draft_model: a second LM proposes the drafts.  With the main model itself as the draft every
    draft token is accepted (k+1 tokens per verify pass); with an unrelated draft model (other
    weights, same vocabulary, fewer layers) drafts are mostly rejected; either way the text is the
    main model's greedy text, and finished requests give their draft KV pages back."""
    from localai_amd.models import synth
    prompt = "speculative decoding with a draft model"
    sp = lambda **kw: SamplingParams(max_tokens=20, temperature=0.0, ignore_eos=True, **kw)  # noqa: E731
    base = _engine(tiny_model_path).generate(prompt, sp())
    eng = _engine(tiny_model_path, draft_model=tiny_model_path)
    out = eng.generate(prompt, sp())
    assert out["text"] == base["text"] and out["completion_tokens"] == 20
    m = eng.metrics
    assert m["spec_steps"] > 0 and m["spec_accepted"] == m["spec_drafted"] > 0
    assert m["spec_steps"] <= 20 // (eng.DRAFT_DEFAULT_K + 1) + 2  # ~k+1 tokens per main-model pass
    assert not eng.drafter._pages  # released on finish
    # a second request reuses the draft cache pages (and n_draft from the request wins)
    out2 = eng.generate(prompt + " again", sp(n_draft=3))
    assert out2["text"] == _engine(tiny_model_path).generate(prompt + " again", sp())["text"]

    other = str(tmp_path / "draft.gguf")
    synth.write_model(other, "tiny-llama", seed=7, exact=True, n_layer=1)
    eng2 = _engine(tiny_model_path, draft_model=other)
    outs = [eng2.generate(p, sp()) for p in (prompt, "a different prompt entirely")]
    assert outs[0]["text"] == base["text"]
    assert outs[1]["text"] == _engine(tiny_model_path).generate("a different prompt entirely", sp())["text"]
    assert eng2.metrics["spec_drafted"] > eng2.metrics["spec_accepted"]


def test_draft_model_vocab_mismatch_is_a_load_error(tiny_model_path, tmp_path):
    from localai_amd.models import synth
    from localai_amd.models.synth import PRESETS
    other = str(tmp_path / "small-vocab.gguf")
    synth.write_model(other, "tiny-llama", exact=True, n_vocab=PRESETS["tiny-llama"].n_vocab - 64)
    with pytest.raises(ValueError, match="vocabulary"):
        _engine(tiny_model_path, draft_model=other)


def test_draft_model_catch_up_is_chunked(tiny_model_path):
    """A long prompt's first draft feeds the whole prompt to the draft model: the catch-up must run
    in forwards of at most max_batched_tokens tokens (like the main engine's chunked prefill), with
    several requests drafting at once, and the text stays the main model's greedy text."""
    import threading
    prompts = [("long prompt number %d " % i) + "word " * 60 for i in range(3)]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    ref = [_engine(tiny_model_path).generate(p, sp)["text"] for p in prompts]
    eng = _engine(tiny_model_path, draft_model=tiny_model_path, max_batched_tokens=32)
    sizes = []
    fwd = eng.drafter.model.forward

    def spy(fb, *a, **kw):
        sizes.append(int(fb.tokens.shape[0]))
        return fwd(fb, *a, **kw)

    eng.drafter.model.forward = spy
    eng.start()
    try:
        outs = [None] * len(prompts)

        def run(j):
            outs[j] = eng.generate(prompts[j], sp)["text"]

        ths = [threading.Thread(target=run, args=(j,)) for j in range(len(prompts))]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
    finally:
        eng.shutdown()
    assert outs == ref
    assert sizes and max(sizes) <= 32, sizes
    assert sum(1 for s in sizes if s == 32) >= 2  # the prompts really were split
