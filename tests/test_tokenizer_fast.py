"""The fast BPE path of tokenizer.Tokenizer (pre-tokenizer split in the `regex` module, BPE cached
per pre-token, misses through a byte-level-only twin of the BPE model) gives the same ids as the
tokenizers-library pipeline (Split on the same pattern + ByteLevel + BPE) for the Llama-3, Qwen2
(chatml) and GPT-2 / phi-2 pre-tokenizer patterns, on adversarial text: unicode letters and
numbers, emoji, digit runs, contractions in both cases, whitespace and newline runs."""
import random

import pytest

from localai_amd.gguf import GGUFReader
from localai_amd.models import synth
from localai_amd.tokenizer import Tokenizer


@pytest.mark.parametrize("preset", ["tiny-llama3-tok", "tiny-qwen2", "tiny-phi2"])
def test_fast_bpe_matches_library_pipeline(preset, tmp_path):
    kw = dict(n_vocab=128256, tokenizer="llama3") if preset == "tiny-llama3-tok" else {}
    p = synth.write_model(str(tmp_path / "t.gguf"), "tiny-llama" if preset == "tiny-llama3-tok" else preset, **kw)
    tok = Tokenizer.from_gguf(GGUFReader(p))
    if tok.model != "gpt2":
        pytest.skip("SPM vocabulary")
    assert tok._pre_re is not None
    rng = random.Random(1)
    alpha = list("abcXYZ 019'\n\t\r.,!?-_()[]{}\"") + ["é", "ß", "漢", "字", "😀", "  ", "\n\n", "'s", "'LL", "'Ve",
                                                    " 123456", " ", "ﬁ", " ", "٣", "Ω"]
    texts = ["", " ", "hello world", "I'm here, aren't you?", "x" * 300, "1234567 89", "\n \n\t\n  a"]
    texts += ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 80))) for _ in range(1500)]
    for t in texts:
        assert tok._bpe_fast(t) == tok._hf.encode(t, add_special_tokens=False).ids, repr(t)
    # through the public API, twice (the second pass is served from the per-word cache)
    for t in texts[:200]:
        a = tok.encode(t, add_bos=False)
        assert a == tok.encode(t, add_bos=False)


def test_fast_bpe_survives_cache_eviction(tmp_path, monkeypatch):
    """A prompt that mixes cached and new pre-tokens right when the cache overflows (the size
    check clears it) still encodes: hits are copied out before any eviction."""
    p = synth.write_model(str(tmp_path / "t.gguf"), "tiny-llama", n_vocab=128256, tokenizer="llama3")
    tok = Tokenizer.from_gguf(GGUFReader(p))
    if tok.model != "gpt2" or tok._pre_re is None:
        pytest.skip("no fast BPE path")
    monkeypatch.setattr(type(tok), "_WORD_CACHE_SIZE", 4)
    ref = lambda t: tok._hf.encode(t, add_special_tokens=False).ids  # noqa: E731
    assert tok._bpe_fast("alpha beta") == ref("alpha beta")       # 2 words cached
    # two hits + three misses: 2 + 3 > 4 clears the cache between the lookup and the output
    t = "alpha beta gamma delta epsilon"
    assert tok._bpe_fast(t) == ref(t)
    # concurrent clear from another thread between calls
    tok._word_cache.clear()
    assert tok._bpe_fast(t) == ref(t)
