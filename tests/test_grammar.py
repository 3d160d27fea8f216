"""GBNF grammar engine (llama.cpp llama-grammar semantics) and grammar-constrained decoding."""
import json

import numpy as np
import pytest

from localai_amd import functions as fn
from localai_amd.native import core


def _state(text, pieces=None, eog=(0,)):
    pieces = pieces or [b"", b"{", b"}", b'"', b"a", b":", b" ", b"1", b"[", b"]", b","]
    return core.GrammarState(core.Grammar(text), core.GrammarVocab(pieces, list(eog)))


@pytest.mark.parametrize("doc,ok", [('{"a": 1}', True), ('{"a": [1, 2, {"b": null}]}', True), ('{"a" 1}', False),
                                    ('{"a": tru}', None), ("[1]", None)])
def test_json_grammar_documents(doc, ok):
    st = _state(fn.JSON_BNF)
    acc = st.accept_bytes(doc.encode())
    if ok is True:
        assert acc and st.can_end()
    elif ok is False:
        assert not acc
    else:
        assert not (acc and st.can_end())


def test_repetition_operators_and_classes():
    g = 'root ::= "a"+ [0-9]? ("x" | "y"){2,3} [^z]*'
    for s, ok in [("a", False), ("aaxy", True), ("a5xyx", True), ("axyxyxz", False), ("ax", False), ("axyq!", True),
                  ("axyz", False)]:
        st = _state(g)
        assert (st.accept_bytes(s.encode()) and st.can_end()) == ok, s


def test_filter_and_eog():
    pieces = [b"", b"ye", b"s", b"no", b"n", b"o", b"yes"]
    st = _state('root ::= "yes" | "no"', pieces, eog=(0,))
    acc = st.filter(np.arange(len(pieces), dtype=np.int32))
    assert list(acc) == [0, 1, 0, 1, 1, 0, 1]
    assert st.accept(6) and st.can_end()
    assert st.check(0)            # EOS allowed once complete
    assert not st.check(2)


def test_function_call_grammar_roundtrip():
    funcs = [{"name": "get_weather", "parameters": {"type": "object", "properties": {"city": {"type": "string"}}}}]
    g = fn.structure_grammar(fn.to_json_structure(funcs, "", ""), fn.grammar_options({}))
    st = _state(g)
    doc = '{"arguments": {"city": "Paris"}, "name": "get_weather"}'
    assert st.accept_bytes(doc.encode()) and st.can_end()
    assert not _state(g).accept_bytes(b'{"arguments": {"town"')


def test_bad_grammar_raises():
    with pytest.raises(ValueError):
        core.Grammar('root ::= undefined-rule')
    with pytest.raises(ValueError):
        core.Grammar('root ::= "unterminated')


def test_engine_constrained_generation(tiny_model_path):
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    eng = LLMEngine(EngineConfig(model_path=tiny_model_path, device="cpu", context_size=512, max_num_seqs=4,
                                 use_graphs=False))
    g = 'root ::= "{" "\\"answer\\"" ":" " "? ("true" | "false") "}"'
    for temp in (0.0, 1.0):
        r = eng.generate("answer in json", SamplingParams(max_tokens=40, temperature=temp, seed=5, grammar=g))
        assert r["text"].replace(" ", "") in ('{"answer":true}', '{"answer":false}'), r
        assert r["finish_reason"] == "stop"
    r = eng.generate("json please", SamplingParams(max_tokens=24, temperature=0.7, seed=1, grammar=fn.JSON_BNF))
    # a random model rarely closes the object within 24 tokens; the prefix must still be valid JSON text
    st = _state(fn.JSON_BNF)
    assert st.accept_bytes(r["text"].encode())
    if r["finish_reason"] == "stop":
        json.loads(r["text"])


def test_trie_mask_equals_linear_scan():
    """The whole-vocabulary mask (depth-first over the vocabulary's byte trie, pruning rejected
    prefixes) decides every token exactly like one check() per token, at every state of a
    function-call grammar walk and with a pending partial UTF-8 code point."""
    import random

    import numpy as np

    import localai_amd.functions as fx
    from localai_amd.models import synth
    from localai_amd.tokenizer import unicode_to_bytes
    a = synth._bpe_asset()
    u2b = unicode_to_bytes()
    pieces = []
    for t in a["tokens"][:6000]:
        try:
            pieces.append(bytes(u2b[c] for c in t))
        except KeyError:
            pieces.append(t.encode())
    pieces += ["é".encode()[:1], "é".encode()[1:], "😀".encode()[:2], b"", b"\"", b"{\"", b"\":\""]
    eog = [len(pieces)]
    pieces.append(b"")
    funcs = [{"name": "get_weather", "parameters": {"type": "object", "properties": {
        "location": {"type": "string"}, "unit": {"type": "string", "enum": ["celsius", "fahrenheit"]},
        "days": {"type": "integer"}}, "required": ["location", "unit", "days"]}}]
    g = fx.structure_grammar(fx.to_json_structure(funcs), fx.grammar_options({}))
    st = core.GrammarState(core.Grammar(g), core.GrammarVocab(pieces, eog))
    rng = random.Random(0)
    for step in range(40):
        m_trie, m_lin = np.asarray(st.mask()), np.asarray(st.mask_linear())
        assert (m_trie == m_lin).all(), step
        ok = np.nonzero(m_lin)[0]
        if len(ok) == 0:
            break
        assert st.accept(int(rng.choice(list(ok))))


def test_mask_limited_and_state_key():
    """mask_limited() equals mask() when the trie walk fits its edge budget and gives up (None)
    on permissive states; key() names the parse state independently of the path that reached it
    (the engine caches device masks under it)."""
    pieces = [b"", b"1", b"2", b"12", b",", b"1,", b"a", b"ab", b"abc", b"b", b"c", b" "]
    st = _state('root ::= ([0-9]+ ",")*', pieces)
    assert (np.asarray(st.mask_limited(10_000)) == np.asarray(st.mask())).all()
    assert st.mask_limited(1) is None
    g, v = core.Grammar('root ::= ([0-9]+ ",")*'), core.GrammarVocab(pieces, [0])
    a, b = core.GrammarState(g, v), core.GrammarState(g, v)   # keys are per Grammar object (the engine caches them)
    assert a.key() == b.key()
    assert a.accept_bytes(b"12,") and b.accept_bytes(b"7,")
    assert a.key() == b.key()                     # same state after different digits
    assert b.accept_bytes(b"3")
    assert a.key() != b.key()                     # inside a number vs after a comma
    free = _state('root ::= [a-c ]*', pieces)
    assert free.mask_limited(3) is None and free.mask_limited(1000) is not None


def test_grammar_mask_op_cpu_fallback():
    import torch

    from localai_amd import ops
    lg = torch.zeros(3, 5)
    pool = torch.tensor([[1, 0, 1, 0, 0], [0, 0, 0, 0, 1]], dtype=torch.bool)
    ops.grammar_mask(lg, torch.tensor([1, -1, 0], dtype=torch.int32), pool)
    inf = float("-inf")
    assert lg.tolist() == [[inf, inf, inf, inf, 0.0], [0.0] * 5, [0.0, inf, 0.0, inf, inf]]


def test_next_keys_and_clone():
    """next_keys() gives the key each candidate token leads to without changing the state (0 when
    rejected); equal parse states reached by different tokens share a key; clone() is an
    independent copy."""
    pieces = [b"", b"1", b"2", b"12", b",", b"1,", b"a"]
    g, v = core.Grammar('root ::= ([0-9]+ ",")*'), core.GrammarVocab(pieces, [0])
    st = core.GrammarState(g, v)
    k0 = st.key()
    keys = st.next_keys(np.arange(len(pieces), dtype=np.int32)).tolist()
    assert keys[0] == 0 and keys[4] == 0 and keys[6] == 0          # eog / "," / "a" rejected here
    assert keys[1] == keys[2] == keys[3] != k0                      # inside a number
    assert keys[5] == k0                                            # "1," loops back to the start
    c = st.clone()
    assert c.accept(1) and c.key() == keys[1] and st.key() == k0


def test_engine_permissive_state_mask_walked_in_background(tiny_model_path):
    """A permissive grammar state (most of the vocabulary allowed) is served by the top-N filter on
    first sight, its full mask is walked on the helper thread when the state recurs, and the cached
    mask is used once ready -- the constrained output obeys the grammar throughout."""
    import re
    import time

    import torch

    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    eng = LLMEngine(EngineConfig(model_path=tiny_model_path, device="cpu", context_size=512, max_num_seqs=4,
                                 use_graphs=False))
    eng.GRAMMAR_MASK_BUDGET = 1           # every state is "permissive" for this test
    g = 'root ::= [a-z ]+'
    r = eng.generate("letters", SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True, grammar=g))
    assert re.fullmatch(r"[a-z ]+", r["text"]), r
    assert eng._gmask_bg is not None                                  # the recurring state went to the helper
    for f in list(eng._gmask_pending.values()):
        f.result(timeout=60)
    V = eng.hp.n_vocab
    r2 = eng.generate("letters", SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True, grammar=g))
    assert re.fullmatch(r"[a-z ]+", r2["text"])
    assert any(v is not None and v >= 0 for v in eng._gmask_cache.values())   # the walked mask is in the pool
    assert eng._gmask_pool is not None and eng._gmask_pool.shape[1] == V
    eng.shutdown()
    assert eng._gmask_bg is None
