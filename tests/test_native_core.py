"""Native engine core: paged-KV block manager with prefix cache, continuous-batching scheduler,
detokenizing stop-word matcher (replaces llama.cpp's slot manager, grpc-server.cpp:1500-2000)."""
import numpy as np
import pytest

from localai_amd.native import core


def test_block_manager_alloc_free_and_prefix_cache():
    bm = core.BlockManager(16, 4, True)
    toks = list(range(10))
    cached = bm.allocate(1, toks, len(toks))
    assert cached == 0
    assert len(bm.table(1)) == 3 and bm.num_free == 13
    bm.commit(1, toks, 10)  # two full blocks become cacheable
    bm.free_seq(1)
    assert bm.num_free == 16
    # same prefix: two full blocks are reused
    cached = bm.allocate(2, toks + [99], 11)
    assert cached == 8
    assert bm.hit_tokens >= 8
    bm.free_seq(2)


def test_block_manager_exhaustion():
    bm = core.BlockManager(4, 4, False)
    assert bm.allocate(1, list(range(12)), 12) == 0
    assert bm.allocate(2, list(range(8)), 8) < 0  # only 1 block left
    bm.free_seq(1)
    assert bm.allocate(2, list(range(8)), 8) == 0


def test_scheduler_prefill_then_decode_with_buckets():
    s = core.Scheduler(64, 4, 8, 64, 256, True, 1)
    s.add(1, [5, 6, 7], 4)
    s.add(2, [8, 9], 4)
    d = s.schedule()
    assert list(d["p_ids"]) == [1, 2]
    assert list(d["p_cu"]) == [0, 3, 5]
    assert list(d["p_tokens"]) == [5, 6, 7, 8, 9]
    assert list(d["p_pos"]) == [0, 1, 2, 0, 1]
    assert len(d["d_ids"]) == 0
    s.append(1, 11)
    s.append(2, 12)
    d = s.schedule()
    assert list(d["d_ids"]) == [1, 2]
    assert list(d["d_tokens"][:2]) == [11, 12]
    assert list(d["d_pos"][:2]) == [3, 2]
    assert list(d["d_lens"][:2]) == [4, 3]
    assert d["d_maxlen"] == 4
    assert len(d["d_tokens"]) in s.buckets()  # padded to a captured graph size
    # slots point into the sequence's own pages
    bt = np.asarray(d["d_bt"])
    assert d["d_slots"][0] == bt[0, 3 // 4] * 4 + 3
    s.finish(1)
    s.finish(2)
    assert s.num_running == 0


def test_scheduler_chunked_prefill_budget():
    s = core.Scheduler(64, 4, 8, 6, 256, False, 0)
    s.add(1, list(range(10)), 2)
    d = s.schedule()
    assert list(d["p_qlen"]) == [6] and d["p_last"][0] == 0
    d = s.schedule()
    assert list(d["p_qlen"]) == [4] and d["p_last"][0] == 1


def test_scheduler_preempts_youngest_when_out_of_blocks():
    s = core.Scheduler(3, 4, 8, 64, 256, False, 0)
    s.add(1, [1, 2, 3], 10)
    s.add(2, [4, 5, 6], 10)
    s.schedule()
    pre = []
    for step in range(12):
        for i in (1, 2):
            if s.has(i) and s.n_tokens(i) < 12:
                s.append(i, 7)
        d = s.schedule()
        pre += list(d["preempted"])
    assert 2 in pre  # the younger sequence is evicted and later recomputed


def test_scheduler_deferred_step_decodes_when_waiting_prompt_does_not_fit():
    """Burst prefill-first mode (defer_decode) with a KV pool too small for the waiting prompt: the
    step must fall back to decoding the running rows (which frees blocks as they finish) instead
    of returning an empty plan forever."""
    s = core.Scheduler(4, 4, 8, 64, 256, False, 0)
    s.add(1, [1, 2, 3], 3)          # 1 block
    d = s.schedule()
    assert list(d["p_ids"]) == [1]
    s.append(1, 9)
    s.add(2, list(range(20)), 2)    # needs 5 blocks: never fits while seq 1 holds one
    d = s.schedule(1, True)
    assert list(d["d_ids"]) == [1], "deferred step came back empty"
    assert len(d["p_ids"]) == 0


def _vocab():
    pieces = [b"", b"Hel", b"lo", b" wor", b"ld", b"<|eot|>", b"\xe2\x82", b"\xac", b"STOP", b"x"]
    return core.Vocab(pieces)


def test_textstream_stop_words_and_holdback():
    v = _vocab()
    ts = core.TextStream(v, ["STOP"])
    out = b""
    for t in (1, 2, 3, 4):
        b, stopped = ts.push(t)
        out += b
        assert not stopped
    b, stopped = ts.push(8)
    out += b
    assert stopped and out == b"Hello world"


def test_textstream_partial_stop_is_held_then_released():
    v = core.Vocab([b"", b"ab", b"S", b"T", b"c"])
    ts = core.TextStream(v, ["STOP"])
    b1, _ = ts.push(1)
    b2, _ = ts.push(2)  # "S" could start "STOP": held back
    b3, _ = ts.push(3)  # "ST" still a prefix
    b4, _ = ts.push(4)  # "STc" is not: released
    assert b1 + b2 + b3 + b4 == b"abSTc"
    assert b2 == b""


def test_textstream_utf8_completeness():
    v = _vocab()
    ts = core.TextStream(v, [])
    b1, _ = ts.push(6)  # first two bytes of the euro sign
    b2, _ = ts.push(7)
    assert b1 == b"" and b2 == "€".encode()


@pytest.mark.parametrize("n", [1, 7, 64])
def test_vocab_decode(n):
    v = _vocab()
    ids = [1, 2] * n
    assert v.decode(ids) == b"Hello" * n


def test_emit_run_matches_python_semantics():
    """Native multi-step token emitter vs. the per-token Python rules (EOS, stop strings with
    hold-back, max_tokens, context limit)."""
    pieces = [b"", b"Hel", b"lo", b" wor", b"ld", b"<eot>", b"ST", b"OP", b"!"]
    v = core.Vocab(pieces)
    K, B = 6, 5
    hist = np.array([[1, 1, 1, 1, 1],
                     [2, 2, 6, 2, 2],
                     [3, 5, 7, 3, 3],
                     [4, 3, 8, 4, 4],
                     [8, 4, 8, 8, 8],
                     [8, 8, 8, 8, 8]], dtype=np.int32)
    streams = [core.TextStream(v, ["STOP"] if j == 2 else []) for j in range(B)]
    # n_gen, max_tokens, n_prompt, ignore_eos, active
    st = np.array([[0, -1, 3, 0, 1],      # runs all 6 tokens
                   [0, -1, 3, 0, 1],      # EOS at k=2
                   [0, -1, 3, 0, 1],      # stop string STOP at k=2
                   [2, 5, 3, 0, 1],       # max_tokens hit after 3 tokens
                   [0, -1, 508, 0, 1]],   # context 512 hit after 4 tokens
                  dtype=np.int32)
    n_acc, reason, texts = core.emit_run(hist, K, B, streams, [None] * B, st, [5], 512)
    assert list(n_acc) == [6, 3, 3, 3, 4]
    assert list(reason) == [0, 1, 2, 3, 3]
    assert texts[0] == b"Hello world!!"
    assert texts[1] == b"Hello"
    assert texts[2] is None or texts[2] == b"Hel"
    assert texts[3] == b"Hello wor"
    assert texts[4] == b"Hello world"


def test_json_escape_keeps_output_valid_utf8():
    """SSE chunks are built in C++ from raw token bytes; dangling or malformed UTF-8 (byte-fallback
    tokens that never complete a code point) must become U+FFFD so every chunk parses as JSON."""
    import json

    def esc(raw):
        out = core.json_escape(raw)
        return out if isinstance(out, bytes) else out.encode("utf-8", "surrogateescape")

    for raw in [b"plain \"q\" \\ \n\t\x01", "h\u00e9llo \u20ac \U0001d11e".encode()]:
        assert json.loads(b'"' + esc(raw) + b'"') == raw.decode()
    for raw in [b"\xdf(", b"ab\xe2\x82", b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xff", b"\x80x"]:
        out = esc(raw)
        out.decode("utf-8")  # strict: valid UTF-8
        s = json.loads(b'"' + out + b'"')
        assert "\ufffd" in s and s.replace("\ufffd", "") == raw.decode("utf-8", "ignore")
