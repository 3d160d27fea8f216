"""Tokenizers built from GGUF metadata (what llama.cpp's llama-vocab does for the reference).

* ``gpt2`` vocab (byte-level BPE: Llama-3, Phi-2, Qwen...): HuggingFace `tokenizers` BPE
  model with the pre-tokenizer regex selected by ``tokenizer.ggml.pre``.
* ``llama`` vocab (SentencePiece BPE: Llama-2, Mistral, Mixtral): the score-driven bigram
  merge of llama.cpp's llm_tokenizer_spm, with <0xNN> byte fallback.

Special (control / user-defined) tokens are matched in the prompt text before BPE, like the
reference's TMP_FORCE_SPECIAL (`backend/cpp/llama/grpc-server.cpp:564`).
"""
from __future__ import annotations

import heapq
import re
from functools import lru_cache
from typing import Dict, List, Optional, Sequence

TOKEN_NORMAL, TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_USER_DEFINED, TOKEN_UNUSED, TOKEN_BYTE = 1, 2, 3, 4, 5, 6

LLAMA3_PAT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*"
              r"|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2_PAT = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"
QWEN2_PAT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*"
             r"|\s*[\r\n]+|\s+(?!\S)|\s+")
PRE_PATTERNS = {"llama-bpe": LLAMA3_PAT, "llama3": LLAMA3_PAT, "smaug-bpe": LLAMA3_PAT, "qwen2": QWEN2_PAT,
                "default": GPT2_PAT, "gpt2": GPT2_PAT, "phi-2": GPT2_PAT}


@lru_cache(maxsize=1)
def bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


@lru_cache(maxsize=1)
def unicode_to_bytes() -> Dict[str, int]:
    return {v: k for k, v in bytes_to_unicode().items()}


class Tokenizer:
    def __init__(self, model: str, tokens: List[str], types: List[int], scores: Optional[List[float]],
                 merges: Optional[List[str]], bos: int, eos: int, add_bos: bool, pre: str = "default",
                 eot: Optional[int] = None, add_space_prefix: bool = True, chat_template: str = "",
                 hf_json: str = ""):
        self.model = model
        self.tokens = tokens
        self.types = types or [TOKEN_NORMAL] * len(tokens)
        self.scores = scores
        self.bos_id, self.eos_id, self.eot_id = bos, eos, eot
        self.add_bos = add_bos
        self.pre = pre
        self.chat_template = chat_template
        self.add_space_prefix = add_space_prefix
        self.vocab = {t: i for i, t in enumerate(tokens)}
        specials = [t for t, ty in zip(tokens, self.types) if ty in (TOKEN_CONTROL, TOKEN_USER_DEFINED) and t]
        specials.sort(key=len, reverse=True)
        self._special_re = re.compile("|".join(re.escape(s) for s in specials)) if specials else None
        self.eog = {x for x in (eos, eot) if x is not None and x >= 0}
        for i, (t, ty) in enumerate(zip(tokens, self.types)):
            if ty == TOKEN_CONTROL and t in ("<|eot_id|>", "<|end_of_text|>", "<|im_end|>", "<|endoftext|>",
                                              "<end_of_turn>", "</s>", "<|end|>"):
                self.eog.add(i)
        self._hf = None
        if model == "gpt2" and hf_json:
            # an HF checkpoint's tokenizer.json (models/hf_checkpoint.py): its own pre-tokenizer and
            # BPE model; specials are split off above, so no post-processor / added-token handling
            from tokenizers import Tokenizer as HFTok
            self._hf = HFTok.from_file(hf_json)
        elif model == "gpt2":
            self._init_bpe(merges or [])
        self.pieces = [self._piece_bytes(i) for i in range(len(tokens))]
        nl = self.encode("\n", add_bos=False)
        self.nl_id = nl[0] if len(nl) == 1 else -1

    # ----------------------------------------------------------------- construction
    @classmethod
    def from_gguf(cls, r) -> "Tokenizer":
        g = r.kv.get
        model = g("tokenizer.ggml.model", "gpt2")
        tokens = g("tokenizer.ggml.tokens")
        if tokens is None:
            raise ValueError("GGUF has no tokenizer.ggml.tokens")
        types = g("tokenizer.ggml.token_type")
        scores = g("tokenizer.ggml.scores")
        merges = g("tokenizer.ggml.merges")
        bos = int(g("tokenizer.ggml.bos_token_id", 1 if model == "llama" else -1))
        eos = int(g("tokenizer.ggml.eos_token_id", 2 if model == "llama" else -1))
        eot = g("tokenizer.ggml.eot_token_id")
        add_bos = bool(g("tokenizer.ggml.add_bos_token", model == "llama"))
        pre = g("tokenizer.ggml.pre", "default")
        asp = bool(g("tokenizer.ggml.add_space_prefix", model == "llama"))
        return cls(model, tokens, types, scores, merges, bos, eos, add_bos, pre, None if eot is None else int(eot),
                   asp, g("tokenizer.chat_template", "") or "", g("tokenizer.hf.json", "") or "")

    def _init_bpe(self, merges: List[str]):
        from tokenizers import Regex, Tokenizer as HFTok, decoders, models, pre_tokenizers
        pat = PRE_PATTERNS.get(self.pre, GPT2_PAT)
        mlist = [tuple(m.split(" ", 1)) for m in merges]
        ignore = self.pre in ("llama-bpe", "llama3", "smaug-bpe")
        bpe = models.BPE(vocab=self.vocab, merges=mlist, ignore_merges=ignore)
        tok = HFTok(bpe)
        tok.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Split(Regex(pat), behavior="isolated"),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
        tok.decoder = decoders.ByteLevel()
        self._hf = tok
        # fast path: the pre-tokenizer split in the `regex` module (~6x faster than the
        # tokenizers library's Split on the Llama-3 pattern: 37 vs 220 us for a 680-character
        # prompt) and BPE results cached per pre-token; misses go to a byte-level-only twin of
        # the same BPE model in one pre-tokenised call.  Same ids (tests/test_gguf.py).
        self._pre_re = None
        try:
            import regex
            self._pre_re = regex.compile(pat)
        except Exception:  # noqa: BLE001 - no `regex` module / pattern it cannot compile: HF path
            return
        twin = HFTok(models.BPE(vocab=self.vocab, merges=mlist, ignore_merges=ignore))
        twin.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)
        self._hf_words = twin
        self._word_cache: Dict[str, tuple] = {}

    _WORD_CACHE_SIZE = 1 << 17

    def _bpe_fast(self, s: str) -> List[int]:
        """Encode through the per-pre-token cache.  The output is built from a local map filled
        before any eviction, so a concurrent or size-triggered clear() of the shared cache (other
        gateway threads share this tokenizer) can never drop an entry this call still needs."""
        words = self._pre_re.findall(s)
        cache = self._word_cache
        got: Dict[str, tuple] = {}
        miss: List[str] = []
        for w in words:
            if w in got:
                continue
            hit = cache.get(w)
            if hit is None:
                miss.append(w)
                got[w] = ()
            else:
                got[w] = hit
        if miss:
            enc = self._hf_words.encode(miss, is_pretokenized=True, add_special_tokens=False)
            per: List[List[int]] = [[] for _ in miss]
            for t, wi in zip(enc.ids, enc.word_ids):
                per[wi].append(t)
            if len(cache) + len(miss) > self._WORD_CACHE_SIZE:
                cache.clear()
            for w, p in zip(miss, per):
                got[w] = cache[w] = tuple(p)
        out: List[int] = []
        for w in words:
            out.extend(got[w])
        return out

    def _piece_bytes(self, i: int) -> bytes:
        t, ty = self.tokens[i], self.types[i]
        if ty == TOKEN_CONTROL or ty == TOKEN_UNUSED:
            return b""
        if ty == TOKEN_USER_DEFINED:
            return t.encode("utf-8")
        if self.model == "gpt2":
            u2b = unicode_to_bytes()
            try:
                return bytes(u2b[c] for c in t)
            except KeyError:
                return t.encode("utf-8")
        if ty == TOKEN_BYTE and len(t) == 6 and t.startswith("<0x"):
            return bytes([int(t[3:5], 16)])
        return t.replace("▁", " ").encode("utf-8")

    # ----------------------------------------------------------------- API
    @property
    def vocab_size(self) -> int:
        return len(self.tokens)

    def is_eog(self, t: int) -> bool:
        return t in self.eog

    def encode(self, text: str, add_bos: Optional[bool] = None, parse_special: bool = True) -> List[int]:
        out: List[int] = []
        if add_bos is None:
            add_bos = self.add_bos
        if add_bos and self.bos_id is not None and self.bos_id >= 0:
            out.append(self.bos_id)
        parts = [(text, False)]
        if parse_special and self._special_re is not None:
            parts = []
            pos = 0
            for m in self._special_re.finditer(text):
                if m.start() > pos:
                    parts.append((text[pos:m.start()], False))
                parts.append((m.group(0), True))
                pos = m.end()
            if pos < len(text):
                parts.append((text[pos:], False))
        first = True
        for s, special in parts:
            if special:
                out.append(self.vocab[s])
            elif s:
                out.extend(self._encode_plain(s, first))
            first = False
        return out

    _PIECE_CACHE_MAX_LEN = 96     # chat-template pieces between special tokens ("user", "\n\n", ...)
    _PIECE_CACHE_SIZE = 8192

    def _encode_plain(self, s: str, at_start: bool) -> List[int]:
        # the short pieces a chat template puts between its special tokens recur on every request:
        # one dict hit instead of a tokenizer call (~0.1 ms of fixed cost each, 3 of the 4 calls
        # of a one-turn Llama-3 chat prompt; scripts/gateway_profile.py)
        short = len(s) <= self._PIECE_CACHE_MAX_LEN
        if short:
            c = self.__dict__.setdefault("_piece_cache", {})
            hit = c.get((s, at_start))
            if hit is not None:
                return list(hit)
        if self.model == "gpt2":
            if getattr(self, "_pre_re", None) is not None:
                ids = self._bpe_fast(s)
            else:
                ids = self._hf.encode(s, add_special_tokens=False).ids
        else:
            ids = self._spm_encode(s, at_start)
        if short:
            if len(c) >= self._PIECE_CACHE_SIZE:
                c.clear()
            c[(s, at_start)] = tuple(ids)
        return ids

    def decode(self, ids: Sequence[int]) -> str:
        return b"".join(self.pieces[i] for i in ids if 0 <= i < len(self.pieces)).decode("utf-8", errors="replace")

    def token_bytes(self, i: int) -> bytes:
        return self.pieces[i]

    # ----------------------------------------------------------------- SPM (llama.cpp llm_tokenizer_spm)
    def _spm_encode(self, text: str, at_start: bool) -> List[int]:
        if self.add_space_prefix and at_start:
            text = " " + text
        text = text.replace(" ", "▁")
        syms = list(text)
        n = len(syms)
        if n == 0:
            return []
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1
        alive = [True] * n
        heap = []
        scores = self.scores or [0.0] * len(self.tokens)
        rev: Dict[str, tuple] = {}

        def add_bigram(l, r):
            if l < 0 or r < 0:
                return
            t = syms[l] + syms[r]
            tid = self.vocab.get(t)
            if tid is None:
                return
            heapq.heappush(heap, (-scores[tid], l, r, t))

        for i in range(n - 1):
            add_bigram(i, i + 1)
        while heap:
            _, l, r, t = heapq.heappop(heap)
            if not alive[l] or not alive[r] or nxt[l] != r or syms[l] + syms[r] != t:
                continue
            rev[t] = (syms[l], syms[r])
            syms[l] = t
            alive[r] = False
            nxt[l] = nxt[r]
            if nxt[r] >= 0:
                prev[nxt[r]] = l
            add_bigram(prev[l], l)
            add_bigram(l, nxt[l])
        out: List[int] = []

        def resegment(s: str):
            tid = self.vocab.get(s)
            if tid is not None:
                out.append(tid)
                return
            pr = rev.get(s)
            if pr is not None:
                resegment(pr[0])
                resegment(pr[1])
                return
            for b in s.encode("utf-8"):
                bt = self.vocab.get(f"<0x{b:02X}>")
                out.append(bt if bt is not None else 0)

        i = 0
        while i != -1 and i < n:
            if alive[i]:
                resegment(syms[i])
            i = nxt[i]
        return out
