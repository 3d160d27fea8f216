"""BERT-family sentence-embedding encoder from a llama.cpp `bert` GGUF (all-MiniLM, bge, e5 ...):
the reference's `bert-embeddings` backend (bert.cpp) and the embeddings half of its
sentencetransformers backend, as one native engine.

WordPiece tokenisation follows llama.cpp's WPM conventions for converted vocabularies (word
pieces that start a word carry a leading U+2581, continuation pieces are stored bare);
encoder = post-LayerNorm transformer with bidirectional attention; pooling mean (default) or
CLS, L2-normalised.

Cross-encoder rerankers (llama.cpp pooling_type 4 = RANK; `cls.weight`/`cls.bias` dense + tanh,
then `cls.output.weight`/`cls.output.bias` to one logit) score "[CLS] query [SEP] doc [SEP]"
pairs with segment ids 0/1: the reference's `rerankers` Python backend
(`backend/python/rerankers/backend.py:60-95`, Jina `/v1/rerank`) on this engine.
"""
from __future__ import annotations

import unicodedata
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..gguf import dequantize

SPACE = "▁"


def _is_punct(ch: str) -> bool:
    cp = ord(ch)
    if 33 <= cp <= 47 or 58 <= cp <= 64 or 91 <= cp <= 96 or 123 <= cp <= 126:
        return True
    return unicodedata.category(ch).startswith("P")


class WordPiece:
    def __init__(self, tokens: Sequence[str], unk: int, cls: int, sep: int, max_chars: int = 100):
        self.vocab: Dict[str, int] = {}
        for i, t in enumerate(tokens):
            self.vocab.setdefault(t, i)
        self.unk, self.cls, self.sep, self.max_chars = unk, cls, sep, max_chars
        self.max_piece = max((len(t) for t in tokens), default=1)

    @staticmethod
    def basic(text: str) -> List[str]:
        text = unicodedata.normalize("NFD", text.lower())
        text = "".join(c for c in text if unicodedata.category(c) != "Mn")
        words, cur = [], []
        for ch in text:
            if ch.isspace():
                if cur:
                    words.append("".join(cur))
                    cur = []
            elif _is_punct(ch) or 0x4E00 <= ord(ch) <= 0x9FFF:
                if cur:
                    words.append("".join(cur))
                    cur = []
                words.append(ch)
            elif unicodedata.category(ch) not in ("Cc", "Cf"):
                cur.append(ch)
        if cur:
            words.append("".join(cur))
        return words

    def encode(self, text: str, add_special: bool = True) -> List[int]:
        out = [self.cls] if add_special else []
        for w in self.basic(text):
            word = SPACE + w
            if len(word) > self.max_chars:
                out.append(self.unk)
                continue
            pieces, start, ok = [], 0, True
            while start < len(word):
                end = min(len(word), start + self.max_piece)
                tid = None
                while end > start:
                    tid = self.vocab.get(word[start:end])
                    if tid is not None:
                        break
                    end -= 1
                if tid is None:
                    ok = False
                    break
                pieces.append(tid)
                start = end
            out.extend(pieces if ok else [self.unk])
        if add_special:
            out.append(self.sep)
        return out


@dataclass
class BertConfig:
    model_path: str
    device: str = "cpu"
    context_size: int = 512


class BertEmbedder:
    """Minimal engine facade (embed / tokenize) the gRPC servicer can host."""

    def __init__(self, cfg: BertConfig):
        self.cfg = cfg
        self.device = torch.device(cfg.device)
        from .hf_checkpoint import open_model
        r = open_model(cfg.model_path)  # bert GGUF or an HF BertModel / cross-encoder checkpoint
        kv = r.kv
        a = r.architecture
        self.arch = a
        self.dim = int(kv[f"{a}.embedding_length"])
        self.n_layer = int(kv[f"{a}.block_count"])
        self.heads = int(kv[f"{a}.attention.head_count"])
        self.eps = float(kv.get(f"{a}.attention.layer_norm_epsilon", 1e-12))
        self.max_pos = int(kv.get(f"{a}.context_length", 512))
        self.pooling = int(kv.get(f"{a}.pooling_type", 1))  # 1 mean, 2 cls, 4 rank
        toks = [t if isinstance(t, str) else t.decode("utf-8", "replace") for t in kv["tokenizer.ggml.tokens"]]

        def tid(name, default):
            v = kv.get(name)
            return int(v) if v is not None else toks.index(default) if default in toks else 0
        self.tok = WordPiece(toks, tid("tokenizer.ggml.unknown_token_id", "[UNK]"),
                             tid("tokenizer.ggml.cls_token_id", "[CLS]"),
                             tid("tokenizer.ggml.seperator_token_id", "[SEP]"))
        T = r.tensors
        dt = torch.bfloat16 if self.device.type == "cuda" else torch.float32

        def t(name, required=True, mm=False):
            if name not in T:
                if required:
                    raise KeyError(f"bert GGUF: missing tensor {name}")
                return None
            x = T[name]
            v = torch.from_numpy(np.ascontiguousarray(dequantize(x.data, x.ggml_type, x.shape).reshape(x.shape),
                                                      dtype=np.float32)).to(self.device)
            return v.to(dt) if mm else v
        self.mmdt = dt
        self.tok_emb = t("token_embd.weight")
        self.type_emb = t("token_types.weight", False)
        self.pos_emb = t("position_embd.weight")
        self.emb_ln = (t("token_embd_norm.weight"), t("token_embd_norm.bias"))
        self.layers = []
        for i in range(self.n_layer):
            b = f"blk.{i}."
            qkv = torch.cat([t(b + "attn_q.weight"), t(b + "attn_k.weight"), t(b + "attn_v.weight")], 0).to(dt)
            qkv_b = torch.cat([t(b + "attn_q.bias"), t(b + "attn_k.bias"), t(b + "attn_v.bias")], 0)
            self.layers.append(dict(
                qkv=qkv, qkv_b=qkv_b, o=t(b + "attn_output.weight", mm=True), o_b=t(b + "attn_output.bias"),
                ln1=(t(b + "attn_output_norm.weight"), t(b + "attn_output_norm.bias")),
                up=t(b + "ffn_up.weight", mm=True), up_b=t(b + "ffn_up.bias"),
                down=t(b + "ffn_down.weight", mm=True), down_b=t(b + "ffn_down.bias"),
                ln2=(t(b + "layer_output_norm.weight"), t(b + "layer_output_norm.bias"))))
        # classification head of a cross-encoder (absent in sentence-embedding models)
        self.cls_w, self.cls_b = t("cls.weight", False), t("cls.bias", False)
        self.cls_out_w, self.cls_out_b = t("cls.output.weight", False), t("cls.output.bias", False)
        self.busy = False
        self.last_request_stats = {}

    def tokenize(self, text: str, add_bos=None) -> List[int]:
        return self.tok.encode(text)

    @property
    def is_ranker(self) -> bool:
        return self.cls_out_w is not None

    @torch.no_grad()
    def _hidden(self, ids: List[int], types: Optional[List[int]] = None) -> torch.Tensor:
        ids = ids[: self.max_pos]
        n = len(ids)
        D, H = self.dim, self.heads
        it = torch.tensor(ids, dtype=torch.long, device=self.device)
        x = self.tok_emb[it] + self.pos_emb[:n]
        if self.type_emb is not None:
            if types is not None and self.type_emb.shape[0] > 1:
                tt = torch.tensor(types[:n], dtype=torch.long, device=self.device)
                x = x + self.type_emb[tt]
            else:
                x = x + self.type_emb[0]
        x = F.layer_norm(x, (D,), self.emb_ln[0], self.emb_ln[1], self.eps)
        for ly in self.layers:
            qkv = (x.to(self.mmdt) @ ly["qkv"].t()).float() + ly["qkv_b"]
            q, k, v = qkv.view(n, 3, H, D // H).permute(1, 2, 0, 3).to(self.mmdt)
            a = F.scaled_dot_product_attention(q, k, v).transpose(0, 1).reshape(n, D)
            a = (a @ ly["o"].t()).float() + ly["o_b"]
            x = F.layer_norm(x + a, (D,), ly["ln1"][0], ly["ln1"][1], self.eps)
            h = F.gelu((x.to(self.mmdt) @ ly["up"].t()).float() + ly["up_b"])
            h = (h.to(self.mmdt) @ ly["down"].t()).float() + ly["down_b"]
            x = F.layer_norm(x + h, (D,), ly["ln2"][0], ly["ln2"][1], self.eps)
        return x

    def _encode(self, ids: List[int]) -> torch.Tensor:
        x = self._hidden(ids)
        v = x[0] if self.pooling in (2, 4) else x.mean(0)
        return F.normalize(v, dim=0)

    @torch.no_grad()
    def score(self, query: str, doc: str) -> float:
        """Cross-encoder relevance logit of (query, doc): CLS -> tanh(dense) -> 1 logit."""
        if not self.is_ranker:
            raise RuntimeError("this BERT model has no classification head (cls.output.weight)")
        q = self.tok.encode(query)                     # [CLS] q [SEP]
        d = self.tok.encode(doc, add_special=False) + [self.tok.sep]
        ids = q + d
        types = [0] * len(q) + [1] * len(d)
        c = self._hidden(ids, types)[0]
        if self.cls_w is not None:
            c = torch.tanh(c @ self.cls_w.t() + (self.cls_b if self.cls_b is not None else 0))
        y = c @ self.cls_out_w.t()
        if self.cls_out_b is not None:
            y = y + self.cls_out_b
        return float(y.reshape(-1)[0])

    def rerank(self, query: str, docs: Sequence[str]) -> List[float]:
        """Relevance in (0, 1) per document: sigmoid of the cross-encoder logit (the
        single-label CrossEncoder convention of sentence-transformers/rerankers)."""
        import math
        return [1.0 / (1.0 + math.exp(-self.score(query, d))) for d in docs]

    def embed(self, texts: Sequence, pool: str = "mean", timeout: float = 600.0) -> List[List[float]]:
        out = []
        for t in texts:
            ids = self.tokenize(t) if isinstance(t, str) else list(t)
            out.append(self._encode(ids).float().cpu().tolist())
        return out

    def add_request(self, *a, **k):
        raise RuntimeError("this is an embedding-only (BERT) model: use /v1/embeddings")

    def start(self):
        pass

    def warmup(self, *a, **k):
        pass

    def shutdown(self):
        pass
