"""Pre-GGUF llama.cpp model files (`ggjt` v3, the last GGML container before GGUF): the reference's
`llama-ggml` backend (go-llama.cpp, `backend/go/llm/llama-ggml/llama.go`), served by
this engine through the same reader interface as `gguf.GGUFReader`.

File layout: magic `ggjt`, version 3, hyper-parameters (n_vocab, n_embd, n_mult, n_head, n_layer,
n_rot, ftype as int32), the SentencePiece vocabulary (length-prefixed piece bytes + f32 score per
token), then tensors until EOF (n_dims, name length, ggml type, dims innermost first, name, data
aligned to 32 bytes).  Block formats are the GGUF ones at this version.  Names map to GGUF names
(`tok_embeddings` -> `token_embd`, `layers.N.attention.wq` -> `blk.N.attn_q`, `feed_forward.w1/w2/w3`
-> `ffn_gate/down/up`, ...).  Q/K rows are already in the interleaved RoPE layout.  The file
carries no GQA factor or RMS epsilon: LLaMA-2-70B GGML files need the model config's `ngqa: 8`
(and `rms_norm_eps`), exactly as the reference's llama-ggml options require
(`core/backend/options.go` NGQA / RMSNormEps).  ggjt v1/v2 (older block layouts) are refused.
"""
from __future__ import annotations

import mmap
import re
import struct
from typing import Any, Dict, Optional

import numpy as np

from ..gguf import GGML_BLOCK, GGUFTensor, type_nbytes

MAGIC_GGJT = 0x67676A74  # 'ggjt'
T_NORMAL, T_UNKNOWN, T_CONTROL, T_BYTE = 1, 2, 3, 6

_NAME_MAP = [
    (r"^tok_embeddings\.weight$", "token_embd.weight"),
    (r"^norm\.weight$", "output_norm.weight"),
    (r"^output\.weight$", "output.weight"),
    (r"^layers\.(\d+)\.attention\.wq\.weight$", r"blk.\1.attn_q.weight"),
    (r"^layers\.(\d+)\.attention\.wk\.weight$", r"blk.\1.attn_k.weight"),
    (r"^layers\.(\d+)\.attention\.wv\.weight$", r"blk.\1.attn_v.weight"),
    (r"^layers\.(\d+)\.attention\.wo\.weight$", r"blk.\1.attn_output.weight"),
    (r"^layers\.(\d+)\.attention_norm\.weight$", r"blk.\1.attn_norm.weight"),
    (r"^layers\.(\d+)\.feed_forward\.w1\.weight$", r"blk.\1.ffn_gate.weight"),
    (r"^layers\.(\d+)\.feed_forward\.w2\.weight$", r"blk.\1.ffn_down.weight"),
    (r"^layers\.(\d+)\.feed_forward\.w3\.weight$", r"blk.\1.ffn_up.weight"),
    (r"^layers\.(\d+)\.ffn_norm\.weight$", r"blk.\1.ffn_norm.weight"),
]


def is_ggjt(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            head = f.read(4)
    except OSError:
        return False
    return len(head) == 4 and struct.unpack("<I", head)[0] == MAGIC_GGJT


def gguf_name(name: str) -> Optional[str]:
    for pat, rep in _NAME_MAP:
        if re.match(pat, name):
            return re.sub(pat, rep, name)
    return None


class GGJTReader:
    def __init__(self, path: str, n_gqa: int = 1, rms_norm_eps: float = 0.0, context_length: int = 2048):
        self.path = path
        self._f = open(path, "rb")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        mm = self._mm
        magic, version = struct.unpack_from("<II", mm, 0)
        if magic != MAGIC_GGJT:
            raise ValueError(f"{path}: not a ggjt file")
        if version != 3:
            raise ValueError(f"{path}: ggjt v{version} uses pre-v3 block layouts; re-quantise or convert to GGUF")
        n_vocab, n_embd, n_mult, n_head, n_layer, n_rot, ftype = struct.unpack_from("<7i", mm, 8)
        pos = 36
        tokens, scores, types = [], [], []
        for i in range(n_vocab):
            (ln,) = struct.unpack_from("<I", mm, pos)
            pos += 4
            piece = mm[pos:pos + ln].decode("utf-8", errors="replace")
            pos += ln
            (sc,) = struct.unpack_from("<f", mm, pos)
            pos += 4
            tokens.append(piece)
            scores.append(float(sc))
            types.append(T_UNKNOWN if i == 0 else T_CONTROL if i in (1, 2)
                         else T_BYTE if re.fullmatch(r"<0x[0-9A-Fa-f]{2}>", piece) else T_NORMAL)
        self.tensors: Dict[str, GGUFTensor] = {}
        size = len(mm)
        while pos < size:
            n_dims, name_len, t = struct.unpack_from("<3i", mm, pos)
            pos += 12
            ne = struct.unpack_from(f"<{n_dims}i", mm, pos)
            pos += 4 * n_dims
            name = mm[pos:pos + name_len].decode("utf-8")
            pos += name_len
            pos = (pos + 31) // 32 * 32
            if t not in GGML_BLOCK:
                raise ValueError(f"{path}: tensor {name} has unsupported ggml type {t}")
            n = int(np.prod(ne))
            nb = type_nbytes(t, n)
            g = gguf_name(name)
            if g is None:
                raise ValueError(f"{path}: unexpected tensor {name}")
            data = np.frombuffer(mm, dtype=np.uint8, count=nb, offset=pos)
            self.tensors[g] = GGUFTensor(g, tuple(int(x) for x in reversed(ne)), int(t), pos, nb, data)
            pos += nb
        n_ff = self.tensors["blk.0.ffn_gate.weight"].shape[0] if "blk.0.ffn_gate.weight" in self.tensors else \
            ((2 * (4 * n_embd) // 3 + n_mult - 1) // n_mult) * n_mult
        n_kv = max(1, n_head // max(1, int(n_gqa or 1)))
        kq = self.tensors.get("blk.0.attn_k.weight")
        if kq is not None:  # the k projection's rows give the kv heads (ngqa is then only a cross-check)
            n_kv = n_head * kq.shape[0] // n_embd
        a = "llama"
        self.kv: Dict[str, Any] = {
            "general.architecture": a, "general.name": path.rsplit("/", 1)[-1],
            f"{a}.context_length": int(context_length), f"{a}.embedding_length": n_embd,
            f"{a}.block_count": n_layer, f"{a}.feed_forward_length": int(n_ff),
            f"{a}.attention.head_count": n_head, f"{a}.attention.head_count_kv": int(n_kv),
            f"{a}.rope.dimension_count": n_rot or n_embd // n_head, f"{a}.rope.freq_base": 10000.0,
            f"{a}.attention.layer_norm_rms_epsilon": float(rms_norm_eps or 5e-6),
            "tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": tokens, "tokenizer.ggml.scores": scores,
            "tokenizer.ggml.token_type": types, "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2,
            "tokenizer.ggml.add_bos_token": True, "tokenizer.ggml.add_space_prefix": True,
            "general.file_type": ftype,
        }

    @property
    def architecture(self) -> str:
        return "llama"

    def get(self, key: str, default=None):
        return self.kv.get(key, default)

    def arch_kv(self, suffix: str, default=None):
        return self.kv.get(f"llama.{suffix}", default)

    def close(self):
        self.tensors = {}
        try:
            self._mm.close()
        except BufferError:
            pass
        self._f.close()


def write_ggjt(path: str, gguf_path: str) -> str:
    """Re-containerise a llama-architecture GGUF with a SentencePiece vocabulary as a ggjt v3 file
    (tests: the same tensor bytes must give the same model through both readers)."""
    from ..gguf import GGUFReader
    r = GGUFReader(gguf_path)
    a = r.architecture
    kv = r.kv
    inv = {}
    names = {"token_embd.weight": "tok_embeddings.weight", "output_norm.weight": "norm.weight",
             "output.weight": "output.weight"}
    per = {"attn_q": "attention.wq", "attn_k": "attention.wk", "attn_v": "attention.wv", "attn_output": "attention.wo",
           "attn_norm": "attention_norm", "ffn_gate": "feed_forward.w1", "ffn_down": "feed_forward.w2",
           "ffn_up": "feed_forward.w3", "ffn_norm": "ffn_norm"}
    for g in r.tensors:
        m = re.match(r"^blk\.(\d+)\.([a-z_]+)\.weight$", g)
        inv[g] = names.get(g) or (f"layers.{m.group(1)}.{per[m.group(2)]}.weight" if m and m.group(2) in per else None)
    toks, scores = kv["tokenizer.ggml.tokens"], kv.get("tokenizer.ggml.scores") or [0.0] * len(kv["tokenizer.ggml.tokens"])
    n_embd = int(kv[f"{a}.embedding_length"])
    with open(path, "wb") as f:
        f.write(struct.pack("<II", MAGIC_GGJT, 3))
        f.write(struct.pack("<7i", len(toks), n_embd, 256, int(kv[f"{a}.attention.head_count"]),
                            int(kv[f"{a}.block_count"]), int(kv.get(f"{a}.rope.dimension_count", 0)), 0))
        for t, s in zip(toks, scores):
            b = t.encode("utf-8")
            f.write(struct.pack("<I", len(b)) + b + struct.pack("<f", float(s)))
        for g, t in r.tensors.items():
            name = inv.get(g)
            if name is None:
                continue
            ne = list(reversed(t.shape))
            nb = name.encode()
            f.write(struct.pack("<3i", len(ne), len(nb), t.ggml_type) + struct.pack(f"<{len(ne)}i", *ne) + nb)
            f.write(b"\0" * ((-f.tell()) % 32))
            f.write(t.data.tobytes())
    r.close()
    return path
