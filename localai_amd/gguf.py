"""GGUF container: reader (mmap, zero-copy), writer, and the block quantizers.

The reference never parses GGUF itself for inference (llama.cpp does, [external]);
it only reads the header for the template guesser (`core/config/guesser.go:145-246`)
and `local-ai util gguf-info` (`core/cli/util.go:39-135`).  This module serves
both roles for our engine: the model loader streams tensors from the mmap straight
into HBM and repacks quantized blocks there (see `localai_amd/ops`).

Quantized formats implemented (bit-exact with ggml's block layouts):
  Q8_0 (34 B / 32), Q4_K (144 B / 256), Q6_K (210 B / 256), plus F32/F16/BF16.
Dequantizers exist for Q4_0, Q5_K too (read-only support).
"""
from __future__ import annotations

import enum
import mmap
import os
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Optional, Tuple

import numpy as np

GGUF_MAGIC = 0x46554747  # "GGUF"
GGUF_VERSION = 3
GGUF_DEFAULT_ALIGNMENT = 32


class GGMLType(enum.IntEnum):
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    I8 = 24
    I16 = 25
    I32 = 26
    I64 = 27
    F64 = 28
    BF16 = 30


# (block size in elements, bytes per block)
GGML_BLOCK: Dict[int, Tuple[int, int]] = {
    GGMLType.F32: (1, 4),
    GGMLType.F16: (1, 2),
    GGMLType.BF16: (1, 2),
    GGMLType.Q4_0: (32, 18),
    GGMLType.Q4_1: (32, 20),
    GGMLType.Q5_0: (32, 22),
    GGMLType.Q5_1: (32, 24),
    GGMLType.Q8_0: (32, 34),
    GGMLType.Q2_K: (256, 84),
    GGMLType.Q3_K: (256, 110),
    GGMLType.Q4_K: (256, 144),
    GGMLType.Q5_K: (256, 176),
    GGMLType.Q6_K: (256, 210),
    GGMLType.Q8_K: (256, 292),
    GGMLType.I8: (1, 1),
    GGMLType.I16: (1, 2),
    GGMLType.I32: (1, 4),
    GGMLType.I64: (1, 8),
    GGMLType.F64: (1, 8),
}


class GGUFValueType(enum.IntEnum):
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


_SCALAR_FMT = {
    GGUFValueType.UINT8: "<B", GGUFValueType.INT8: "<b",
    GGUFValueType.UINT16: "<H", GGUFValueType.INT16: "<h",
    GGUFValueType.UINT32: "<I", GGUFValueType.INT32: "<i",
    GGUFValueType.FLOAT32: "<f", GGUFValueType.BOOL: "<?",
    GGUFValueType.UINT64: "<Q", GGUFValueType.INT64: "<q",
    GGUFValueType.FLOAT64: "<d",
}
_NP_OF_VT = {
    GGUFValueType.UINT8: np.uint8, GGUFValueType.INT8: np.int8,
    GGUFValueType.UINT16: np.uint16, GGUFValueType.INT16: np.int16,
    GGUFValueType.UINT32: np.uint32, GGUFValueType.INT32: np.int32,
    GGUFValueType.FLOAT32: np.float32, GGUFValueType.BOOL: np.bool_,
    GGUFValueType.UINT64: np.uint64, GGUFValueType.INT64: np.int64,
    GGUFValueType.FLOAT64: np.float64,
}


def type_nbytes(t: int, n_elements: int) -> int:
    bs, bb = GGML_BLOCK[t]
    if n_elements % bs:
        raise ValueError(f"{GGMLType(t).name}: {n_elements} elements not a multiple of block {bs}")
    return n_elements // bs * bb


@dataclass
class GGUFTensor:
    name: str
    shape: Tuple[int, ...]          # torch/numpy order (outermost first); ggml ne reversed
    ggml_type: int
    offset: int                      # absolute file offset of the data
    nbytes: int
    data: Optional[np.ndarray] = None  # uint8 view of the raw bytes (mmap-backed)

    @property
    def n_elements(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n

    @property
    def type_name(self) -> str:
        return GGMLType(self.ggml_type).name


class GGUFReader:
    """Zero-copy GGUF reader.  Tensor data are uint8 numpy views into an mmap."""

    def __init__(self, path: str, load_tensors: bool = True):
        self.path = path
        self._f = open(path, "rb")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        self.kv: Dict[str, Any] = {}
        self.kv_types: Dict[str, Tuple[int, Optional[int]]] = {}
        self.tensors: Dict[str, GGUFTensor] = {}
        self._parse(load_tensors)

    # -- low level -------------------------------------------------------
    def _read(self, fmt: str):
        v = struct.unpack_from(fmt, self._mm, self._pos)
        self._pos += struct.calcsize(fmt)
        return v[0]

    def _read_str(self) -> str:
        n = self._read("<Q")
        b = self._mm[self._pos:self._pos + n]
        self._pos += n
        return b.decode("utf-8", errors="replace")

    def _read_value(self, vt: int):
        if vt == GGUFValueType.STRING:
            return self._read_str()
        if vt == GGUFValueType.ARRAY:
            et = self._read("<I")
            n = self._read("<Q")
            if et == GGUFValueType.STRING:
                return [self._read_str() for _ in range(n)]
            if et == GGUFValueType.ARRAY:
                return [self._read_value(GGUFValueType.ARRAY) for _ in range(n)]
            dt = np.dtype(_NP_OF_VT[GGUFValueType(et)]).newbyteorder("<")
            arr = np.frombuffer(self._mm, dtype=dt, count=n, offset=self._pos).copy()
            self._pos += n * dt.itemsize
            return arr.tolist()
        return self._read(_SCALAR_FMT[GGUFValueType(vt)])

    def _parse(self, load_tensors: bool):
        self._pos = 0
        magic = self._read("<I")
        if magic != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file (magic {magic:#x})")
        self.version = self._read("<I")
        if self.version not in (2, 3):
            raise ValueError(f"{self.path}: unsupported GGUF version {self.version}")
        n_tensors = self._read("<Q")
        n_kv = self._read("<Q")
        for _ in range(n_kv):
            key = self._read_str()
            vt = self._read("<I")
            sub = None
            if vt == GGUFValueType.ARRAY:
                sub = struct.unpack_from("<I", self._mm, self._pos)[0]
            self.kv[key] = self._read_value(vt)
            self.kv_types[key] = (vt, sub)
        infos = []
        for _ in range(n_tensors):
            name = self._read_str()
            nd = self._read("<I")
            ne = [self._read("<Q") for _ in range(nd)]
            t = self._read("<I")
            off = self._read("<Q")
            infos.append((name, ne, t, off))
        align = int(self.kv.get("general.alignment", GGUF_DEFAULT_ALIGNMENT))
        self.data_offset = (self._pos + align - 1) // align * align
        for name, ne, t, off in infos:
            shape = tuple(int(x) for x in reversed(ne))
            n = 1
            for s in ne:
                n *= int(s)
            nb = type_nbytes(t, n)
            abs_off = self.data_offset + off
            data = None
            if load_tensors:
                data = np.frombuffer(self._mm, dtype=np.uint8, count=nb, offset=abs_off)
            self.tensors[name] = GGUFTensor(name, shape, t, abs_off, nb, data)

    # -- convenience -------------------------------------------------------
    def get(self, key: str, default=None):
        return self.kv.get(key, default)

    @property
    def architecture(self) -> str:
        return self.kv.get("general.architecture", "llama")

    def arch_kv(self, suffix: str, default=None):
        return self.kv.get(f"{self.architecture}.{suffix}", default)

    def close(self):
        for t in self.tensors.values():
            t.data = None
        try:
            self._mm.close()
        except BufferError:
            pass  # outstanding numpy views keep the map alive; GC will release it
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class GGUFWriter:
    """Streaming GGUF v3 writer.  Tensor payloads may be numpy arrays or callables
    producing raw bytes lazily (used to write multi-GB random-init models without
    holding them in RAM)."""

    def __init__(self, path: str, arch: str, alignment: int = GGUF_DEFAULT_ALIGNMENT):
        self.path = path
        self.alignment = alignment
        self.kv: List[Tuple[str, int, Any, Optional[int]]] = []
        self.tensors: List[Tuple[str, Tuple[int, ...], int, Any, int]] = []
        self.add_string("general.architecture", arch)
        if alignment != GGUF_DEFAULT_ALIGNMENT:
            self.add_uint32("general.alignment", alignment)

    # kv helpers
    def add(self, key: str, vt: int, value: Any, sub: Optional[int] = None):
        self.kv.append((key, int(vt), value, sub))

    def add_string(self, k, v): self.add(k, GGUFValueType.STRING, v)
    def add_uint32(self, k, v): self.add(k, GGUFValueType.UINT32, int(v))
    def add_int32(self, k, v): self.add(k, GGUFValueType.INT32, int(v))
    def add_float32(self, k, v): self.add(k, GGUFValueType.FLOAT32, float(v))
    def add_bool(self, k, v): self.add(k, GGUFValueType.BOOL, bool(v))
    def add_array(self, k, values, sub: int): self.add(k, GGUFValueType.ARRAY, values, sub)

    def add_tensor(self, name: str, shape: Tuple[int, ...], ggml_type: int, payload):
        n = 1
        for s in shape:
            n *= int(s)
        nb = type_nbytes(ggml_type, n)
        if isinstance(payload, np.ndarray):
            if payload.nbytes != nb:
                raise ValueError(f"{name}: payload {payload.nbytes} B != expected {nb} B")
        self.tensors.append((name, tuple(int(s) for s in shape), int(ggml_type), payload, nb))

    # serialisation
    @staticmethod
    def _pack_str(s: str) -> bytes:
        b = s.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    def _pack_value(self, vt: int, v, sub: Optional[int]) -> bytes:
        if vt == GGUFValueType.STRING:
            return self._pack_str(v)
        if vt == GGUFValueType.ARRAY:
            out = [struct.pack("<IQ", sub, len(v))]
            if sub == GGUFValueType.STRING:
                out.extend(self._pack_str(x) for x in v)
            else:
                dt = np.dtype(_NP_OF_VT[GGUFValueType(sub)]).newbyteorder("<")
                out.append(np.asarray(v, dtype=dt).tobytes())
            return b"".join(out)
        return struct.pack(_SCALAR_FMT[GGUFValueType(vt)], v)

    def write(self):
        hdr = [struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(self.tensors), len(self.kv))]
        for k, vt, v, sub in self.kv:
            hdr.append(self._pack_str(k) + struct.pack("<I", vt) + self._pack_value(vt, v, sub))
        off = 0
        offsets = []
        for name, shape, t, _, nb in self.tensors:
            offsets.append(off)
            ne = list(reversed(shape))
            hdr.append(self._pack_str(name) + struct.pack("<I", len(ne)) +
                       b"".join(struct.pack("<Q", x) for x in ne) + struct.pack("<IQ", t, off))
            off += (nb + self.alignment - 1) // self.alignment * self.alignment
        head = b"".join(hdr)
        pad = (-len(head)) % self.alignment
        with open(self.path, "wb") as f:
            f.write(head + b"\0" * pad)
            for (name, shape, t, payload, nb), o in zip(self.tensors, offsets):
                data = payload() if callable(payload) else payload
                if isinstance(data, np.ndarray):
                    data = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
                    if data.nbytes != nb:
                        raise ValueError(f"{name}: payload {data.nbytes} B != expected {nb} B")
                    f.write(memoryview(data))
                else:
                    if len(data) != nb:
                        raise ValueError(f"{name}: payload {len(data)} B != expected {nb} B")
                    f.write(data)
                f.write(b"\0" * ((-nb) % self.alignment))


# ---------------------------------------------------------------------------
# Quantizers (numpy, vectorised over blocks).  Layouts match ggml exactly.
# ---------------------------------------------------------------------------

def _f16(x) -> np.ndarray:
    return np.asarray(x, dtype=np.float32).astype(np.float16)


def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1)
    d = amax / 127.0
    inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0.0)
    q = np.clip(np.rint(x * inv[:, None]), -127, 127).astype(np.int8)
    out = np.zeros((x.shape[0], 34), dtype=np.uint8)
    out[:, 0:2] = _f16(d).view(np.uint8).reshape(-1, 2)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(-1)


def _pack_q4k_scales(sc: np.ndarray, mn: np.ndarray) -> np.ndarray:
    """sc, mn: [nb, 8] uint8 (6-bit) -> [nb, 12] packed (ggml get_scale_min_k4 inverse)."""
    nb = sc.shape[0]
    s = np.zeros((nb, 12), dtype=np.uint8)
    for j in range(4):
        s[:, j] = sc[:, j] & 63
        s[:, j + 4] = mn[:, j] & 63
    for j in range(4, 8):
        s[:, j + 4] = (sc[:, j] & 0xF) | ((mn[:, j] & 0xF) << 4)
        s[:, j - 4] |= (sc[:, j] >> 4) << 6
        s[:, j] |= (mn[:, j] >> 4) << 6
    return s


def unpack_q4k_scales(s: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """[nb, 12] -> (sc [nb,8], mn [nb,8]) as uint8."""
    s = s.astype(np.uint8)
    sc = np.zeros((s.shape[0], 8), dtype=np.uint8)
    mn = np.zeros((s.shape[0], 8), dtype=np.uint8)
    for j in range(4):
        sc[:, j] = s[:, j] & 63
        mn[:, j] = s[:, j + 4] & 63
    for j in range(4, 8):
        sc[:, j] = (s[:, j + 4] & 0xF) | ((s[:, j - 4] >> 6) << 4)
        mn[:, j] = (s[:, j + 4] >> 4) | ((s[:, j] >> 6) << 4)
    return sc, mn


def quantize_q4_k(x: np.ndarray) -> np.ndarray:
    """Asymmetric min/max quantiser producing valid ggml Q4_K blocks."""
    x = np.asarray(x, dtype=np.float32).reshape(-1, 8, 32)
    nb = x.shape[0]
    mn = np.minimum(x.min(axis=2), 0.0)            # [nb,8]  (<= 0)
    mx = x.max(axis=2)
    scale = (mx - mn) / 15.0                        # per sub-block
    mins = -mn                                       # >= 0
    max_scale = scale.max(axis=1)
    max_min = mins.max(axis=1)
    d = np.where(max_scale > 0, max_scale / 63.0, 0.0).astype(np.float32)
    dmin = np.where(max_min > 0, max_min / 63.0, 0.0).astype(np.float32)
    d16 = _f16(d).astype(np.float32)
    dm16 = _f16(dmin).astype(np.float32)
    inv_d = np.where(d16 > 0, 1.0 / np.where(d16 > 0, d16, 1), 0.0)
    inv_m = np.where(dm16 > 0, 1.0 / np.where(dm16 > 0, dm16, 1), 0.0)
    ls = np.clip(np.rint(scale * inv_d[:, None]), 0, 63).astype(np.uint8)
    lm = np.clip(np.rint(mins * inv_m[:, None]), 0, 63).astype(np.uint8)
    eff_d = d16[:, None] * ls.astype(np.float32)          # [nb,8]
    eff_m = dm16[:, None] * lm.astype(np.float32)
    inv_eff = np.where(eff_d > 0, 1.0 / np.where(eff_d > 0, eff_d, 1), 0.0)
    L = np.clip(np.rint((x + eff_m[:, :, None]) * inv_eff[:, :, None]), 0, 15).astype(np.uint8)
    L = L.reshape(nb, 256)
    out = np.zeros((nb, 144), dtype=np.uint8)
    out[:, 0:2] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dm16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(ls, lm)
    qs = np.zeros((nb, 128), dtype=np.uint8)
    for c in range(4):
        lo = L[:, 64 * c: 64 * c + 32]
        hi = L[:, 64 * c + 32: 64 * c + 64]
        qs[:, 32 * c: 32 * c + 32] = lo | (hi << 4)
    out[:, 16:] = qs
    return out.reshape(-1)


def quantize_q5_k(x: np.ndarray) -> np.ndarray:
    """Asymmetric min/max quantiser producing valid ggml Q5_K blocks (d, dmin, the Q4_K 6-bit
    scale/min packing, qh[32] high bits -- bit 2c of byte l for sub-block 2c, bit 2c+1 for 2c+1 --
    and qs[128] low nibbles)."""
    x = np.asarray(x, dtype=np.float32).reshape(-1, 8, 32)
    nb = x.shape[0]
    mn = np.minimum(x.min(axis=2), 0.0)
    scale = (x.max(axis=2) - mn) / 31.0
    mins = -mn
    d = np.where(scale.max(axis=1) > 0, scale.max(axis=1) / 63.0, 0.0).astype(np.float32)
    dmin = np.where(mins.max(axis=1) > 0, mins.max(axis=1) / 63.0, 0.0).astype(np.float32)
    d16 = _f16(d).astype(np.float32)
    dm16 = _f16(dmin).astype(np.float32)
    inv_d = np.where(d16 > 0, 1.0 / np.where(d16 > 0, d16, 1), 0.0)
    inv_m = np.where(dm16 > 0, 1.0 / np.where(dm16 > 0, dm16, 1), 0.0)
    ls = np.clip(np.rint(scale * inv_d[:, None]), 0, 63).astype(np.uint8)
    lm = np.clip(np.rint(mins * inv_m[:, None]), 0, 63).astype(np.uint8)
    eff_d = d16[:, None] * ls.astype(np.float32)
    eff_m = dm16[:, None] * lm.astype(np.float32)
    inv_eff = np.where(eff_d > 0, 1.0 / np.where(eff_d > 0, eff_d, 1), 0.0)
    L = np.clip(np.rint((x + eff_m[:, :, None]) * inv_eff[:, :, None]), 0, 31).astype(np.uint8).reshape(nb, 256)
    out = np.zeros((nb, 176), dtype=np.uint8)
    out[:, 0:2] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = dm16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(ls, lm)
    qh = np.zeros((nb, 32), dtype=np.uint8)
    qs = np.zeros((nb, 128), dtype=np.uint8)
    for c in range(4):
        lo = L[:, 64 * c: 64 * c + 32]
        hi = L[:, 64 * c + 32: 64 * c + 64]
        qs[:, 32 * c: 32 * c + 32] = (lo & 0xF) | ((hi & 0xF) << 4)
        qh |= ((lo >> 4) << (2 * c)) | ((hi >> 4) << (2 * c + 1))
    out[:, 16:48] = qh
    out[:, 48:] = qs
    return out.reshape(-1)


def quantize_q6_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32).reshape(-1, 16, 16)
    nb = x.shape[0]
    amax_sub = np.abs(x).max(axis=2)                        # [nb,16]
    s = amax_sub / 31.0
    max_s = s.max(axis=1)
    d = np.where(max_s > 0, max_s / 127.0, 0.0)
    d16 = _f16(d).astype(np.float32)
    inv_d = np.where(d16 > 0, 1.0 / np.where(d16 > 0, d16, 1), 0.0)
    sc = np.clip(np.rint(s * inv_d[:, None]), -128, 127).astype(np.int8)
    eff = d16[:, None] * sc.astype(np.float32)
    inv_eff = np.where(eff != 0, 1.0 / np.where(eff != 0, eff, 1), 0.0)
    L = (np.clip(np.rint(x * inv_eff[:, :, None]), -32, 31) + 32).astype(np.uint8).reshape(nb, 256)
    ql = np.zeros((nb, 128), dtype=np.uint8)
    qh = np.zeros((nb, 64), dtype=np.uint8)
    for h in range(2):
        Lh = L[:, 128 * h: 128 * h + 128]
        q1, q2, q3, q4 = Lh[:, 0:32], Lh[:, 32:64], Lh[:, 64:96], Lh[:, 96:128]
        ql[:, 64 * h: 64 * h + 32] = (q1 & 0xF) | ((q3 & 0xF) << 4)
        ql[:, 64 * h + 32: 64 * h + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
        qh[:, 32 * h: 32 * h + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    out = np.zeros((nb, 210), dtype=np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = d16.astype(np.float16).view(np.uint8).reshape(-1, 2)
    return out.reshape(-1)


def quantize(x: np.ndarray, t: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float32)
    if t == GGMLType.F32:
        return x.astype(np.float32).reshape(-1).view(np.uint8)
    if t == GGMLType.F16:
        return x.astype(np.float16).reshape(-1).view(np.uint8)
    if t == GGMLType.BF16:
        u = x.reshape(-1).view(np.uint32)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
        return r.view(np.uint8)
    if t == GGMLType.Q8_0:
        return quantize_q8_0(x)
    if t == GGMLType.Q4_K:
        return quantize_q4_k(x)
    if t == GGMLType.Q6_K:
        return quantize_q6_k(x)
    if t == GGMLType.Q5_K:
        return quantize_q5_k(x)
    raise NotImplementedError(f"quantize to {GGMLType(t).name}")


# ---------------------------------------------------------------------------
# Dequantizers (numpy).  Used by the reference model and by tests.
# ---------------------------------------------------------------------------

def dequantize(raw: np.ndarray, t: int, shape: Tuple[int, ...]) -> np.ndarray:
    raw = np.asarray(raw, dtype=np.uint8).reshape(-1)
    n = int(np.prod(shape))
    if t == GGMLType.F32:
        return raw.view(np.float32).reshape(shape).copy()
    if t == GGMLType.F16:
        return raw.view(np.float16).astype(np.float32).reshape(shape)
    if t == GGMLType.BF16:
        return (raw.view(np.uint16).astype(np.uint32) << 16).view(np.float32).reshape(shape)
    if t == GGMLType.Q8_0:
        b = raw.reshape(-1, 34)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
        q = b[:, 2:].view(np.int8).astype(np.float32)
        return (q * d).reshape(shape)
    if t == GGMLType.Q4_0:
        b = raw.reshape(-1, 18)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
        qs = b[:, 2:]
        lo = (qs & 0xF).astype(np.float32) - 8
        hi = (qs >> 4).astype(np.float32) - 8
        return (np.concatenate([lo, hi], axis=1) * d).reshape(shape)
    if t == GGMLType.Q4_K:
        b = raw.reshape(-1, 144)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
        dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
        sc, mn = unpack_q4k_scales(b[:, 4:16])
        qs = b[:, 16:]
        out = np.empty((b.shape[0], 256), dtype=np.float32)
        for c in range(4):
            q = qs[:, 32 * c: 32 * c + 32]
            d1 = d * sc[:, 2 * c]; m1 = dmin * mn[:, 2 * c]
            d2 = d * sc[:, 2 * c + 1]; m2 = dmin * mn[:, 2 * c + 1]
            out[:, 64 * c: 64 * c + 32] = d1[:, None] * (q & 0xF) - m1[:, None]
            out[:, 64 * c + 32: 64 * c + 64] = d2[:, None] * (q >> 4) - m2[:, None]
        return out.reshape(shape)
    if t == GGMLType.Q5_K:
        b = raw.reshape(-1, 176)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
        dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
        sc, mn = unpack_q4k_scales(b[:, 4:16])
        qh = b[:, 16:48]
        qs = b[:, 48:176]
        out = np.empty((b.shape[0], 256), dtype=np.float32)
        for c in range(4):
            q = qs[:, 32 * c: 32 * c + 32]
            u1 = 1 << (2 * c); u2 = 2 << (2 * c)
            lo = (q & 0xF) + np.where(qh & u1, 16, 0)
            hi = (q >> 4) + np.where(qh & u2, 16, 0)
            d1 = d * sc[:, 2 * c]; m1 = dmin * mn[:, 2 * c]
            d2 = d * sc[:, 2 * c + 1]; m2 = dmin * mn[:, 2 * c + 1]
            out[:, 64 * c: 64 * c + 32] = d1[:, None] * lo - m1[:, None]
            out[:, 64 * c + 32: 64 * c + 64] = d2[:, None] * hi - m2[:, None]
        return out.reshape(shape)
    if t == GGMLType.Q6_K:
        b = raw.reshape(-1, 210)
        ql = b[:, 0:128].astype(np.int32)
        qh = b[:, 128:192].astype(np.int32)
        sc = b[:, 192:208].view(np.int8).astype(np.float32)
        d = b[:, 208:210].copy().view(np.float16).astype(np.float32)[:, 0]
        out = np.empty((b.shape[0], 256), dtype=np.float32)
        for h in range(2):
            L = ql[:, 64 * h: 64 * h + 64]
            H = qh[:, 32 * h: 32 * h + 32]
            S = sc[:, 8 * h: 8 * h + 8]
            q1 = ((L[:, 0:32] & 0xF) | (((H >> 0) & 3) << 4)) - 32
            q2 = ((L[:, 32:64] & 0xF) | (((H >> 2) & 3) << 4)) - 32
            q3 = ((L[:, 0:32] >> 4) | (((H >> 4) & 3) << 4)) - 32
            q4 = ((L[:, 32:64] >> 4) | (((H >> 6) & 3) << 4)) - 32
            for qi, (qv, base) in enumerate(((q1, 0), (q2, 32), (q3, 64), (q4, 96))):
                # sub-block index for l in [0,16) is is=0, for [16,32) is=1 ; +2*qi
                s_lo = S[:, 2 * qi][:, None]
                s_hi = S[:, 2 * qi + 1][:, None]
                sv = np.concatenate([np.repeat(s_lo, 16, axis=1), np.repeat(s_hi, 16, axis=1)], axis=1)
                out[:, 128 * h + base: 128 * h + base + 32] = d[:, None] * sv * qv
        return out.reshape(shape)
    if t in (GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1):
        # legacy 32-element blocks (ggml-quants.c dequantize_row_q4_1 / q5_0 / q5_1):
        # fp16 d [, fp16 m] [, u32 high bits], 16 bytes of nibbles (element j low, j + 16 high)
        nb = GGML_BLOCK[t][1]
        b = raw.reshape(-1, nb)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
        o = 2
        m = None
        if t != GGMLType.Q5_0:
            m = b[:, 2:4].copy().view(np.float16).astype(np.float32)
            o = 4
        qs = b[:, -16:].astype(np.int32)
        lo, hi = qs & 0xF, qs >> 4
        if t != GGMLType.Q4_1:
            qh = b[:, o:o + 4].copy().view(np.uint32).astype(np.int64)        # [nb, 1]
            j = np.arange(16)
            lo = lo | (((qh >> j) & 1) << 4)
            hi = hi | (((qh >> (j + 16)) & 1) << 4)
        q = np.concatenate([lo, hi], axis=1).astype(np.float32)
        if t == GGMLType.Q5_0:
            return ((q - 16) * d).reshape(shape)
        return (q * d + m).reshape(shape)
    if t == GGMLType.Q2_K:
        # struct { u8 scales[16]; u8 qs[64]; f16 d; f16 dmin; }: per 128-element half, four 2-bit
        # planes of 32 bytes; each 16-element run has its own 4-bit scale and 4-bit min
        b = raw.reshape(-1, 84)
        sc = b[:, 0:16].astype(np.float32)
        qs = b[:, 16:80].astype(np.int32)
        d = b[:, 80:82].copy().view(np.float16).astype(np.float32)
        dmin = b[:, 82:84].copy().view(np.float16).astype(np.float32)
        out = np.empty((b.shape[0], 256), dtype=np.float32)
        for h in range(2):
            q = qs[:, 32 * h: 32 * h + 32]
            for j in range(4):
                for half in range(2):
                    i = 8 * h + 2 * j + half
                    s = sc[:, i:i + 1]
                    v = (q[:, 16 * half: 16 * half + 16] >> (2 * j)) & 3
                    base = 128 * h + 32 * j + 16 * half
                    out[:, base: base + 16] = d * (s % 16) * v - dmin * np.floor(s / 16)
        return out.reshape(shape)
    if t == GGMLType.Q3_K:
        # struct { u8 hmask[32]; u8 qs[64]; u8 scales[12]; f16 d; }: 2 low bits in qs, the third
        # (inverted: set = no -4) in hmask, sixteen 6-bit signed scales packed in 12 bytes
        b = raw.reshape(-1, 110)
        hm = b[:, 0:32].astype(np.int32)
        qs = b[:, 32:96].astype(np.int32)
        a = b[:, 96:108].copy().view(np.uint32).astype(np.int64)                # [nb, 3]
        d = b[:, 108:110].copy().view(np.float16).astype(np.float32)
        k1, k2 = 0x03030303, 0x0F0F0F0F
        a0, a1, tmp = a[:, 0], a[:, 1], a[:, 2]
        aux = np.stack([(a0 & k2) | (((tmp >> 0) & k1) << 4), (a1 & k2) | (((tmp >> 2) & k1) << 4),
                        ((a0 >> 4) & k2) | (((tmp >> 4) & k1) << 4), ((a1 >> 4) & k2) | (((tmp >> 6) & k1) << 4)],
                       axis=1).astype(np.uint32)
        scales = aux.view(np.int8).reshape(-1, 16).astype(np.float32) - 32
        out = np.empty((b.shape[0], 256), dtype=np.float32)
        for h in range(2):
            q = qs[:, 32 * h: 32 * h + 32]
            for j in range(4):
                bit = 1 << (4 * h + j)
                for half in range(2):
                    i = 8 * h + 2 * j + half
                    sl = slice(16 * half, 16 * half + 16)
                    v = ((q[:, sl] >> (2 * j)) & 3) - np.where(hm[:, sl] & bit, 0, 4)
                    base = 128 * h + 32 * j + 16 * half
                    out[:, base: base + 16] = (d * scales[:, i:i + 1]) * v
        return out.reshape(shape)
    raise NotImplementedError(f"dequantize {GGMLType(t).name}")


def random_q4_k_blocks(rng: np.random.Generator, n_blocks: int, std: float) -> np.ndarray:
    """Random *valid* Q4_K blocks whose dequantised weights have ~zero mean and the
    requested std.  Used to synthesise multi-GB random-init models in seconds
    (quantising float weights in numpy would take many minutes)."""
    out = np.empty((n_blocks, 144), dtype=np.uint8)
    sc = rng.integers(32, 64, size=(n_blocks, 8), dtype=np.uint8)
    mn = np.clip(np.rint(sc.astype(np.float32) * 7.5 / 8.0), 0, 63).astype(np.uint8)
    d = np.full(n_blocks, std / (47.5 * 4.61), dtype=np.float32)
    out[:, 0:2] = _f16(d).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = _f16(d * 8.0).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(sc, mn)
    out[:, 16:] = rng.integers(0, 256, size=(n_blocks, 128), dtype=np.uint8)
    return out.reshape(-1)


def random_q5_k_blocks(rng: np.random.Generator, n_blocks: int, std: float) -> np.ndarray:
    """Random valid Q5_K blocks (5-bit codes uniform in 0..31), ~zero mean, the requested std."""
    out = np.empty((n_blocks, 176), dtype=np.uint8)
    sc = rng.integers(32, 64, size=(n_blocks, 8), dtype=np.uint8)
    mn = np.clip(np.rint(sc.astype(np.float32) * 15.5 / 16.0), 0, 63).astype(np.uint8)
    d = np.full(n_blocks, std / (47.5 * 9.23), dtype=np.float32)
    out[:, 0:2] = _f16(d).view(np.uint8).reshape(-1, 2)
    out[:, 2:4] = _f16(d * 16.0).view(np.uint8).reshape(-1, 2)
    out[:, 4:16] = _pack_q4k_scales(sc, mn)
    out[:, 16:] = rng.integers(0, 256, size=(n_blocks, 160), dtype=np.uint8)
    return out.reshape(-1)


def random_q6_k_blocks(rng: np.random.Generator, n_blocks: int, std: float) -> np.ndarray:
    out = np.empty((n_blocks, 210), dtype=np.uint8)
    out[:, 0:192] = rng.integers(0, 256, size=(n_blocks, 192), dtype=np.uint8)
    sc = rng.integers(64, 128, size=(n_blocks, 16), dtype=np.int16).astype(np.int8)
    out[:, 192:208] = sc.view(np.uint8)
    d = np.full(n_blocks, std / (96.0 * 18.5), dtype=np.float32)
    out[:, 208:210] = _f16(d).view(np.uint8).reshape(-1, 2)
    return out.reshape(-1)


def random_q8_0_blocks(rng: np.random.Generator, n_blocks: int, std: float) -> np.ndarray:
    out = np.empty((n_blocks, 34), dtype=np.uint8)
    out[:, 2:] = rng.integers(0, 256, size=(n_blocks, 32), dtype=np.uint8)
    d = np.full(n_blocks, std / 73.9, dtype=np.float32)
    out[:, 0:2] = _f16(d).view(np.uint8).reshape(-1, 2)
    return out.reshape(-1)


def gguf_info(path: str) -> Dict[str, Any]:
    """Summary used by `local-ai util gguf-info` (`core/cli/util.go:39-135`)."""
    with GGUFReader(path, load_tensors=False) as r:
        kv = {}
        for k, v in r.kv.items():
            if isinstance(v, list) and len(v) > 16:
                kv[k] = f"[{len(v)} items]"
            else:
                kv[k] = v
        tensors = [{"name": t.name, "shape": list(t.shape), "type": t.type_name} for t in r.tensors.values()]
        return {"version": r.version, "metadata": kv, "tensors": tensors}
