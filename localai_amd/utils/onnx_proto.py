"""ONNX model files without the onnx package: a protobuf wire-format reader (and the matching
writer, for synthetic test models) for the parts of onnx.proto an inference graph uses.

Field numbers are onnx.proto's (ModelProto.graph = 7, GraphProto.node = 1 / initializer = 5 /
input = 11 / output = 12, NodeProto.input = 1 / output = 2 / op_type = 4 / attribute = 5,
AttributeProto name = 1 / f = 2 / i = 3 / s = 4 / t = 5 / g = 6 / floats = 7 / ints = 8 /
strings = 9 / type = 20, TensorProto dims = 1 / data_type = 2 / float_data = 4 / int32_data = 5 /
int64_data = 7 / name = 8 / raw_data = 9 / double_data = 10).  Nothing in a file is executed:
tensors are decoded into numpy arrays from their declared dtype only.

Used by the piper TTS backend (models/piper.py), whose voices ship as `.onnx` graphs
(reference: backend/go/tts/piper.go:20-24 loads `<voice>.onnx` through onnxruntime).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional, Tuple

import numpy as np

# TensorProto.DataType -> numpy dtype
DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64,
          9: np.bool_, 10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}
NP_TO_ONNX = {np.dtype(v): k for k, v in DTYPES.items()}


def _varint(b: memoryview, p: int) -> Tuple[int, int]:
    r = s = 0
    while True:
        c = b[p]
        p += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, p
        s += 7


def _fields(b: memoryview) -> Iterator[Tuple[int, int, Any]]:
    """(field number, wire type, value): varint -> int, 64/32-bit -> raw bytes, bytes -> memoryview."""
    p, n = 0, len(b)
    while p < n:
        key, p = _varint(b, p)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, p = _varint(b, p)
        elif wt == 1:
            v, p = b[p:p + 8], p + 8
        elif wt == 2:
            ln, p = _varint(b, p)
            v, p = b[p:p + ln], p + ln
        elif wt == 5:
            v, p = b[p:p + 4], p + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _signed(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


def _packed_ints(wt: int, v) -> List[int]:
    if wt == 0:
        return [_signed(v)]
    out, p = [], 0
    while p < len(v):
        x, p = _varint(v, p)
        out.append(_signed(x))
    return out


def _packed_floats(wt: int, v) -> List[float]:
    if wt == 5:
        return [struct.unpack("<f", v)[0]]
    return list(np.frombuffer(v, dtype="<f4"))


@dataclass
class Node:
    op: str
    inputs: List[str]
    outputs: List[str]
    attrs: Dict[str, Any] = field(default_factory=dict)
    name: str = ""
    domain: str = ""


@dataclass
class Graph:
    nodes: List[Node]
    initializers: Dict[str, np.ndarray]
    inputs: List[str]
    outputs: List[str]
    name: str = ""


@dataclass
class Model:
    graph: Graph
    opset: int
    producer: str = ""


def _tensor(b: memoryview) -> Tuple[str, np.ndarray]:
    dims: List[int] = []
    dt, name, raw = 1, "", None
    fl: List[float] = []
    i32: List[int] = []
    i64: List[int] = []
    dbl: List[float] = []
    for f, wt, v in _fields(b):
        if f == 1:
            dims += _packed_ints(wt, v)
        elif f == 2:
            dt = v
        elif f == 4:
            fl += _packed_floats(wt, v)
        elif f == 5:
            i32 += _packed_ints(wt, v)
        elif f == 7:
            i64 += _packed_ints(wt, v)
        elif f == 8:
            name = bytes(v).decode()
        elif f == 9:
            raw = bytes(v)
        elif f == 10:
            dbl += list(np.frombuffer(v, dtype="<f8")) if wt == 2 else [struct.unpack("<d", v)[0]]
        elif f == 14 and v == 1:
            raise ValueError(f"tensor {name!r}: external data is not supported")
    if dt not in DTYPES:
        raise ValueError(f"tensor {name!r}: unsupported data type {dt}")
    npdt = np.dtype(DTYPES[dt]).newbyteorder("<")
    if raw is not None:
        a = np.frombuffer(raw, dtype=npdt).copy()
    elif dt == 1:
        a = np.asarray(fl, dtype=np.float32)
    elif dt == 11:
        a = np.asarray(dbl, dtype=np.float64)
    elif dt in (7,):
        a = np.asarray(i64, dtype=np.int64)
    elif dt == 10:  # float16 bits travel in int32_data
        a = np.asarray(i32, dtype=np.uint16).view(np.float16)
    else:
        a = np.asarray(i32 if i32 else i64, dtype=DTYPES[dt])
    return name, a.reshape(dims) if dims else a.reshape(())


def _attr(b: memoryview) -> Tuple[str, Any]:
    name, typ = "", 0
    vals: Dict[int, Any] = {}
    ints: List[int] = []
    floats: List[float] = []
    strings: List[bytes] = []
    for f, wt, v in _fields(b):
        if f == 1:
            name = bytes(v).decode()
        elif f == 2:
            vals[2] = struct.unpack("<f", v)[0]
        elif f == 3:
            vals[3] = _signed(v)
        elif f == 4:
            vals[4] = bytes(v)
        elif f == 5:
            vals[5] = _tensor(v)[1]
        elif f == 6:
            vals[6] = _graph(v)
        elif f == 7:
            floats += _packed_floats(wt, v)
        elif f == 8:
            ints += _packed_ints(wt, v)
        elif f == 9:
            strings.append(bytes(v))
        elif f == 20:
            typ = v
    # AttributeType: FLOAT 1, INT 2, STRING 3, TENSOR 4, GRAPH 5, FLOATS 6, INTS 7, STRINGS 8
    if typ == 6 or (not typ and floats):
        return name, floats
    if typ == 7 or (not typ and ints):
        return name, ints
    if typ == 8:
        return name, strings
    for k in (2, 3, 4, 5, 6):
        if k in vals:
            return name, vals[k]
    return name, ints if typ == 7 else floats if typ == 6 else None


def _node(b: memoryview) -> Node:
    n = Node("", [], [])
    for f, wt, v in _fields(b):
        if f == 1:
            n.inputs.append(bytes(v).decode())
        elif f == 2:
            n.outputs.append(bytes(v).decode())
        elif f == 3:
            n.name = bytes(v).decode()
        elif f == 4:
            n.op = bytes(v).decode()
        elif f == 5:
            k, a = _attr(v)
            n.attrs[k] = a
        elif f == 7:
            n.domain = bytes(v).decode()
    return n


def _value_name(b: memoryview) -> str:
    for f, wt, v in _fields(b):
        if f == 1:
            return bytes(v).decode()
    return ""


def _graph(b: memoryview) -> Graph:
    g = Graph([], {}, [], [])
    for f, wt, v in _fields(b):
        if f == 1:
            g.nodes.append(_node(v))
        elif f == 2:
            g.name = bytes(v).decode()
        elif f == 5:
            k, a = _tensor(v)
            g.initializers[k] = a
        elif f == 11:
            g.inputs.append(_value_name(v))
        elif f == 12:
            g.outputs.append(_value_name(v))
    g.inputs = [i for i in g.inputs if i not in g.initializers]
    return g


def load_model(path_or_bytes) -> Model:
    data = path_or_bytes
    if isinstance(path_or_bytes, str):
        with open(path_or_bytes, "rb") as f:
            data = f.read()
    b = memoryview(data)
    graph: Optional[Graph] = None
    opset, producer = 0, ""
    for f, wt, v in _fields(b):
        if f == 7:
            graph = _graph(v)
        elif f == 2:
            producer = bytes(v).decode()
        elif f == 8:
            dom, ver = "", 0
            for f2, _, v2 in _fields(v):
                if f2 == 1:
                    dom = bytes(v2).decode()
                elif f2 == 2:
                    ver = v2
            if dom in ("", "ai.onnx"):
                opset = ver
    if graph is None:
        raise ValueError("not an ONNX model (no graph)")
    return Model(graph, opset, producer)


# ----------------------------------------------------------------------------- writer
def _key(f: int, wt: int) -> bytes:
    return _enc_varint((f << 3) | wt)


def _enc_varint(x: int) -> bytes:
    if x < 0:
        x += 1 << 64
    out = bytearray()
    while True:
        c = x & 0x7F
        x >>= 7
        if x:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def _ld(f: int, payload: bytes) -> bytes:
    return _key(f, 2) + _enc_varint(len(payload)) + payload


def _s(f: int, s: str) -> bytes:
    return _ld(f, s.encode())


def encode_tensor(name: str, a: np.ndarray) -> bytes:
    a = np.array(a, copy=True, order="C")  # (np.ascontiguousarray would make a 0-d array 1-d)
    dt = NP_TO_ONNX[a.dtype]
    out = b"".join(_key(1, 0) + _enc_varint(d) for d in a.shape) + _key(2, 0) + _enc_varint(dt)
    return out + _s(8, name) + _ld(9, a.astype(a.dtype.newbyteorder("<")).tobytes())


def encode_attr(name: str, v: Any) -> bytes:
    out = _s(1, name)
    if isinstance(v, bool) or isinstance(v, (int, np.integer)):
        return out + _key(3, 0) + _enc_varint(int(v)) + _key(20, 0) + _enc_varint(2)
    if isinstance(v, float):
        return out + _key(2, 5) + struct.pack("<f", v) + _key(20, 0) + _enc_varint(1)
    if isinstance(v, (bytes, str)):
        return out + _ld(4, v.encode() if isinstance(v, str) else v) + _key(20, 0) + _enc_varint(3)
    if isinstance(v, np.ndarray):
        return out + _ld(5, encode_tensor("", v)) + _key(20, 0) + _enc_varint(4)
    v = list(v)
    if v and all(isinstance(x, (int, np.integer)) for x in v):
        return out + _ld(8, b"".join(_enc_varint(int(x)) for x in v)) + _key(20, 0) + _enc_varint(7)
    return out + _ld(7, struct.pack(f"<{len(v)}f", *v)) + _key(20, 0) + _enc_varint(6)


def encode_model(nodes: List[Node], initializers: Dict[str, np.ndarray], inputs: List[str], outputs: List[str],
                 opset: int = 15, name: str = "graph") -> bytes:
    g = b"".join(_ld(1, b"".join([*(_s(1, i) for i in n.inputs), *(_s(2, o) for o in n.outputs), _s(3, n.name),
                                  _s(4, n.op), *(_ld(5, encode_attr(k, v)) for k, v in n.attrs.items())]))
                 for n in nodes)
    g += _s(2, name)
    g += b"".join(_ld(5, encode_tensor(k, v)) for k, v in initializers.items())
    g += b"".join(_ld(11, _s(1, i)) for i in inputs) + b"".join(_ld(12, _s(1, o)) for o in outputs)
    opset_b = _ld(8, _s(1, "") + _key(2, 0) + _enc_varint(opset))
    return _key(1, 0) + _enc_varint(8) + _s(2, "localai_amd") + opset_b + _ld(7, g)
