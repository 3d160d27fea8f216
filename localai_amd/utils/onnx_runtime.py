"""A small ONNX graph executor on PyTorch (CPU or the GPU), for the exported networks the serving
stack loads as `.onnx` files -- piper's VITS voices first of all (reference:
backend/go/tts/piper.go:20-24 runs them through onnxruntime, which is not in this image).

The graph (utils/onnx_proto.py) is run node by node in file order (ONNX requires topological
order).  Float work runs on `device`; shape arithmetic (Shape / Gather / Concat / Range ... on
int64 scalars and short vectors) stays on the CPU, so the only host round trips are the ones
data-dependent shapes need anyway (NonZero, the durations of a TTS model).  Intermediates are
dropped after their last consumer.  Control flow (If / Loop / Scan) is not supported.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .onnx_proto import DTYPES, Graph, Model, Node, load_model

_TORCH_DT = {1: torch.float32, 2: torch.uint8, 3: torch.int8, 5: torch.int16, 6: torch.int32, 7: torch.int64,
             9: torch.bool, 10: torch.float16, 11: torch.float64, 16: torch.bfloat16}
_SMALL = 64  # int tensors up to this many elements count as shape arithmetic (kept on the CPU)


def _t(a: np.ndarray) -> torch.Tensor:
    if a.dtype == np.uint16:
        a = a.astype(np.int32)
    if not a.flags.c_contiguous:  # (np.ascontiguousarray would turn a 0-d array into 1-d)
        a = a.copy()
    return torch.from_numpy(a)


def _ints(x) -> List[int]:
    if isinstance(x, torch.Tensor):
        return [int(v) for v in x.reshape(-1).tolist()]
    return [int(v) for v in x]


def _is_shape_like(x: torch.Tensor) -> bool:
    return not x.is_floating_point() and x.numel() <= _SMALL


class OnnxRunner:
    def __init__(self, model, device="cpu", generator: Optional[torch.Generator] = None):
        if not isinstance(model, Model):
            model = load_model(model)
        self.model = model
        self.graph: Graph = model.graph
        self.device = torch.device(device)
        self.opset = model.opset
        self.consts: Dict[str, torch.Tensor] = {}
        for k, a in self.graph.initializers.items():
            t = _t(a)
            self.consts[k] = t if _is_shape_like(t) else t.to(self.device)
        for n in self.graph.nodes:
            if n.op not in _OPS:
                raise NotImplementedError(f"ONNX op {n.domain + '.' if n.domain else ''}{n.op} is not supported")
        # last consumer of every value (free it after that node)
        self._last: Dict[str, int] = {}
        for i, n in enumerate(self.graph.nodes):
            for v in n.inputs:
                if v:
                    self._last[v] = i
        self.generator = generator

    @property
    def input_names(self) -> List[str]:
        return list(self.graph.inputs)

    def _place(self, x: torch.Tensor) -> torch.Tensor:
        if x.device == self.device or _is_shape_like(x):
            return x
        return x.to(self.device)

    def run(self, feeds: Dict[str, object], outputs: Optional[Sequence[str]] = None) -> Dict[str, torch.Tensor]:
        env: Dict[str, torch.Tensor] = dict(self.consts)
        for k in self.graph.inputs:
            if k not in feeds:
                raise KeyError(f"missing ONNX graph input {k!r}")
            v = feeds[k]
            env[k] = self._place(v if isinstance(v, torch.Tensor) else _t(np.asarray(v)))
        want = list(outputs or self.graph.outputs)
        keep = set(want) | set(self.consts)
        for i, n in enumerate(self.graph.nodes):
            args = [env[v] if v else None for v in n.inputs]
            try:
                res = _OPS[n.op](self, n, args)
            except Exception as e:  # name the node: exported graphs are thousands of nodes long
                raise RuntimeError(f"ONNX node {i} {n.op} {n.name!r}: {e}") from e
            if not isinstance(res, (list, tuple)):
                res = (res,)
            for name, r in zip(n.outputs, res):
                if name:
                    env[name] = r
            for v in n.inputs:
                if v and self._last.get(v) == i and v not in keep:
                    env.pop(v, None)
        return {k: env[k] for k in want}


# ----------------------------------------------------------------------------- ops
def _dev(a: torch.Tensor, b: torch.Tensor):
    """Bring two operands onto one device (CPU shape tensors meet device tensors here)."""
    if a.device == b.device:
        return a, b
    if a.device.type == "cpu":
        return a.to(b.device), b
    return a, b.to(a.device)


def _bin(fn):
    def op(r, n, a):
        x, y = _dev(a[0], a[1])
        return fn(x, y)
    return op


def _div(x, y):
    x, y = _dev(x, y)
    if not x.is_floating_point() and not y.is_floating_point():
        return torch.div(x, y, rounding_mode="trunc")
    return x / y


def _variadic(fn):
    def op(r, n, a):
        out = a[0]
        for y in a[1:]:
            out, y = _dev(out, y)
            out = fn(out, y)
        return out
    return op


def _constant(r, n, a):
    at = n.attrs
    if "value" in at:
        v = _t(np.asarray(at["value"]))
    elif "value_float" in at:
        v = torch.tensor(float(at["value_float"]), dtype=torch.float32)
    elif "value_int" in at:
        v = torch.tensor(int(at["value_int"]), dtype=torch.int64)
    elif "value_floats" in at:
        v = torch.tensor(list(at["value_floats"]), dtype=torch.float32)
    elif "value_ints" in at:
        v = torch.tensor(list(at["value_ints"]), dtype=torch.int64)
    else:
        raise NotImplementedError(f"Constant attributes {list(at)}")
    return r._place(v)


def _const_of_shape(r, n, a):
    shape = _ints(a[0])
    val = n.attrs.get("value")
    if val is None:
        return torch.zeros(shape, dtype=torch.float32, device=r.device)
    v = _t(np.asarray(val)).reshape(-1)[0]
    out = torch.full(shape, v.item(), dtype=v.dtype)
    return r._place(out)


def _cast(r, n, a):
    dt = _TORCH_DT[int(n.attrs["to"])]
    return a[0].to(dt)


def _shape(r, n, a):
    s = list(a[0].shape)
    start, end = int(n.attrs.get("start", 0)), n.attrs.get("end")
    s = s[start:] if end is None else s[start:int(end)]
    return torch.tensor(s, dtype=torch.int64)


def _reshape(r, n, a):
    x, shape = a[0], _ints(a[1])
    if not int(n.attrs.get("allowzero", 0)):
        shape = [x.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return x.reshape(shape)


def _transpose(r, n, a):
    perm = n.attrs.get("perm")
    return a[0].permute(*(perm if perm is not None else reversed(range(a[0].dim()))))


def _axes(r, n, a, idx=1):
    if len(a) > idx and a[idx] is not None:
        return _ints(a[idx])
    v = n.attrs.get("axes")
    return None if v is None else [int(x) for x in v]


def _unsqueeze(r, n, a):
    x = a[0]
    axes = _axes(r, n, a)
    rank = x.dim() + len(axes)
    for ax in sorted(ax % rank for ax in axes):
        x = x.unsqueeze(ax)
    return x


def _squeeze(r, n, a):
    x = a[0]
    axes = _axes(r, n, a)
    if axes is None:
        return x.squeeze()
    for ax in sorted((ax % x.dim() for ax in axes), reverse=True):
        x = x.squeeze(ax)
    return x


def _flatten(r, n, a):
    ax = int(n.attrs.get("axis", 1)) % max(a[0].dim(), 1)
    return a[0].reshape(int(np.prod(a[0].shape[:ax])), -1)


def _expand(r, n, a):
    x, shape = a[0], _ints(a[1])
    out = list(np.broadcast_shapes(tuple(x.shape), tuple(shape)))
    return x.expand(out)


def _concat(r, n, a):
    xs = [x for x in a if x is not None]
    if any(x.device != xs[0].device for x in xs):
        xs = [x.to(r.device) for x in xs]
    return torch.cat(xs, dim=int(n.attrs["axis"]))


def _split(r, n, a):
    x = a[0]
    ax = int(n.attrs.get("axis", 0))
    sizes = _ints(a[1]) if len(a) > 1 and a[1] is not None else n.attrs.get("split")
    if sizes is None:
        k = int(n.attrs.get("num_outputs", len(n.outputs)))
        d = x.shape[ax]
        c = -(-d // k)
        sizes = [c] * (k - 1) + [d - c * (k - 1)]
    return list(torch.split(x, [int(s) for s in sizes], dim=ax))


def _slice(r, n, a):
    x = a[0]
    if len(a) > 1:
        starts, ends = _ints(a[1]), _ints(a[2])
        axes = _ints(a[3]) if len(a) > 3 and a[3] is not None else list(range(len(starts)))
        steps = _ints(a[4]) if len(a) > 4 and a[4] is not None else [1] * len(starts)
    else:  # opset < 10
        starts, ends = n.attrs["starts"], n.attrs["ends"]
        axes = n.attrs.get("axes", list(range(len(starts))))
        steps = [1] * len(starts)
    for st, en, ax, sp in zip(starts, ends, axes, steps):
        ax %= x.dim()
        d = x.shape[ax]
        if sp > 0:
            st = max(0, min(d, st + d if st < 0 else st))
            en = max(0, min(d, en + d if en < 0 else en))
            x = x.narrow(ax, st, max(0, en - st))
            if sp > 1:
                x = x.index_select(ax, torch.arange(0, x.shape[ax], sp, device=x.device))
        else:
            st = max(-1, min(d - 1, st + d if st < 0 else st))
            en = max(-1, min(d - 1, en + d if en < 0 else en)) if en >= -d else -1
            idx = torch.arange(st, en, sp, device=x.device)
            x = x.index_select(ax, idx)
    return x


def _gather(r, n, a):
    x, idx = a[0], a[1]
    ax = int(n.attrs.get("axis", 0)) % x.dim()
    idx = idx.to(x.device)
    idx = torch.where(idx < 0, idx + x.shape[ax], idx)
    out = torch.index_select(x, ax, idx.reshape(-1).long())
    return out.reshape(tuple(x.shape[:ax]) + tuple(idx.shape) + tuple(x.shape[ax + 1:]))


def _gather_elements(r, n, a):
    x, idx = a[0], a[1].to(a[0].device).long()
    ax = int(n.attrs.get("axis", 0)) % x.dim()
    idx = torch.where(idx < 0, idx + x.shape[ax], idx)
    return torch.gather(x, ax, idx)


def _gather_nd(r, n, a):
    x, idx = a[0], a[1].to(a[0].device).long()
    if int(n.attrs.get("batch_dims", 0)):
        raise NotImplementedError("GatherND batch_dims > 0")
    k = idx.shape[-1]
    dims = torch.tensor(x.shape[:k], device=x.device)
    idx = torch.where(idx < 0, idx + dims, idx)
    return x[tuple(idx.unbind(-1))]


def _scatter_nd(r, n, a):
    x, idx, upd = a[0], a[1].to(a[0].device).long(), a[2].to(a[0].device)
    if n.attrs.get("reduction", b"none") not in (b"none", "none"):
        raise NotImplementedError("ScatterND reduction")
    out = x.clone()
    k = idx.shape[-1]
    dims = torch.tensor(x.shape[:k], device=x.device)
    idx = torch.where(idx < 0, idx + dims, idx)
    out[tuple(idx.unbind(-1))] = upd.to(out.dtype)
    return out


def _scatter_elements(r, n, a):
    x, idx, upd = a[0], a[1].to(a[0].device).long(), a[2].to(a[0].device)
    ax = int(n.attrs.get("axis", 0)) % x.dim()
    idx = torch.where(idx < 0, idx + x.shape[ax], idx)
    red = n.attrs.get("reduction", b"none")
    red = red.decode() if isinstance(red, bytes) else red
    if red in ("none", None):
        return x.scatter(ax, idx, upd)
    return x.scatter_reduce(ax, idx, upd, {"add": "sum", "mul": "prod", "max": "amax", "min": "amin"}[red])


def _nonzero(r, n, a):
    return torch.nonzero(a[0]).T.contiguous()


def _where(r, n, a):
    c, x, y = a
    dev = next((t.device for t in (x, y, c) if t.device.type != "cpu"), c.device)
    return torch.where(c.to(dev), x.to(dev), y.to(dev))


def _range(r, n, a):
    st, lim, dl = (v.item() for v in a)
    out = torch.arange(st, lim, dl, dtype=a[0].dtype)
    return out if _is_shape_like(out) else r._place(out)


def _cumsum(r, n, a):
    x = a[0]
    ax = _ints(a[1])[0] % x.dim()
    rev, exc = int(n.attrs.get("reverse", 0)), int(n.attrs.get("exclusive", 0))
    if rev:
        x = x.flip(ax)
    y = torch.cumsum(x, ax)
    if exc:
        y = y - x
    return y.flip(ax) if rev else y


def _reduce(fn):
    def op(r, n, a):
        x = a[0]
        axes = _axes(r, n, a)
        keep = bool(int(n.attrs.get("keepdims", 1)))
        if not axes:
            if int(n.attrs.get("noop_with_empty_axes", 0)):
                return x
            axes = list(range(x.dim()))
        axes = [ax % x.dim() for ax in axes]
        return fn(x, axes, keep)
    return op


def _red_max(x, axes, keep):
    for ax in sorted(axes, reverse=True):
        x = x.amax(ax, keepdim=keep) if keep else x.amax(ax)
    return x


def _red_min(x, axes, keep):
    for ax in sorted(axes, reverse=True):
        x = x.amin(ax, keepdim=keep) if keep else x.amin(ax)
    return x


def _softmax(fn):
    def op(r, n, a):
        x = a[0]
        ax = int(n.attrs.get("axis", -1 if r.opset >= 13 else 1))
        if r.opset >= 13:
            return fn(x, ax)
        ax %= x.dim()  # opset < 13: coerce to 2-D at axis
        s = x.shape
        return fn(x.reshape(int(np.prod(s[:ax])), -1), 1).reshape(s)
    return op


def _pads_split(pads: List[int], k: int):
    return pads[:k], pads[k:]


def _conv(r, n, a):
    x, w = _dev(a[0], a[1])
    b = a[2].to(x.device) if len(a) > 2 and a[2] is not None else None
    k = w.dim() - 2
    strides = n.attrs.get("strides", [1] * k)
    dil = n.attrs.get("dilations", [1] * k)
    groups = int(n.attrs.get("group", 1))
    pads = list(n.attrs.get("pads", [0] * (2 * k)))
    ap = n.attrs.get("auto_pad", b"NOTSET")
    ap = ap.decode() if isinstance(ap, bytes) else ap
    if ap in ("SAME_UPPER", "SAME_LOWER"):
        pads = [0] * (2 * k)
        for i in range(k):
            d_in = x.shape[2 + i]
            eff = (w.shape[2 + i] - 1) * dil[i] + 1
            out = -(-d_in // strides[i])
            tot = max(0, (out - 1) * strides[i] + eff - d_in)
            lo = tot // 2 if ap == "SAME_UPPER" else tot - tot // 2
            pads[i], pads[k + i] = lo, tot - lo
    beg, end = _pads_split(pads, k)
    if beg != end:
        fp = []
        for i in reversed(range(k)):
            fp += [beg[i], end[i]]
        x = F.pad(x, fp)
        beg = [0] * k
    fn = {1: F.conv1d, 2: F.conv2d, 3: F.conv3d}[k]
    return fn(x, w, b, stride=strides, padding=beg, dilation=dil, groups=groups)


def _conv_transpose(r, n, a):
    x, w = _dev(a[0], a[1])
    b = a[2].to(x.device) if len(a) > 2 and a[2] is not None else None
    k = w.dim() - 2
    strides = n.attrs.get("strides", [1] * k)
    dil = n.attrs.get("dilations", [1] * k)
    groups = int(n.attrs.get("group", 1))
    pads = list(n.attrs.get("pads", [0] * (2 * k)))
    opad = list(n.attrs.get("output_padding", [0] * k))
    if n.attrs.get("output_shape") is not None:
        raise NotImplementedError("ConvTranspose output_shape")
    beg, end = _pads_split(pads, k)
    fn = {1: F.conv_transpose1d, 2: F.conv_transpose2d, 3: F.conv_transpose3d}[k]
    if beg == end:
        return fn(x, w, b, stride=strides, padding=beg, output_padding=opad, groups=groups, dilation=dil)
    y = fn(x, w, b, stride=strides, padding=0, output_padding=opad, groups=groups, dilation=dil)
    for i in range(k):
        y = y.narrow(2 + i, beg[i], y.shape[2 + i] - beg[i] - end[i])
    return y


def _pad(r, n, a):
    x = a[0]
    if len(a) > 1 and a[1] is not None:
        pads = _ints(a[1])
        val = a[2].item() if len(a) > 2 and a[2] is not None and a[2].numel() else 0.0
        axes = _ints(a[3]) if len(a) > 3 and a[3] is not None else list(range(x.dim()))
    else:
        pads, val = list(n.attrs["pads"]), float(n.attrs.get("value", 0.0))
        axes = list(range(x.dim()))
    mode = n.attrs.get("mode", b"constant")
    mode = mode.decode() if isinstance(mode, bytes) else mode
    k = len(axes)
    full_b, full_e = [0] * x.dim(), [0] * x.dim()
    for i, ax in enumerate(axes):
        full_b[ax % x.dim()], full_e[ax % x.dim()] = pads[i], pads[k + i]
    # F.pad wants (last dim begin, end, second-to-last ...), trimmed to the padded dims
    last = max([i for i in range(x.dim()) if full_b[i] or full_e[i]], default=-1)
    if last < 0:
        return x
    first = min(i for i in range(x.dim()) if full_b[i] or full_e[i])
    fp = []
    for i in reversed(range(first, x.dim())):
        fp += [full_b[i], full_e[i]]
    if mode == "constant":
        return F.pad(x, fp, value=val)
    tmode = {"reflect": "reflect", "edge": "replicate"}[mode]
    # torch's reflect / replicate pad only the trailing 1-3 dims of a batched input
    return F.pad(x, fp, mode=tmode)


def _matmul(r, n, a):
    x, y = _dev(a[0], a[1])
    return torch.matmul(x, y)


def _gemm(r, n, a):
    A, B = _dev(a[0], a[1])
    if int(n.attrs.get("transA", 0)):
        A = A.T
    if int(n.attrs.get("transB", 0)):
        B = B.T
    y = float(n.attrs.get("alpha", 1.0)) * (A @ B)
    if len(a) > 2 and a[2] is not None:
        y = y + float(n.attrs.get("beta", 1.0)) * a[2].to(y.device)
    return y


def _clip(r, n, a):
    x = a[0]
    lo = a[1].item() if len(a) > 1 and a[1] is not None else n.attrs.get("min")
    hi = a[2].item() if len(a) > 2 and a[2] is not None else n.attrs.get("max")
    return torch.clamp(x, min=lo, max=hi)


def _leaky(r, n, a):
    return F.leaky_relu(a[0], float(n.attrs.get("alpha", 0.01)))


def _random_normal_like(r, n, a):
    x = a[0]
    dt = _TORCH_DT[int(n.attrs["dtype"])] if "dtype" in n.attrs else x.dtype
    mean, scale = float(n.attrs.get("mean", 0.0)), float(n.attrs.get("scale", 1.0))
    z = torch.randn(x.shape, dtype=torch.float32, generator=r.generator)  # CPU generator: same draw everywhere
    return (z * scale + mean).to(device=x.device, dtype=dt)


def _random_normal(r, n, a):
    shape = [int(s) for s in n.attrs["shape"]]
    dt = _TORCH_DT[int(n.attrs.get("dtype", 1))]
    z = torch.randn(shape, generator=r.generator)
    return (z * float(n.attrs.get("scale", 1.0)) + float(n.attrs.get("mean", 0.0))).to(device=r.device, dtype=dt)


def _random_uniform_like(r, n, a):
    x = a[0]
    lo, hi = float(n.attrs.get("low", 0.0)), float(n.attrs.get("high", 1.0))
    z = torch.rand(x.shape, generator=r.generator)
    return (z * (hi - lo) + lo).to(device=x.device, dtype=x.dtype)


def _layer_norm(r, n, a):
    x, w = _dev(a[0], a[1])
    b = a[2].to(x.device) if len(a) > 2 and a[2] is not None else None
    ax = int(n.attrs.get("axis", -1)) % x.dim()
    return F.layer_norm(x, x.shape[ax:], w, b, float(n.attrs.get("epsilon", 1e-5)))


def _instance_norm(r, n, a):
    x, w = _dev(a[0], a[1])
    return F.instance_norm(x, weight=w, bias=a[2].to(x.device), eps=float(n.attrs.get("epsilon", 1e-5)))


def _tile(r, n, a):
    return a[0].repeat(*_ints(a[1]))


def _argmax(fn):
    def op(r, n, a):
        ax = int(n.attrs.get("axis", 0))
        y = fn(a[0], dim=ax, keepdim=bool(int(n.attrs.get("keepdims", 1))))
        return y
    return op


def _mod(r, n, a):
    x, y = _dev(a[0], a[1])
    return torch.fmod(x, y) if int(n.attrs.get("fmod", 0)) else torch.remainder(x, y)


def _einsum(r, n, a):
    eq = n.attrs["equation"]
    eq = eq.decode() if isinstance(eq, bytes) else eq
    xs = [x.to(r.device) for x in a]
    return torch.einsum(eq, *xs)


def _size(r, n, a):
    return torch.tensor(a[0].numel(), dtype=torch.int64)


def _u(fn):
    return lambda r, n, a: fn(a[0])


_OPS: Dict[str, Callable] = {
    "Identity": lambda r, n, a: a[0], "Dropout": lambda r, n, a: a[0],
    "Constant": _constant, "ConstantOfShape": _const_of_shape, "Cast": _cast,
    "CastLike": lambda r, n, a: a[0].to(a[1].dtype),
    "Shape": _shape, "Size": _size, "Reshape": _reshape, "Transpose": _transpose, "Unsqueeze": _unsqueeze,
    "Squeeze": _squeeze, "Flatten": _flatten, "Expand": _expand, "Concat": _concat, "Split": _split,
    "Slice": _slice, "Gather": _gather, "GatherElements": _gather_elements, "GatherND": _gather_nd,
    "ScatterND": _scatter_nd, "ScatterElements": _scatter_elements, "NonZero": _nonzero, "Where": _where,
    "Range": _range, "CumSum": _cumsum, "Tile": _tile, "Pad": _pad,
    "Add": _bin(torch.add), "Sub": _bin(torch.sub), "Mul": _bin(torch.mul), "Div": lambda r, n, a: _div(a[0], a[1]),
    "Pow": _bin(lambda x, y: torch.pow(x, y).to(x.dtype)), "Mod": _mod,
    "Equal": _bin(torch.eq), "Less": _bin(torch.lt), "LessOrEqual": _bin(torch.le), "Greater": _bin(torch.gt),
    "GreaterOrEqual": _bin(torch.ge), "And": _bin(torch.logical_and), "Or": _bin(torch.logical_or),
    "Xor": _bin(torch.logical_xor), "Not": _u(torch.logical_not),
    "Max": _variadic(torch.maximum), "Min": _variadic(torch.minimum), "Sum": _variadic(torch.add),
    "Mean": lambda r, n, a: _variadic(torch.add)(r, n, a) / len(a),
    "Neg": _u(torch.neg), "Abs": _u(torch.abs), "Sqrt": _u(torch.sqrt), "Exp": _u(torch.exp), "Log": _u(torch.log),
    "Erf": _u(torch.erf), "Tanh": _u(torch.tanh), "Sigmoid": _u(torch.sigmoid), "Relu": _u(torch.relu),
    "Softplus": _u(F.softplus), "Ceil": _u(torch.ceil), "Floor": _u(torch.floor), "Round": _u(torch.round),
    "Sign": _u(torch.sign), "Sin": _u(torch.sin), "Cos": _u(torch.cos), "Reciprocal": _u(torch.reciprocal),
    "IsNaN": _u(torch.isnan), "IsInf": _u(torch.isinf),
    "LeakyRelu": _leaky, "Clip": _clip,
    "Elu": lambda r, n, a: F.elu(a[0], float(n.attrs.get("alpha", 1.0))),
    "Gelu": lambda r, n, a: F.gelu(a[0]),
    "HardSigmoid": lambda r, n, a: torch.clamp(float(n.attrs.get("alpha", 0.2)) * a[0] + float(n.attrs.get("beta", 0.5)), 0, 1),
    "Softmax": _softmax(torch.softmax), "LogSoftmax": _softmax(torch.log_softmax),
    "ReduceMean": _reduce(lambda x, ax, k: x.mean(ax, keepdim=k)),
    "ReduceSum": _reduce(lambda x, ax, k: x.sum(ax, keepdim=k)),
    "ReduceProd": _reduce(lambda x, ax, k: _red_prod(x, ax, k)),
    "ReduceMax": _reduce(_red_max), "ReduceMin": _reduce(_red_min),
    "ReduceL2": _reduce(lambda x, ax, k: x.pow(2).sum(ax, keepdim=k).sqrt()),
    "ArgMax": _argmax(torch.argmax), "ArgMin": _argmax(torch.argmin),
    "MatMul": _matmul, "Gemm": _gemm, "Conv": _conv, "ConvTranspose": _conv_transpose, "Einsum": _einsum,
    "LayerNormalization": _layer_norm, "InstanceNormalization": _instance_norm,
    "RandomNormalLike": _random_normal_like, "RandomNormal": _random_normal,
    "RandomUniformLike": _random_uniform_like,
}


def _red_prod(x, axes, keep):
    for ax in sorted(axes, reverse=True):
        x = x.prod(ax, keepdim=keep)
    return x
