"""Semantics of gfx950's scaled fp8 / fp6 -> bf16 conversions (v_cvt_scalef32_pk_bf16_fp8,
v_cvt_scalef32_pk32_bf16_fp6): is the f32 scale a full multiplier or exponent-only, and what is
the fp6 bit packing?  Built by hand: hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/cvt_probe.so"""
import ctypes
import os

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "cvt_probe.so"))
L.run8.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
L.run6.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_int]


def e4m3(b):
    s = -1.0 if b & 0x80 else 1.0
    e = (b >> 3) & 15
    m = b & 7
    if e == 0:
        return s * m / 8 * 2.0 ** -6
    return s * (1 + m / 8) * 2.0 ** (e - 7)


def e2m3(b):
    s = -1.0 if b & 0x20 else 1.0
    e = (b >> 3) & 3
    m = b & 7
    if e == 0:
        return s * m / 8
    return s * (1 + m / 8) * 2.0 ** (e - 1)


dev = torch.device("cuda:0")
for scale in (1.0, 0.3173, 3.0e-3, 0.75):
    bytes_ = np.arange(256, dtype=np.uint8)
    words = bytes_.view(np.uint32) if False else np.frombuffer(bytes_.tobytes(), dtype=np.uint32).copy()
    n = len(words)
    src = torch.from_numpy(words.view(np.int32)).to(dev)
    o2 = torch.empty(n * 2, dtype=torch.bfloat16, device=dev)
    o2h = torch.empty(n * 2, dtype=torch.bfloat16, device=dev)
    assert L.run8(src.data_ptr(), scale, o2.data_ptr(), o2h.data_ptr(), n) == 0
    lo = o2.float().cpu().numpy().reshape(n, 2)
    hi = o2h.float().cpu().numpy().reshape(n, 2)
    exp_lo = np.array([[e4m3(b[0]) * scale, e4m3(b[1]) * scale] for b in bytes_.reshape(n, 4)])
    exp_hi = np.array([[e4m3(b[2]) * scale, e4m3(b[3]) * scale] for b in bytes_.reshape(n, 4)])
    ok = np.isfinite(exp_lo)
    rel_lo = np.nanmax(np.abs(lo - exp_lo)[ok] / np.maximum(np.abs(exp_lo[ok]), 1e-30))
    rel_hi = np.nanmax(np.abs(hi - exp_hi)[ok] / np.maximum(np.abs(exp_hi[ok]), 1e-30))
    print(f"fp8 scale={scale}: max rel err lo {rel_lo:.3e} hi {rel_hi:.3e}; sample {lo[14]} vs {exp_lo[14]}", flush=True)
    # fp6: 32 values per lane, value i = bits [6i, 6i+6) of a 192-bit little-endian word
    vals = np.arange(64, dtype=np.uint64) % 64
    nl = 2
    packed = []
    codes = []
    for lane in range(nl):
        cs = [(lane * 32 + i) % 64 for i in range(32)]
        codes.append(cs)
        big = 0
        for i, c in enumerate(cs):
            big |= int(c) << (6 * i)
        packed += [(big >> (32 * j)) & 0xFFFFFFFF for j in range(6)]
    src6 = torch.tensor(np.array(packed, dtype=np.uint32).view(np.int32), device=dev)
    o32 = torch.empty(nl * 32, dtype=torch.bfloat16, device=dev)
    assert L.run6(src6.data_ptr(), scale, o32.data_ptr(), nl) == 0
    got = o32.float().cpu().numpy().reshape(nl, 32)
    exp = np.array([[e2m3(c) * scale for c in cs] for cs in codes])
    rel = np.max(np.abs(got - exp) / np.maximum(np.abs(exp), 1e-30))
    print(f"fp6 scale={scale}: max rel err {rel:.3e}; lane0 first 8 got {got[0,:8]} exp {exp[0,:8]}", flush=True)
