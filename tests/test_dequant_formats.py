"""Block formats beyond the engine's native ones (Q4_1, Q5_0, Q5_1, Q2_K, Q3_K): the vectorised
dequantisers in gguf.py vs element-by-element transcriptions of ggml's dequantize_row_* loops,
on random block bytes (any byte pattern is a valid block once the fp16 fields are finite)."""
import struct

import numpy as np
import pytest

from localai_amd.gguf import GGML_BLOCK, GGMLType, dequantize


def _f16(b, o):
    return float(np.frombuffer(bytes(b[o:o + 2]), np.float16)[0])


def ref_block(t, b):
    y = [0.0] * GGML_BLOCK[t][0]
    if t in (GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1):
        d = _f16(b, 0)
        o, m = 2, 0.0
        if t != GGMLType.Q5_0:
            m, o = _f16(b, 2), 4
        qh = struct.unpack("<I", bytes(b[o:o + 4]))[0] if t != GGMLType.Q4_1 else 0
        qs = b[-16:]
        for j in range(16):
            x0, x1 = qs[j] & 0x0F, qs[j] >> 4
            if t != GGMLType.Q4_1:
                x0 |= ((qh >> j) << 4) & 0x10
                x1 |= (qh >> (j + 12)) & 0x10
            if t == GGMLType.Q5_0:
                y[j], y[j + 16] = (x0 - 16) * d, (x1 - 16) * d
            else:
                y[j], y[j + 16] = x0 * d + m, x1 * d + m
        return y
    if t == GGMLType.Q2_K:
        scales, q = b[0:16], b[16:80]
        d, mn = _f16(b, 80), _f16(b, 82)
        i = is_ = 0
        for n in range(0, 256, 128):
            shift = 0
            for _ in range(4):
                sc = scales[is_]; is_ += 1
                dl, ml = d * (sc & 0xF), mn * (sc >> 4)
                for ll in range(16):
                    y[i] = dl * ((q[n // 4 + ll] >> shift) & 3) - ml; i += 1
                sc = scales[is_]; is_ += 1
                dl, ml = d * (sc & 0xF), mn * (sc >> 4)
                for ll in range(16):
                    y[i] = dl * ((q[n // 4 + ll + 16] >> shift) & 3) - ml; i += 1
                shift += 2
        return y
    if t == GGMLType.Q3_K:
        hm, q, sb, d = b[0:32], b[32:96], b[96:108], _f16(b, 108)
        aux = list(struct.unpack("<3I", bytes(sb))) + [0]
        k1, k2 = 0x03030303, 0x0F0F0F0F
        tmp = aux[2]
        aux[2] = ((aux[0] >> 4) & k2) | (((tmp >> 4) & k1) << 4)
        aux[3] = ((aux[1] >> 4) & k2) | (((tmp >> 6) & k1) << 4)
        aux[0] = (aux[0] & k2) | (((tmp >> 0) & k1) << 4)
        aux[1] = (aux[1] & k2) | (((tmp >> 2) & k1) << 4)
        scales = struct.unpack("<16b", struct.pack("<4I", *aux))
        i = is_ = 0
        m = 1
        for n in range(0, 256, 128):
            shift = 0
            for _ in range(4):
                dl = d * (scales[is_] - 32); is_ += 1
                for ll in range(16):
                    y[i] = dl * (((q[n // 4 + ll] >> shift) & 3) - (0 if hm[ll] & m else 4)); i += 1
                dl = d * (scales[is_] - 32); is_ += 1
                for ll in range(16):
                    y[i] = dl * (((q[n // 4 + ll + 16] >> shift) & 3) - (0 if hm[ll + 16] & m else 4)); i += 1
                shift += 2
                m <<= 1
        return y
    raise ValueError(t)


@pytest.mark.parametrize("t", [GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1, GGMLType.Q2_K, GGMLType.Q3_K])
def test_dequant_matches_ggml_loops(t):
    rng = np.random.default_rng(int(t))
    bs, nbytes = GGML_BLOCK[t]
    nblk = 6
    raw = rng.integers(0, 256, size=(nblk, nbytes), dtype=np.uint8)
    # finite, modest fp16 scale fields
    f16_fields = {GGMLType.Q4_1: (0, 2), GGMLType.Q5_0: (0,), GGMLType.Q5_1: (0, 2), GGMLType.Q2_K: (80, 82),
                  GGMLType.Q3_K: (108,)}[t]
    for o in f16_fields:
        raw[:, o:o + 2] = np.frombuffer(rng.uniform(-0.5, 0.5, nblk).astype(np.float16).tobytes(),
                                        np.uint8).reshape(nblk, 2)
    got = dequantize(raw.reshape(-1), t, (nblk * bs,))
    want = np.concatenate([np.asarray(ref_block(t, [int(x) for x in raw[i]]), np.float32) for i in range(nblk)])
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-6)


def test_qweight_tile_ok_is_a_shape_predicate():
    """QWeight.tile_ok is a property (a bound method would be truthy for every weight and send a
    K = 588 CLIP patch embedding into the tile GEMM, which needs K % 256 == 0)."""
    import torch

    from localai_amd import ops
    a = ops.QWeight.from_float(torch.randn(64, 588))
    assert isinstance(type(a).tile_ok, property) and a.tile_ok is False
