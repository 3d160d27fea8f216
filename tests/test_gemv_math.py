"""CPU checks of the int8-dot decode GEMV (ops/csrc/gemv_dp4.hip) arithmetic.

The kernel's per-lane integer math is emulated here in NumPy exactly as the HIP code does it
(8 lanes per 256-weight super-block, q8_1-style activation blocks of 32, v_dot4_i32_i8 dots,
unpacked Q4_K scale planes), and compared against the fp32 dequantised GEMV.  A wrong lane ->
weight/activation mapping shows up as an O(1) error; the q8 activation rounding stays < 2%.
"""
import numpy as np
import pytest
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, dequantize, quantize


def _u32(a):
    return np.frombuffer(np.ascontiguousarray(a).tobytes(), np.uint32).astype(np.int64)


def _dot4(a, b, c=0):
    A = np.frombuffer(np.uint32(a & 0xFFFFFFFF).tobytes(), np.int8).astype(np.int64)
    B = np.frombuffer(np.uint32(b & 0xFFFFFFFF).tobytes(), np.int8).astype(np.int64)
    return c + int((A * B).sum())


def _quant_x(x):
    """x [K] -> int8 codes, per-32 scale, per-16 code sums (the kernel's LDS image)."""
    blk = x.reshape(-1, 32)
    amax = np.abs(blk).max(1)
    inv = np.where(amax > 0, 127.0 / np.maximum(amax, 1e-30), 0.0)
    q = np.rint(blk * inv[:, None]).astype(np.int64).reshape(-1)
    return q.astype(np.int8), (amax / 127.0).astype(np.float32), q.reshape(-1, 16).sum(1)


def _emulate(raw, t, N, K, x):
    nsb = K // 256
    xq, dx, bs = _quant_x(x)
    out = np.zeros(N)
    if t == GGMLType.Q4_K:
        b = torch.from_numpy(raw).view(N, nsb, 144)
        qs = b[:, :, 16:].reshape(N, K // 2).numpy()
        scm, dd = (p.numpy() for p in ops._q4k_gemv_planes(b[:, :, :16]))
    else:
        b = raw.reshape(N, nsb, 210)
        ql, qh = b[:, :, :128].reshape(N, -1), b[:, :, 128:192].reshape(N, -1)
        sc, dp = b[:, :, 192:208].reshape(N, -1), b[:, :, 208:210].reshape(N, -1)
    for n in range(N):
        acc = 0.0
        for sb in range(nsb):
            xs = xq[sb * 256:(sb + 1) * 256]
            for lane in range(8):
                if t == GGMLType.Q4_K:
                    j, h = lane >> 1, lane & 1
                    xlo, blo = 64 * j + 16 * h, 4 * j + h
                    qa = _u32(qs[n, sb * 128 + 16 * lane: sb * 128 + 16 * lane + 16])
                    xl, xh = _u32(xs[xlo:xlo + 16]), _u32(xs[xlo + 32:xlo + 48])
                    dl = dh = 0
                    for i in range(4):
                        dl = _dot4(qa[i] & 0x0F0F0F0F, xl[i], dl)
                        dh = _dot4((qa[i] >> 4) & 0x0F0F0F0F, xh[i], dh)
                    s = int(_u32(scm[n, sb * 16 + 4 * j: sb * 16 + 4 * j + 4])[0])
                    dxl, dxh = dx[sb * 8 + 2 * j], dx[sb * 8 + 2 * j + 1]
                    bl, bh = bs[sb * 16 + blo] * dxl, bs[sb * 16 + blo + 2] * dxh
                    fs = dl * (s & 255) * dxl + dh * ((s >> 16) & 255) * dxh
                    fm = ((s >> 8) & 255) * bl + (s >> 24) * bh
                    d, dmin = np.frombuffer(dd[n, sb * 4:sb * 4 + 4].tobytes(), np.float16).astype(np.float64)
                    acc += d * fs - dmin * fm
                else:
                    hh, u = lane >> 2, lane & 3
                    s2 = u >> 1
                    xlo = 128 * hh + 32 * s2 + 16 * (u & 1)
                    blo, shl, shr, scb = xlo >> 4, 4 - 2 * s2, 2 * s2, 8 * (2 * s2 + (u & 1))
                    la = _u32(ql[n, sb * 128 + 64 * hh + 16 * u: sb * 128 + 64 * hh + 16 * u + 16])
                    ha = _u32(qh[n, sb * 64 + 32 * hh + 16 * (u & 1): sb * 64 + 32 * hh + 16 * (u & 1) + 16])
                    xl, xh = _u32(xs[xlo:xlo + 16]), _u32(xs[xlo + 64:xlo + 80])
                    dl, dh = -32 * bs[sb * 16 + blo], -32 * bs[sb * 16 + blo + 4]
                    for i in range(4):
                        lo = (la[i] & 0x0F0F0F0F) | ((ha[i] << shl) & 0x30303030)
                        hi = ((la[i] >> 4) & 0x0F0F0F0F) | ((ha[i] >> shr) & 0x30303030)
                        dl, dh = _dot4(lo, xl[i], dl), _dot4(hi, xh[i], dh)
                    c = _u32(sc[n, sb * 16 + 8 * hh: sb * 16 + 8 * hh + 8])
                    sl, sh = np.int8((c[0] >> scb) & 255), np.int8((c[1] >> scb) & 255)
                    d = float(np.frombuffer(dp[n, sb * 2:sb * 2 + 2].tobytes(), np.float16)[0])
                    acc += d * (dl * int(sl) * dx[(sb * 256 + xlo) // 32] + dh * int(sh) * dx[(sb * 256 + xlo) // 32 + 2])
        out[n] = acc
    return out


@pytest.mark.parametrize("t", [GGMLType.Q4_K, GGMLType.Q6_K])
def test_dp4_lane_math_matches_dequant(t):
    rng = np.random.default_rng(3)
    N, K = 6, 512
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    raw = quantize(w, t)
    x = rng.standard_normal(K).astype(np.float32)
    ref = dequantize(raw, t, (N, K)) @ x
    got = _emulate(raw, t, N, K, x)
    assert np.abs(got - ref).max() < 2e-2 * max(1.0, np.abs(ref).max())


def test_q4k_gemv_planes_reconstruct_weights():
    """scm/dd planes + the raw nibbles reproduce ggml's Q4_K dequantisation exactly."""
    rng = np.random.default_rng(4)
    N, K = 5, 768
    raw = quantize(rng.standard_normal((N, K)).astype(np.float32), GGMLType.Q4_K)
    ref = dequantize(raw, GGMLType.Q4_K, (N, K))
    b = torch.from_numpy(raw).view(N, K // 256, 144)
    scm, dd = ops._q4k_gemv_planes(b[:, :, :16])
    qs = b[:, :, 16:].numpy().astype(np.int64)                  # [N, nsb, 128]
    sc = scm.view(N, K // 256, 8, 2).numpy().astype(np.float64)
    d = dd.view(torch.float16).view(N, K // 256, 2).numpy().astype(np.float64)
    w = np.zeros((N, K))
    for sb in range(K // 256):
        for j in range(4):
            q = qs[:, sb, 32 * j:32 * j + 32]
            for half, nib in ((0, q & 15), (1, q >> 4)):
                s = 2 * j + half
                col = sb * 256 + 64 * j + 32 * half
                w[:, col:col + 32] = d[:, sb, :1] * sc[:, sb, s, :1] * nib - d[:, sb, 1:] * sc[:, sb, s, 1:]
    assert np.allclose(w, ref, atol=1e-6)


@pytest.mark.parametrize("K,M", [(4096, 1), (14336, 1), (14336, 2), (14336, 4), (28672, 4)])
def test_gemv_splits_fit_lds(K, M):
    w = ops.QWeight(ops.FMT_Q4_K, 4096, K, (None,) * 4)
    S = ops._gemv_splits([w], K, M)
    nsb = K // 256
    mt = 1 if M == 1 else (2 if M == 2 else 4)
    assert nsb % S == 0
    kper = K // S
    assert mt * (kper + kper // 16 * 4 + kper // 32 * 4) <= 64 * 1024


def test_norm_in_prologue_mapping_and_materialize():
    """GV_NORM prologue (gemv_dp4.hip norm_quantize_x): thread tid's float4 chunk c = tid + 256 i is
    super-block w + 4 i, elements 4l..4l+3 -- the quantiser's own lane mapping -- for every split
    range; and NormIn.materialize() (the non-fused fallback) gives add_norm's x with the updated
    residual in res_out and res itself updated in place."""
    K = 4096
    for tid in range(256):
        wv, l = tid >> 6, tid & 63
        for i in range(8):
            c = tid + 256 * i
            sb, within = divmod(4 * c, 256)
            assert (sb, within) == (wv + 4 * i, 4 * l)
    g = torch.Generator().manual_seed(0)
    res = torch.randn(2, K, generator=g)
    add = ops.Partial(torch.randn(3, 2, K, generator=g))
    w = torch.rand(K, generator=g) + 0.5
    out = torch.empty_like(res)
    nin = ops.NormIn(res.clone(), add, w, 1e-5, out)
    x = nin.materialize()
    r = res + add.t.sum(0)
    ref = r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + 1e-5) * w
    assert torch.allclose(out, r, atol=1e-5) and torch.allclose(nin.res, r, atol=1e-5)
    assert torch.allclose(x.float(), ref, rtol=1e-2, atol=1e-2)
    assert not ops.norm_in_ok(res, add, w, None)  # CPU tensors: never the fused path


def test_anyres_assembly_index_matches_torch_path():
    """LLaVA-1.6 anyres assembly as ONE gather (ops.gather_rows through an index vector derived
    by running the torch assembly on row numbers, clip.py ClipVision._assemble) equals the torch
    permute / unpad / newline / cat path, for wide and tall images and without a newline row."""
    from localai_amd.models.clip import ClipVision

    class M:
        grid = 4

    for layout in [(2, 2, 300, 200), (2, 1, 200, 500), (3, 2, 640, 480)]:
        gw, gh = layout[0], layout[1]
        for nl in (torch.randn(8), None):
            m = M()
            m.newline = nl
            e = torch.randn(1 + gw * gh, 16, 8)
            ref = ClipVision._assemble_torch(m, e, layout)
            rows = torch.arange(e.shape[0] * 16, dtype=torch.float64).view(e.shape[0], 16, 1)
            m.newline = torch.full((1,), -1.0, dtype=torch.float64) if nl is not None else None
            idx = ClipVision._assemble_torch(m, rows, layout).view(-1).round().long()
            got = ops.gather_rows(e.reshape(-1, 8), idx, nl)
            assert torch.equal(ref, got), (layout, nl is None)
