"""CLIP ViT image encoder + LLaVA projector, loaded from a llama.cpp `mmproj` GGUF (the reference
reaches this through grpc-server.cpp -> llava/clip.cpp).

Preprocessing: PIL decodes on the host; on the GPU the resize (PIL-exact BICUBIC), centre crop /
letterbox, normalisation and tiling run in two HIP launches per resized image (ops/csrc/image.hip,
K26); on the CPU the same steps run through PIL.  The ViT
runs on the device in bf16: patch embedding as one GEMM over unfolded patches (im2col), fused
QKV, SDPA attention, LayerNorm / quick-GELU, the two-layer GELU projector into the LLM's
embedding space.  LLaVA-1.5 (one 336^2 tile -> 576 embeddings) and LLaVA-1.6 "anyres"
(grid tiles + a base tile, spatial unpadding, image_newline rows) layouts are supported, and so are
SigLIP-style towers without a class token (moondream2's mmproj: 378^2 / patch 14 -> 729
embeddings, GELU, post-LayerNorm only; clip.cpp treats `v.class_embd` as optional the same way).
"""
from __future__ import annotations

import base64
import io
import math
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..gguf import GGUFReader, dequantize

DEFAULT_MEAN = (0.48145466, 0.4578275, 0.40821073)
DEFAULT_STD = (0.26862954, 0.26130258, 0.27577711)


def decode_image(data) -> "PIL.Image.Image":
    from PIL import Image
    if isinstance(data, str):
        if data.startswith("data:"):
            data = data.split(",", 1)[1]
        data = base64.b64decode(data)
    return Image.open(io.BytesIO(data)).convert("RGB")


class ClipVision:
    def __init__(self, path: str, device: torch.device, dtype=torch.bfloat16):
        r = GGUFReader(path)
        kv = r.kv
        self.device, self.dtype = device, dtype
        self.image_size = int(kv.get("clip.vision.image_size", 336))
        self.patch = int(kv.get("clip.vision.patch_size", 14))
        self.dim = int(kv.get("clip.vision.embedding_length", 1024))
        self.heads = int(kv.get("clip.vision.attention.head_count", 16))
        self.eps = float(kv.get("clip.vision.attention.layer_norm_epsilon", 1e-5))
        self.n_layer = int(kv.get("clip.vision.block_count", 23))
        self.mean = tuple(float(x) for x in kv.get("clip.vision.image_mean", DEFAULT_MEAN))
        self.std = tuple(float(x) for x in kv.get("clip.vision.image_std", DEFAULT_STD))
        self.use_gelu = bool(kv.get("clip.use_gelu", False))
        self.merge = str(kv.get("clip.vision.mm_patch_merge_type", "flat"))
        pins = kv.get("clip.vision.image_grid_pinpoints", None)
        self.pinpoints = [(int(pins[i]), int(pins[i + 1])) for i in range(0, len(pins), 2)] if pins else []
        T = r.tensors

        def t(name, required=True):
            if name not in T:
                if required:
                    raise KeyError(f"mmproj: missing tensor {name}")
                return None
            x = T[name]
            a = dequantize(x.data, x.ggml_type, x.shape).reshape(x.shape)
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(device)

        D = self.dim
        pe = t("v.patch_embd.weight")                       # [D, 3, p, p]
        self.patch_w = pe.reshape(D, -1).to(dtype)          # im2col GEMM weight [D, 3*p*p]
        self.patch_b = t("v.patch_embd.bias", False)
        self.cls = t("v.class_embd", False)  # SigLIP towers (moondream2) have no class token
        self.pos = t("v.position_embd.weight")
        self.pre_ln = (t("v.pre_ln.weight", False), t("v.pre_ln.bias", False))
        self.post_ln = (t("v.post_ln.weight", False), t("v.post_ln.bias", False))
        self.layers = []
        for i in range(self.n_layer):
            b = f"v.blk.{i}."
            qkv_w = torch.cat([t(b + "attn_q.weight"), t(b + "attn_k.weight"), t(b + "attn_v.weight")], 0)
            qkv_b = torch.cat([t(b + "attn_q.bias"), t(b + "attn_k.bias"), t(b + "attn_v.bias")], 0)
            f1, f2 = t(b + "ffn_down.weight"), t(b + "ffn_up.weight")  # llama.cpp naming: down = fc1
            f1b, f2b = t(b + "ffn_down.bias"), t(b + "ffn_up.bias")
            if f1.shape[1] != D:  # other converters name them the natural way round
                f1, f2, f1b, f2b = f2, f1, f2b, f1b
            self.layers.append(dict(
                ln1=(t(b + "ln1.weight"), t(b + "ln1.bias")), ln2=(t(b + "ln2.weight"), t(b + "ln2.bias")),
                qkv_w=qkv_w.to(dtype), qkv_b=qkv_b, o_w=t(b + "attn_out.weight").to(dtype), o_b=t(b + "attn_out.bias"),
                f1_w=f1.to(dtype), f1_b=f1b, f2_w=f2.to(dtype), f2_b=f2b))
        self.mm0 = (t("mm.0.weight").to(dtype), t("mm.0.bias"))
        self.mm2 = (t("mm.2.weight").to(dtype), t("mm.2.bias"))
        self.out_dim = self.mm2[0].shape[0]
        self.newline = t("model.image_newline", False)
        self.grid = self.image_size // self.patch
        self.n_patches = self.grid * self.grid
        # GPU: the tower's projections through ops.linear (bf16 weights: the tile GEMM at small
        # M, the library GEMM on the weight in place at large M), residual + LayerNorm fused in
        # add_norm, activations in the act kernel (SURVEY K19 / K20 / K21 on the native ops)
        self.native = device.type == "cuda" and os.environ.get("LOCALAI_AMD_CLIP_NATIVE", "1") == "1"
        if self.native:
            from .. import ops
            qw = ops.QWeight.from_float
            self.q_patch = qw(self.patch_w)
            for ly in self.layers:
                for k in ("qkv_w", "o_w", "f1_w", "f2_w"):
                    ly["q_" + k] = qw(ly[k])
            self.q_mm0, self.q_mm2 = qw(self.mm0[0]), qw(self.mm2[0])

    # ------------------------------------------------------------------ preprocessing
    def _norm(self, img) -> torch.Tensor:
        a = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        m = torch.tensor(self.mean).view(3, 1, 1)
        s = torch.tensor(self.std).view(3, 1, 1)
        return (a - m) / s

    def _resize_square(self, img):
        """CLIP: shortest side -> image_size (bicubic), center crop."""
        from PIL import Image
        S = self.image_size
        w, h = img.size
        sc = S / min(w, h)
        img = img.resize((max(S, round(w * sc)), max(S, round(h * sc))), Image.BICUBIC)
        w, h = img.size
        l, tp = (w - S) // 2, (h - S) // 2
        return img.crop((l, tp, l + S, tp + S))

    def _best_resolution(self, w: int, h: int) -> Tuple[int, int]:
        best, best_eff, best_waste = None, -1, float("inf")
        for pw, ph in self.pinpoints:
            sc = min(pw / w, ph / h)
            dw, dh = int(w * sc), int(h * sc)
            eff = min(dw * dh, w * h)
            waste = pw * ph - eff
            if eff > best_eff or (eff == best_eff and waste < best_waste):
                best, best_eff, best_waste = (pw, ph), eff, waste
        return best

    def preprocess(self, data) -> Tuple[torch.Tensor, Optional[Tuple[int, int, int, int]]]:
        """-> (tiles [n, 3, S, S], anyres layout (grid_w, grid_h, orig_w, orig_h) or None).  On the
        GPU the resize / crop / letterbox / normalise / tiling run in the image kernels
        (ops.image_tiles, PIL-exact bicubic); LOCALAI_AMD_CLIP_HOST_PREPROC=1 keeps the PIL path."""
        img = decode_image(data)
        if self.device.type == "cuda" and os.environ.get("LOCALAI_AMD_CLIP_HOST_PREPROC", "0") != "1":
            return self._preprocess_device(img)
        return self._preprocess_host(img)

    def _placements(self, w: int, h: int):
        """The PIL path's geometry as kernel placements: (n_tiles, placements, layout)."""
        S = self.image_size
        if not self.pinpoints or self.merge == "flat":
            sc = S / min(w, h)
            rw, rh = max(S, round(w * sc)), max(S, round(h * sc))
            return 1, [dict(ow=rw, oh=rh, cw=S, ch=S, ox=-((rw - S) // 2), oy=-((rh - S) // 2), t0=0)], None
        bw, bh = self._best_resolution(w, h)
        sc = min(bw / w, bh / h)
        nw, nh = max(1, int(w * sc)), max(1, int(h * sc))
        fill = tuple(int(255 * m) for m in self.mean)
        pls = [dict(ow=S, oh=S, cw=S, ch=S, t0=0),  # base image first
               dict(ow=nw, oh=nh, cw=bw, ch=bh, ox=(bw - nw) // 2, oy=(bh - nh) // 2, t0=1, fill=fill)]
        return 1 + (bw // S) * (bh // S), pls, (bw // S, bh // S, w, h)

    def _preprocess_device(self, img):
        from .. import ops
        w, h = img.size
        n, pls, layout = self._placements(w, h)
        u8 = torch.from_numpy(np.ascontiguousarray(np.asarray(img, dtype=np.uint8))).to(self.device)
        out = torch.empty(n, 3, self.image_size, self.image_size, dtype=torch.float32, device=self.device)
        return ops.image_tiles(u8, pls, out, self.mean, self.std), layout

    def _preprocess_host(self, img) -> Tuple[torch.Tensor, Optional[Tuple[int, int, int, int]]]:
        if not self.pinpoints or self.merge == "flat":
            return self._norm(self._resize_square(img)).unsqueeze(0), None
        from PIL import Image
        w, h = img.size
        bw, bh = self._best_resolution(w, h)
        sc = min(bw / w, bh / h)
        nw, nh = max(1, int(w * sc)), max(1, int(h * sc))
        canvas = Image.new("RGB", (bw, bh), tuple(int(255 * m) for m in self.mean))
        canvas.paste(img.resize((nw, nh), Image.BICUBIC), ((bw - nw) // 2, (bh - nh) // 2))
        S = self.image_size
        tiles = [self._norm(img.resize((S, S), Image.BICUBIC))]  # base image first
        for y in range(0, bh, S):
            for x in range(0, bw, S):
                tiles.append(self._norm(canvas.crop((x, y, x + S, y + S))))
        return torch.stack(tiles), (bw // S, bh // S, w, h)

    # ------------------------------------------------------------------ encoder
    @torch.no_grad()
    def encode_tiles(self, pix: torch.Tensor) -> torch.Tensor:
        """pixels [n, 3, S, S] -> projected patch embeddings [n, n_patches, out_dim] (f32)."""
        if self.native:
            return self._encode_native(pix)
        n = pix.shape[0]
        D, P, H = self.dim, self.patch, self.heads
        x = pix.to(self.device, torch.float32)
        cols = F.unfold(x, kernel_size=P, stride=P).transpose(1, 2)           # [n, np, 3*P*P]
        h = (cols.to(self.dtype) @ self.patch_w.t()).float()                  # im2col patch GEMM
        if self.patch_b is not None:
            h = h + self.patch_b
        if self.cls is not None:
            h = torch.cat([self.cls.view(1, 1, D).expand(n, 1, D), h], 1)
        h = h + self.pos[: h.shape[1]]
        if self.pre_ln[0] is not None:
            h = F.layer_norm(h, (D,), self.pre_ln[0], self.pre_ln[1], self.eps)
        L = h.shape[1]
        for ly in self.layers:
            res = h
            a = F.layer_norm(h, (D,), ly["ln1"][0], ly["ln1"][1], self.eps)
            qkv = (a.to(self.dtype) @ ly["qkv_w"].t()).float() + ly["qkv_b"]
            q, k, v = qkv.view(n, L, 3, H, D // H).permute(2, 0, 3, 1, 4).to(self.dtype)
            o = F.scaled_dot_product_attention(q, k, v)                        # non-causal
            o = o.transpose(1, 2).reshape(n, L, D)
            h = res + (o @ ly["o_w"].t()).float() + ly["o_b"]
            res = h
            a = F.layer_norm(h, (D,), ly["ln2"][0], ly["ln2"][1], self.eps)
            f = (a.to(self.dtype) @ ly["f1_w"].t()).float() + ly["f1_b"]
            f = F.gelu(f) if self.use_gelu else f * torch.sigmoid(1.702 * f)
            h = res + (f.to(self.dtype) @ ly["f2_w"].t()).float() + ly["f2_b"]
        if self.post_ln[0] is not None:
            h = F.layer_norm(h, (D,), self.post_ln[0], self.post_ln[1], self.eps)
        if self.cls is not None:
            h = h[:, 1:]                                                       # drop CLS
        y = (h.to(self.dtype) @ self.mm0[0].t()).float() + self.mm0[1]
        y = F.gelu(y)
        y = (y.to(self.dtype) @ self.mm2[0].t()).float() + self.mm2[1]
        return y

    def _encode_native(self, pix: torch.Tensor) -> torch.Tensor:
        """encode_tiles on the native ops: im2col + GEMM patch embedding, fused residual +
        LayerNorm (add_norm mode 1), GELU / quick-GELU in the act kernel (llama.cpp's clip uses
        the tanh GELU too), non-causal attention on the MFMA flash-attention kernel read straight
        from the fused q|k|v output (ops.attn_dense)."""
        from .. import ops
        n = pix.shape[0]
        D, P, H = self.dim, self.patch, self.heads
        x = pix.to(self.device, torch.float32)
        cols = F.unfold(x, kernel_size=P, stride=P).transpose(1, 2)           # [n, np, 3*P*P]
        npch = cols.shape[1]
        pe = ops.reduce(ops.linear(cols.reshape(n * npch, -1).to(self.dtype).contiguous(), self.q_patch,
                                   bias=self.patch_b)).view(n, npch, D)
        if self.cls is not None:
            pe = torch.cat([self.cls.view(1, 1, D).expand(n, 1, D), pe], 1)
        L = pe.shape[1]
        h = (pe + self.pos[:L]).reshape(n * L, D).contiguous()                 # fp32 residual stream
        eps = self.eps
        if self.pre_ln[0] is not None:
            nrm = torch.empty_like(h)
            ops.add_norm(h, None, self.pre_ln[0], self.pre_ln[1], eps, mode=1, out_f32=nrm)  # (out_f32 needs the bf16 output too)
            h = nrm
        act = ops.ACT_GELU if self.use_gelu else ops.ACT_GELU_QUICK
        a = ops.add_norm(h, None, self.layers[0]["ln1"][0], self.layers[0]["ln1"][1], eps, mode=1)
        for i, ly in enumerate(self.layers):
            qkv = ops.reduce(ops.linear(a, ly["q_qkv_w"], bias=ly["qkv_b"]), dtype=self.dtype)
            if self.dtype == torch.bfloat16 and (D // H) in (64, 80, 96, 128):
                o = ops.attn_dense(qkv.contiguous(), n, L, H)                   # non-causal, MFMA
            else:
                q, k, v = qkv.view(n, L, 3, H, D // H).permute(2, 0, 3, 1, 4)
                o = F.scaled_dot_product_attention(q, k, v)                    # non-causal
                o = o.transpose(1, 2).reshape(n * L, D).contiguous()
            a2 = ops.add_norm(h, ops.linear(o, ly["q_o_w"], bias=ly["o_b"]), ly["ln2"][0], ly["ln2"][1], eps, mode=1)
            f1 = ops.linear(a2, ly["q_f1_w"], bias=ly["f1_b"])
            g = ops.act(f1, f1.N, act)
            f2 = ops.linear(g, ly["q_f2_w"], bias=ly["f2_b"])
            if i + 1 < len(self.layers):
                nx = self.layers[i + 1]["ln1"]
                a = ops.add_norm(h, f2, nx[0], nx[1], eps, mode=1)
            elif self.post_ln[0] is not None:
                nrm = torch.empty_like(h)
                ops.add_norm(h, f2, self.post_ln[0], self.post_ln[1], eps, mode=1, out_f32=nrm)  # (out_f32 needs the bf16 output too)
                h = nrm
            else:
                ops.add_norm(h, f2, self.layers[-1]["ln2"][0], self.layers[-1]["ln2"][1], eps, mode=1, want_out=False)
        h = h.view(n, L, D)
        if self.cls is not None:
            h = h[:, 1:]                                                       # drop CLS
        hb = h.reshape(-1, D).to(self.dtype).contiguous()
        y = ops.act(ops.linear(hb, self.q_mm0, bias=self.mm0[1]), self.mm0[0].shape[0], ops.ACT_GELU)
        y = ops.reduce(ops.linear(y, self.q_mm2, bias=self.mm2[1]))
        return y.view(n, -1, self.out_dim)

    def embed_image(self, data) -> torch.Tensor:
        """One image -> [n_tokens, out_dim] f32 rows to splice into the prompt."""
        return self.embed_images([data])[0]

    TILE_BATCH = 64  # tiles per vision-tower launch sequence (bounds the attention workspace)

    def embed_images(self, datas) -> List[torch.Tensor]:
        """Several images (e.g. every request that arrived in one engine step) through the vision
        tower together: their tiles are concatenated into batches of up to TILE_BATCH, so the ViT's
        GEMMs run at batch 64 instead of one image's 1-5 tiles at a time."""
        pre = [self.preprocess(d) for d in datas]
        tiles = torch.cat([t for t, _ in pre], 0)
        enc = torch.cat([self.encode_tiles(tiles[i:i + self.TILE_BATCH])
                         for i in range(0, tiles.shape[0], self.TILE_BATCH)], 0)
        out, o = [], 0
        for t, layout in pre:
            out.append(self._assemble(enc[o:o + t.shape[0]], layout))
            o += t.shape[0]
        return out

    def _assemble(self, e: torch.Tensor, layout) -> torch.Tensor:
        """Encoded tiles of one image -> its prompt rows (anyres: base tile, unpadded grid, newlines).
        On the GPU: one gather (ops.gather_rows) through an index vector cached per layout."""
        if layout is None:
            return e[0]
        if e.is_cuda:
            from .. import ops
            n_t, n_p, C = e.shape
            key = (tuple(layout), n_t, n_p, self.newline is not None)
            idx = self._asm_idx.get(key) if hasattr(self, "_asm_idx") else None
            if idx is None:
                # the torch assembly below run on row numbers gives the source row of every output row
                rows = torch.arange(n_t * n_p, dtype=torch.float64).view(n_t, n_p, 1)
                saved, self.newline = self.newline, (torch.full((1,), -1.0, dtype=torch.float64)
                                                     if self.newline is not None else None)
                try:
                    idx = self._assemble_torch(rows, layout).view(-1).round().long().to(e.device)
                finally:
                    self.newline = saved
                if not hasattr(self, "_asm_idx"):
                    self._asm_idx = {}
                self._asm_idx[key] = idx
            fill = self.newline.to(e.dtype) if self.newline is not None else None
            return ops.gather_rows(e.reshape(n_t * n_p, C), idx, fill)
        return self._assemble_torch(e, layout)

    def _assemble_torch(self, e: torch.Tensor, layout) -> torch.Tensor:
        gw, gh, ow, oh = layout
        g = self.grid
        base, rest = e[0], e[1:]                                               # [np, C]
        C = e.shape[-1]
        feat = rest.view(gh, gw, g, g, C).permute(0, 2, 1, 3, 4).reshape(gh * g, gw * g, C)
        # spatial unpad: drop the padding rows / cols the letterboxing added
        cur_h, cur_w = feat.shape[0], feat.shape[1]
        if ow / oh > cur_w / cur_h:
            nh = int(oh * cur_w / ow)
            pad = (cur_h - nh) // 2
            feat = feat[pad:pad + nh]
        else:
            nw = int(ow * cur_h / oh)
            pad = (cur_w - nw) // 2
            feat = feat[:, pad:pad + nw]
        if self.newline is not None:
            nl = self.newline.view(1, 1, C).expand(feat.shape[0], 1, C)
            feat = torch.cat([feat, nl], 1)
        return torch.cat([base, feat.reshape(-1, C)], 0)
