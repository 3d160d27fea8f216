"""One-shot and two-shot all-reduce over IPC-mapped peer buffers (ops/csrc/allreduce.hip) for the
tensor-parallel messages up to 4 M elements (decode rows of any batch, small prefill chunks); RCCL
stays the path for anything larger or when peer mapping is unavailable.  SURVEY §2.9 (planned TP collective shapes) and §2.11 (custom one-shot all-reduce
over peer-mapped IPC buffers, hipIpcGetMemHandle).  The reference has no collective of its own:
its only tensor parallelism is vLLM's NCCL (backend/python/vllm/backend.py:102-103).

Setup (once per TP group): every rank hipMallocs one region (flags, per-block call counters, two
1 MiB data slots), exports it with hipIpcGetMemHandle, all-gathers the 64-byte handles over the
group, and opens the peers' handles with hipIpcOpenMemHandle.  Each call is then one kernel on
the caller's stream -- capturable in the decode hipGraph, since the per-block epochs live in
device memory.
"""
from __future__ import annotations

import ctypes
import logging
import os
from typing import List, Optional

import torch

log = logging.getLogger("localai_amd.custom_ar")

# decode layer boundaries as one fused all-reduce + residual + norm launch (CustomAllReduce.add_norm)
FUSED_ADD_NORM = os.environ.get("LOCALAI_AMD_AR_ADD_NORM", "1") == "1"

HIP_IPC_HANDLE_SIZE = 64
_hipIpcMemLazyEnablePeerAccess = 0x1
_hipDeviceMallocUncached = 0x3
# regions are rounded up to this so no allocator ever sub-allocates them from a shared chunk
# (hipIpcGetMemHandle exports whole allocations only: a sub-allocated pointer fails with
# hipErrorInvalidValue)
_REGION_ALIGN = 2 << 20


class _HipIpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * HIP_IPC_HANDLE_SIZE)]


def _hip():
    """The HIP runtime torch itself loaded (one runtime per process)."""
    import torch.cuda  # noqa: F401
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    h = ctypes.CDLL(lib if os.path.exists(lib) else "libamdhip64.so")
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    h.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.c_void_p]
    h.hipFree.argtypes = [ctypes.c_void_p]
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_HipIpcHandle), ctypes.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), _HipIpcHandle, ctypes.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    for f in ("hipMalloc", "hipFree", "hipMemset", "hipIpcGetMemHandle", "hipIpcOpenMemHandle",
              "hipIpcCloseMemHandle", "hipMemcpy", "hipExtMallocWithFlags", "hipMemGetAddressRange"):
        getattr(h, f).restype = ctypes.c_int
    return h


class CustomAllReduce:
    """In-place sum over the ranks of `group` for fp32 / bf16 tensors of at most `max_elems`."""

    # ~1 s of polling (s_sleep 2 + one system-scope load per poll): a peer that never arrives costs one bounded wait
    # (err flag set, result wrong) instead of a hung GPU
    SPIN_LIMIT = 1 << 20

    def __init__(self, group, rank: int, world: int, device: torch.device, twoshot: Optional[bool] = None):
        from .. import ops
        import torch.distributed as dist
        if world < 2 or world > 8:
            raise ValueError("custom all-reduce needs 2..8 ranks")
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.L = ops.lib()
        for f in ("la_ar_buffer_bytes", "la_ar_max_elems", "la_ar_err_offset", "la_ar2_buffer_bytes",
                  "la_ar2_max_elems", "la_ar2_err_offset"):
            getattr(self.L, f).restype = ctypes.c_long
        for f in ("la_allreduce_oneshot", "la_allreduce_twoshot"):
            getattr(self.L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long,
                                           ctypes.c_void_p] + ([ctypes.c_int] if "twoshot" in f else [])
            getattr(self.L, f).restype = ctypes.c_int
        self.L.la_allreduce_add_norm.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                 ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                                                 ctypes.c_void_p]
        self.L.la_allreduce_add_norm.restype = ctypes.c_int
        if twoshot is None:
            twoshot = os.environ.get("LOCALAI_AMD_AR_TWOSHOT", "1") != "0"
        self.max_elems = int(self.L.la_ar_max_elems())          # one-shot: latency-bound decode rows
        self.max_elems2 = int(self.L.la_ar2_max_elems()) if twoshot else 0  # two-shot: wide batches
        # one region per protocol: (bytes, error-word offset)
        sizes = [int(self.L.la_ar_buffer_bytes())] + ([int(self.L.la_ar2_buffer_bytes())] if twoshot else [])
        self.err_offs = [int(self.L.la_ar_err_offset())] + ([int(self.L.la_ar2_err_offset())] if twoshot else [])
        self.nbytes = sizes[0]
        self.hip = _hip()
        self.owns: List[int] = []
        self.own = None
        self._opened: List[int] = []
        err = ""
        with torch.cuda.device(self.device):
            # every rank reaches every collective below whatever fails locally, and all of them
            # agree at the end: a group where one rank cannot map a peer must stay on RCCL
            hbs: List[bytes] = []
            try:
                for nb in sizes:
                    nb = -(-nb // _REGION_ALIGN) * _REGION_ALIGN
                    ptr = self._alloc(nb)
                    self.owns.append(ptr)
                    self._check(self.hip.hipMemset(ctypes.c_void_p(ptr), 0, nb), "hipMemset")
                torch.cuda.synchronize(self.device)
                for k, o in enumerate(self.owns):
                    hnd = _HipIpcHandle()
                    rc = self.hip.hipIpcGetMemHandle(ctypes.byref(hnd), ctypes.c_void_p(o))
                    if rc != 0:
                        raise RuntimeError(f"hipIpcGetMemHandle failed with hipError {rc} on region {k} "
                                           f"({self._describe(o, sizes[k])})")
                    hbs.append(ctypes.string_at(ctypes.addressof(hnd), HIP_IPC_HANDLE_SIZE))  # .reserved stops at a NUL
            except Exception as e:  # noqa: BLE001
                err = str(e)
                log.warning("rank %d: custom all-reduce setup: %s", rank, err)
            self.own = self.owns[0] if self.owns else None
            handles: List[Optional[list]] = [None] * world
            dist.all_gather_object(handles, hbs, group=group)
            # ranks sharing this GPU (tests, rehearsals): the two-shot grid is capped so all of
            # their persistent grids fit on the device at once (allreduce.hip two-shot comment)
            keys: List[Optional[str]] = [None] * world
            dist.all_gather_object(keys, self._device_key(), group=group)
            self.share = max(1, sum(1 for k in keys if k == keys[rank]))
            self.max_grid2 = max(16, 128 // self.share)
            self.ptr_sets: List[List[int]] = [[] for _ in sizes]
            for r, h_list in enumerate(handles):
                for k in range(len(sizes)):
                    if r == rank:
                        self.ptr_sets[k].append(self.owns[k] if k < len(self.owns) else 0)
                        continue
                    h_bytes = h_list[k] if h_list and k < len(h_list) else None
                    if err or not h_bytes or len(h_bytes) != HIP_IPC_HANDLE_SIZE:
                        err = err or f"rank {r} exported no handle"
                        self.ptr_sets[k].append(0)
                        continue
                    try:
                        h = _HipIpcHandle()
                        ctypes.memmove(ctypes.addressof(h), h_bytes, HIP_IPC_HANDLE_SIZE)
                        p = ctypes.c_void_p()
                        self._check(self.hip.hipIpcOpenMemHandle(ctypes.byref(p), h, _hipIpcMemLazyEnablePeerAccess),
                                    f"hipIpcOpenMemHandle(rank {r})")
                        self.ptr_sets[k].append(p.value)
                        self._opened.append(p.value)
                    except Exception as e:  # noqa: BLE001
                        err = str(e)
                        self.ptr_sets[k].append(0)
            oks: List[Optional[str]] = [None] * world
            dist.all_gather_object(oks, err, group=group)
            bad = [f"rank {r}: {m}" for r, m in enumerate(oks) if m]
            if bad:
                self.close()
                raise RuntimeError("; ".join(bad))
        self.ptrs = self.ptr_sets[0]
        self._bufs = [(ctypes.c_void_p * world)(*ps) for ps in self.ptr_sets]

    def _alloc(self, nb: int) -> int:
        """The region: uncached device memory (MTYPE UC), so the peers' flag stores and data are
        seen by polling loads without relying on system-scope L2 write-back / invalidate; plain
        hipMalloc if the driver refuses that flag.  Sized to whole 2 MiB granules: never a
        sub-allocation, which IPC export would reject."""
        ptr = ctypes.c_void_p()
        self.uncached = self.hip.hipExtMallocWithFlags(ctypes.byref(ptr), nb, _hipDeviceMallocUncached) == 0
        if not self.uncached:
            self._check(self.hip.hipMalloc(ctypes.byref(ptr), nb), "hipMalloc")
        return ptr.value

    def _describe(self, ptr: int, nb: int) -> str:
        """Pointer, size and whether it is the base of its allocation (diagnostics for an IPC
        export failure)."""
        base, size = ctypes.c_void_p(), ctypes.c_size_t()
        rc = self.hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(ptr))
        if rc != 0:
            return f"ptr 0x{ptr:x}, {nb} B, hipMemGetAddressRange error {rc}"
        return (f"ptr 0x{ptr:x}, {nb} B, allocation base 0x{(base.value or 0):x} size {size.value} B"
                f"{'' if base.value == ptr else ' (SUB-ALLOCATED)'}, uncached={getattr(self, 'uncached', None)}")

    def _device_key(self) -> str:
        try:
            p = torch.cuda.get_device_properties(self.device)
            u = getattr(p, "uuid", None)
            if u is not None:
                return str(u)
            return f"{os.uname().nodename}:{p.name}:{self.device.index}"
        except Exception:  # noqa: BLE001
            return f"{os.uname().nodename}:{self.device}"

    @staticmethod
    def _check(rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what} failed with hipError {rc}")

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and 0 < t.numel() <= max(self.max_elems, self.max_elems2))

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In place; the caller checks supports(t).  Runs on the current stream: one-shot up to
        max_elems (one flag round trip, every rank reads all copies), two-shot beyond (reduce-
        scatter + all-gather: ~2n bytes read per rank instead of world x n)."""
        two = t.numel() > self.max_elems
        args = (t.data_ptr(), t.data_ptr(), t.numel(), int(t.dtype == torch.bfloat16), self.rank, self.world,
                self._bufs[1 if two else 0], self.SPIN_LIMIT, torch.cuda.current_stream(self.device).cuda_stream)
        rc = self.L.la_allreduce_twoshot(*args, self.max_grid2) if two else self.L.la_allreduce_oneshot(*args)
        if rc != 0:
            raise RuntimeError(f"la_allreduce_{'twoshot' if two else 'oneshot'} failed with code {rc}")
        return t

    ADD_NORM_CHANNELS = 256   # one-shot channels (1024 elements each) a fused call may span

    def supports_add_norm(self, M: int, D: int) -> bool:
        """The fused all-reduce + residual + norm kernel takes M rows of D: D % 8 == 0, D <= 8192,
        every row on its own one-shot channels (M * ceil(D / 1024) <= 256)."""
        return (FUSED_ADD_NORM and 1 <= M and 8 <= D <= 8192 and D % 8 == 0
                and M * -(-D // 1024) <= self.ADD_NORM_CHANNELS)

    def add_norm(self, part, bias, residual: torch.Tensor, weight: torch.Tensor, nbias, eps: float,
                 mode: int) -> torch.Tensor:
        """residual += all_reduce(part) (+ bias); return norm(residual) * weight (+ nbias) as bf16 --
        the decode layer boundary of a TP group in one launch (allreduce.hip
        allreduce_add_norm_kernel).  `part` is this rank's un-reduced ops.Partial (fp32 slabs or one
        bf16 matrix); every rank gets identical bits (rank-ordered fp32 sum of the bf16 wire rows)."""
        M, D = residual.shape
        t = part.t
        if t.dim() == 3:
            S, slab = t.shape[0], t.shape[1] * t.shape[2]
            assert t.dtype == torch.float32 and t.is_contiguous()
        else:
            S, slab = 0, 0
            assert t.dtype == torch.bfloat16 and t.is_contiguous()
        out = torch.empty(M, D, dtype=torch.bfloat16, device=residual.device)
        fp = lambda x: None if x is None else x.data_ptr()  # noqa: E731
        rc = self.L.la_allreduce_add_norm(t.data_ptr(), slab, S, M, D, self.rank, self.world, self._bufs[0],
                                          self.SPIN_LIMIT, residual.data_ptr(), fp(bias), weight.data_ptr(),
                                          fp(nbias), out.data_ptr(), float(eps), int(mode),
                                          torch.cuda.current_stream(self.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"la_allreduce_add_norm failed with code {rc}")
        return out

    def timed_out(self) -> bool:
        """True if a wait ever hit the spin limit (a peer never arrived): results since are suspect."""
        torch.cuda.synchronize(self.device)
        return self.error_flag()

    def error_flag(self) -> bool:
        """This rank's error words, without a device-wide synchronize: read at a point where the
        stream is already drained (the engine's token readback).  A timed-out wait on ANY rank
        writes every rank's word (allreduce.hip), so one rank's read speaks for the group."""
        for own, off in zip(self.owns, self.err_offs):
            v = ctypes.c_int(0)
            self._check(self.hip.hipMemcpy(ctypes.byref(v), ctypes.c_void_p(own + off), 4, 2),
                        "hipMemcpy")  # hipMemcpyDeviceToHost
            if v.value:
                return True
        return False

    def close(self):
        if not getattr(self, "owns", None):
            self.own = None
            return
        try:
            torch.cuda.synchronize(self.device)
            for p in self._opened:
                self.hip.hipIpcCloseMemHandle(ctypes.c_void_p(p))
            self._opened = []
            for o in self.owns:
                self.hip.hipFree(ctypes.c_void_p(o))
        finally:
            self.owns = []
            self.own = None


def maybe_create(group, rank: int, world: int, device) -> Optional[CustomAllReduce]:
    """A CustomAllReduce for a GPU TP group, or None (CPU, a single rank, LOCALAI_AMD_CUSTOM_AR=0,
    or peer mapping refused) -- callers then keep RCCL."""
    if world < 2 or not torch.cuda.is_available() or str(device) == "cpu":
        return None
    if os.environ.get("LOCALAI_AMD_CUSTOM_AR", "1") == "0":
        return None
    try:
        return CustomAllReduce(group, rank, world, torch.device(device))
    except Exception as e:  # noqa: BLE001 - no IPC / peer access: RCCL only
        log.warning("custom all-reduce unavailable (%s); using RCCL", e)
        return None
