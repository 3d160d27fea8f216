"""The inference engine: one per loaded model (per GPU, or per TP group).

Reference behaviour it reproduces (`backend/cpp/llama/grpc-server.cpp`):
  * continuous batching over many concurrent sequences (update_slots :1546-1982) -- here a
    native C++ scheduler over a paged KV pool (localai_amd/native/engine_core.cpp);
  * prompt-prefix reuse (:1732-1750) -- global hashed prefix cache;
  * truncation keeping n_keep (:1694-1720); context-full => finish "length" (:1574-1590);
  * stop strings with partial hold-back and UTF-8 completeness (:1010-1123);
  * final reply carries token counts (:2354-2358); per-request timings (:305-359).
Differences: sampling runs on the GPU (no logits D2H), cancellation frees the sequence
(fixes SURVEY Q4), ignore_eos is honoured (Q16), TokenizeString is implemented (Q10).

Decode steps replay per-batch-size HIP graphs (torch.cuda.CUDAGraph == hipGraph on ROCm).
"""
from __future__ import annotations

import collections
import dataclasses
import hashlib
import logging
import math
import os
import pickle
import queue
import re
import struct
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..gguf import GGUFReader  # noqa: F401 (re-exported for callers)
from ..models.hf_checkpoint import open_model
from ..models.decoder import DecoderModel, ForwardBatch, TPInfo
from ..native import core
from ..tokenizer import Tokenizer
from .prompt_cache import PromptCacheFiles
from .sampling_params import SamplingParams
from .speculative import DraftModel, ngram_draft
from ..utils import faults
from ..utils.trace import get_tracer, roctx

log = logging.getLogger("localai_amd.engine")
# multi-step decode runs stream each step's tokens as its event fires (LLMEngine._run_streamed)
STREAM_STEPS = os.environ.get("LOCALAI_AMD_STREAM_STEPS", "1") == "1"


@dataclass
class EngineConfig:
    model_path: str
    device: str = "cuda:0"
    context_size: int = 4096
    max_num_seqs: int = 256
    max_batched_tokens: int = 8192
    block_size: int = 32
    gpu_memory_utilization: float = 0.85
    max_kv_tokens: int = 0            # 0: max_num_seqs * context_size (capped by memory)
    prefix_cache: bool = True
    use_graphs: bool = True
    embeddings: bool = False
    rope_freq_base: float = 0.0
    rope_freq_scale: float = 0.0
    rope_scaling: str = ""
    decode_steps: int = 8             # device-resident decode steps per host round trip (graphs only)
    # ... and at batch >= wide_batch with nothing waiting: the host round trip (sync, emit, schedule,
    # upload) is then paid half as often (batch 256: +1.4 % tok/s measured, arrivals still cut a
    # run short through the num_waiting check)
    decode_steps_wide: int = 16
    wide_batch: int = 128
    mmproj: str = ""                  # LLaVA vision tower + projector GGUF (images in prompts)
    bias_capacity: int = 16           # logit-bias / EOS-ban entries per sequence inside the graph
    blas_tune: bool = True            # tune the hipBLASLt/rocBLAS solution per decode GEMM shape at warm-up
    lora_adapters: tuple = ()         # ((adapter GGUF path, scale), ...) merged into the weights at load
    record_tokens: bool = False       # final Event carries the generated token ids (numerics tests)
    # ... and the raw model logits row (fp32, on the device) each token was sampled from: the
    # decode graph copies every step's logits into a [K, B, V] buffer (one extra copy kernel in
    # the graph; numerics tests only)
    record_logits: bool = False
    # burst admission: an idle engine that receives work waits until arrivals pause for
    # admission_quiet_ms (at most admission_window_ms) before its first prefill, so a burst of
    # concurrent requests is prefilled in full chunks instead of the first arrival alone while the
    # gateway thread is still parsing the rest (it holds the GIL meanwhile); 0 disables
    admission_window_ms: float = 30.0
    admission_quiet_ms: float = 2.0
    # ... and closes early once the waiting prompts fill half a prefill chunk (that chunk runs
    # while the rest of the burst arrives; HTTP C=256 p50 TTFT 293 -> 275 ms vs closing at a full
    # chunk, r5_k2_*.log); -1 = max_batched_tokens / 2, 0 = never
    admission_close_tokens: int = -1
    # burst prefill first: while prompts of a burst are still being prefilled and every sequence
    # that could decode holds only its first token (younger than this many ms), steps are
    # prefill-only, so the burst's chunks run back to back (TTFT) and its rows then decode as one
    # batch; a running stream (rows past their first token) keeps prefill and decode mixed.
    # 2 s covers a Mixtral-8x7B C=256 burst (r5_k2_mx_*.log); 0 disables
    prefill_first_ms: float = 2000.0
    # ... where a burst is the requests of an idle -> busy transition plus every later arrival
    # within burst_gap_ms of the burst's previous one (a synchronised client wave lands 0.3 ms
    # apart; open-loop arrivals at 90 req/s average 11 ms apart and never form a long burst)
    burst_gap_ms: float = 5.0
    # while new prompts wait or are mid-prefill, a decode run holds at most this many ms of device
    # steps (their admission waits for the run); 0: one step per round trip
    admit_budget_ms: float = 25.0
    draft_model: str = ""             # speculative decoding: draft LM GGUF (engine/speculative.DraftModel)
    quantization: str = ""            # HF checkpoints: load-time quantisation (bnb_4bit / bnb_8bit / ...)
    draft_max_seqs: int = 16          # draft-model KV cache capacity in sequences of context_size
    # constrained rows inside multi-step graph runs: the device transition table
    # (grammar_advance_kernel) walks the learned parse-state transitions, permissive states
    # (JSON strings) are expanded on the helper thread, and rows park only at table misses.  On
    # by default since the background expansion (FC C=32: 1914 single-step round trips per 6
    # waves -> 121; gpurun_out/r5_fc_base.log vs r5_fc_ra.log)
    grammar_run_ahead: bool = dataclasses.field(
        default_factory=lambda: os.environ.get("LOCALAI_AMD_GRAMMAR_RUN_AHEAD", "1") == "1")


@dataclass
class Event:
    text: bytes = b""
    token: int = -1
    finished: bool = False
    finish_reason: str = ""
    prompt_tokens: int = 0
    completion_tokens: int = 0
    error: str = ""
    token_ids: Optional[List[int]] = None   # final event, with EngineConfig.record_tokens
    logits: Optional[List[torch.Tensor]] = None  # final event, with EngineConfig.record_logits


@dataclass
class Request:
    id: int
    prompt: List[int]
    params: SamplingParams
    callback: Callable[[Event], None]
    stream: object = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_t: float = 0.0
    burst: bool = False      # member of the burst that woke the engine (_defer_decode)
    done: bool = False
    n_prompt: int = 0
    n_gen: int = 0
    mu: float = 0.0
    cancelled: bool = False
    sink: object = None
    grammar: object = None       # native GrammarState (GBNF-constrained decoding)
    mm_pos: object = None        # {prompt position: row of mm_emb} for image-embedding positions
    mm_emb: object = None        # [rows, n_embd] f32 projected image embeddings (device)
    spec_drafted: int = 0        # n-gram speculation bookkeeping (adaptive back-off)
    spec_accepted: int = 0
    spec_off: bool = False
    out_ids: Optional[List[int]] = None  # generated ids (EngineConfig.record_tokens)
    out_logits: Optional[list] = None    # their logits rows (EngineConfig.record_logits)
    prompt_text: Optional[str] = None    # the prompt as given (GetMetrics' prompt_json_for_slot)


def _noop_callback(ev):  # follower ranks: the leader talks to the client
    pass


class LLMEngine:
    def __init__(self, cfg: EngineConfig, tp: Optional[TPInfo] = None, ctrl_group=None):
        """tp: tensor-parallel rank info (one engine per GPU, identical schedulers on every rank).
        ctrl_group: a gloo process group the leader (rank 0) uses to broadcast new requests /
        aborts to the followers each step; required when tp.world > 1."""
        self.cfg = cfg
        self.tp = tp or TPInfo()
        self.leader = self.tp.rank == 0
        self.ctrl = ctrl_group
        if self.tp.world > 1 and ctrl_group is None:
            raise ValueError("tensor-parallel engines need a control process group")
        self._shm = None
        if self.tp.world > 1:
            from ..parallel.shm_channel import ShmChannel
            self._shm = ShmChannel.create(ctrl_group, self.tp.rank, self.tp.world)
        self.device = torch.device(cfg.device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            ops.lib()  # fail loudly if the kernel library is missing on a GPU box
        self.reader = open_model(cfg.model_path, cfg.quantization)  # GGUF file or HF checkpoint directory
        self.tokenizer = Tokenizer.from_gguf(self.reader)
        ro = {}
        if cfg.rope_freq_base:
            ro["freq_base"] = cfg.rope_freq_base
        if cfg.rope_freq_scale:
            ro["freq_scale"] = cfg.rope_freq_scale
        if cfg.rope_scaling:
            ro["type"] = cfg.rope_scaling
        lora = None
        if cfg.lora_adapters:
            from ..models.lora import LoraSet
            lora = LoraSet(cfg.lora_adapters)
        self.model = DecoderModel(self.reader, self.device, tp=tp, max_pos=cfg.context_size, rope_overrides=ro,
                                  lora=lora)
        self.hp = self.model.hp
        self.vocab = core.Vocab(self.tokenizer.pieces)
        self.gvocab = core.GrammarVocab(self.tokenizer.pieces, sorted(self.tokenizer.eog))
        self._eog_list = sorted(self.tokenizer.eog)
        self._grammars: Dict[str, object] = {}
        # allowed-token masks of grammar parse states, resident on the device (_grammar_mask_slot)
        self._gmask_cache: "collections.OrderedDict" = collections.OrderedDict()
        self._gslot_key: Dict[int, tuple] = {}   # device mask slot -> its (grammar, state key) cache entry
        self._gmask_pool: Optional[torch.Tensor] = None
        self._gmask_free: List[int] = []
        self._gmask_over: Dict[tuple, int] = {}   # states whose budgeted walk gave up once
        self._gmask_pending: Dict[tuple, object] = {}   # full walks running on the helper thread
        self._gmask_bg = None
        self._gnext: Optional[torch.Tensor] = None
        self._gtrans: Dict[tuple, Optional[int]] = {}   # (slot, token) -> next slot (host mirror)
        self._gtrans_in: Dict[int, set] = {}
        self._gpend: List[tuple] = []                    # learned, not yet written to the device
        self._gdev: set = set()                          # (slot, token) keys the device table holds
        self._gepoch = 0                                 # bumped whenever a mask slot is reused
        self._ghit: Dict[str, float] = {}                # per grammar: EMA of learned-transition hits
        self._gexpanded: set = set()                     # slots whose outgoing transitions are all learned
        self._gexp_pend: dict = {}                       # slot -> background expansion in flight
        self._gmask_np: Dict[int, np.ndarray] = {}       # host copies of the pool's masks (run-ahead)
        self._mm_embs: Dict[int, list] = {}  # inbox "mm" item -> its images' embeddings (batched encode)
        self.clip = None
        if cfg.mmproj:
            from ..models.clip import ClipVision
            self.clip = ClipVision(cfg.mmproj, self.device)
            if self.clip.out_dim != self.hp.n_embd:
                raise ValueError(f"mmproj projects to {self.clip.out_dim}, the LLM embeds {self.hp.n_embd}")
        self.ctx = cfg.context_size
        bs = cfg.block_size
        if self.device.type == "cuda":
            # legacy path (LOCALAI_AMD_TILE_GEMM=0): prefill / big decode batches run hipBLASLt on
            # bf16 copies, materialised before any graph capture.  The default path multiplies the
            # quantised weights directly (gemm_q.hip) and keeps no copy -- except for formats the
            # tile GEMM does not read (Q5_K, Q3_K, Q2_K, IQ*, F16, K % 256 != 0): those get a
            # persistent bf16 copy up front, so a decode batch of 65-256 rows never re-dequantises
            # them into scratch inside its graph (2 B/weight written + read back every step)
            self._materialize_bf16(only_non_tile=ops.TILE_GEMM)
        num_blocks = self._num_kv_blocks()
        if self.tp.world > 1:
            # the schedulers are replicated: every rank must admit and preempt exactly as rank 0
            # does, so the KV pool is the smallest any rank can hold (each rank sized it from its
            # own free memory)
            import torch.distributed as dist
            nb = torch.tensor([num_blocks], dtype=torch.int64)
            dist.all_reduce(nb, op=dist.ReduceOp.MIN, group=self.ctrl)
            num_blocks = int(nb.item())
        if faults.hit("kv_alloc"):
            raise faults.InjectedFault("hipMalloc failed for the KV cache (injected fault): out of memory")
        self.kv = self.model.new_kv_cache(num_blocks, bs)
        self.drafter = None
        if cfg.draft_model:
            self.drafter = DraftModel(cfg.draft_model, self.device, cfg.draft_max_seqs, self.ctx, self.hp.n_vocab,
                                      max_batched_tokens=cfg.max_batched_tokens)
        self.sched = core.Scheduler(num_blocks, bs, cfg.max_num_seqs, cfg.max_batched_tokens, self.ctx,
                                    cfg.prefix_cache, 1 if (cfg.use_graphs and self.device.type == "cuda") else 0)
        self.max_blocks = (self.ctx + bs - 1) // bs
        self.requests: Dict[int, Request] = {}
        self._inbox: "queue.Queue" = queue.Queue()
        self._next_id = 1
        self._id_lock = threading.Lock()
        self._wake = threading.Event()
        # diagnostics (bench.py BENCH_ARRIVALS=1): perf_counter of every add_request and, per idle ->
        # busy transition, (time the admission window closed, requests waiting then)
        self._burst_last = 0.0    # arrival time of the current burst's latest member (_defer_decode)
        self._step_ms = 8.0       # EMA of one device decode step (_lookahead's admission budget)
        self.arrival_log: Optional[list] = None
        self.admit_log: Optional[list] = None
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self.healthy = True          # False after a fatal device error: the model manager respawns
        self.fatal_error = ""
        self._graphs: Dict[int, tuple] = {}
        # tensor parallelism, all-greedy batches: graphs whose sampler is the distributed argmax
        # (TPInfo.argmax_cols) -- no full-vocabulary all-gather, no RCCL call in the graph
        self._graphs_tpg: Dict[int, tuple] = {}
        self._graphs_tps: Dict[tuple, tuple] = {}   # (Bp, mirostat rows) -> distributed-sampler graph
        self.tracer = get_tracer()
        self._pcache = PromptCacheFiles()
        self._graph_pool = None
        self.k1_reasons = collections.Counter()
        self.k_hist = collections.Counter()   # (device steps, constrained rows in the batch) per decode run
        self.k_log = collections.deque(maxlen=1024)  # (K, constrained rows, batch, waiting) per run, in order
        self.metrics = {"prompt_tokens": 0, "gen_tokens": 0, "steps": 0, "prefill_s": 0.0, "decode_s": 0.0,
                        "requests": 0, "spec_steps": 0, "spec_drafted": 0, "spec_accepted": 0,
                        "grammar_runs": 0, "grammar_run_rows": 0, "grammar_run_tokens": 0, "grammar_drift": 0}
        self.last_request_stats: dict = {}
        self.busy = False

    # ------------------------------------------------------------------ setup
    def _materialize_bf16(self, only_non_tile: bool = False):
        """bf16 copies for the weights the quantised GEMMs cannot read (only_non_tile), or for all
        of them (legacy LOCALAI_AMD_TILE_GEMM=0 path).  The copies for non-tile formats are a speed
        option (no re-dequantisation of Q5_K / Q3_K / IQ* ... per call), so they are made only when
        they fit: after them the KV cache must still get every block the config asks for within
        gpu_memory_utilization (a 70B Q5_K_M would otherwise gain ~140 GB of copies and stop
        loading).  LOCALAI_AMD_BF16_COPIES=always|never overrides; the bytes spent are logged."""
        m = self.model

        def want(ws) -> bool:
            return not only_non_tile or not all(w.tile_ok for w in ws)
        groups = []
        for L in m.layers:
            for grp in (L.qkv, L.gate_up, [L.wo]) + (([L.down],) if L.down is not None else ()):
                if want(grp):
                    groups.append(grp)
            if L.experts and not only_non_tile:   # (the grouped MoE kernels read their own planes)
                for gu, d in L.experts:
                    for grp in (gu, [d]):
                        if want(grp):
                            groups.append(grp)
        if want([m.output]):
            groups.append([m.output])
        need = sum(w.N * w.K * 2 for grp in groups for w in grp if w.bf16 is None and w.fmt != ops.FMT_BF16)
        if not need:
            # only bf16-format weights (or copies made already): their "copy" is a view of the planes
            for grp in groups:
                for w in grp:
                    w.materialize_bf16()
                if len(grp) > 1:
                    ops.fuse_bf16(grp)
            return
        policy = os.environ.get("LOCALAI_AMD_BF16_COPIES", "auto")
        if policy == "never" and only_non_tile:
            log.info("bf16 copies disabled: %.2f GB of weights stay quantised (dequantised per call)", need / 2**30)
            return
        if policy == "auto" and only_non_tile and self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            # memory PyTorch's caching allocator holds but no tensor uses is free for these copies
            free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
            budget = int(free - (1.0 - self.cfg.gpu_memory_utilization) * total) - (4 << 30)
            kv = self._kv_blocks_wanted() * self._kv_block_bytes()
            # copies under 1 GiB are always made (a small model beside other tenants of the GPU --
            # e.g. earlier engines of the same process -- would otherwise lose them to a budget
            # computed from the device-wide free memory)
            if need > budget - kv and need > (1 << 30):
                log.warning("not materialising %.2f GB of bf16 weight copies (%.2f GB left after the %.2f GB KV "
                            "cache): those weights are dequantised per call", need / 2**30,
                            max(0, budget - kv) / 2**30, kv / 2**30)
                return
        for grp in groups:
            for w in grp:
                w.materialize_bf16()
            if len(grp) > 1:
                ops.fuse_bf16(grp)   # one library GEMM for a mixed-format q|k + v
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        log.info("materialised %.2f GB of bf16 weight copies", need / 2**30)

    def _kv_block_bytes(self) -> int:
        return 2 * self.hp.n_layer * self.model.Hkv * self.cfg.block_size * self.model.Dh * 2

    def _kv_blocks_wanted(self) -> int:
        cfg = self.cfg
        bs = cfg.block_size
        want_tokens = cfg.max_kv_tokens or cfg.max_num_seqs * self.ctx
        return (want_tokens + bs - 1) // bs + cfg.max_num_seqs + 4

    def _num_kv_blocks(self) -> int:
        cfg = self.cfg
        bpb = self._kv_block_bytes()
        want = self._kv_blocks_wanted()
        if self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            free += torch.cuda.memory_reserved(self.device) - torch.cuda.memory_allocated(self.device)
            budget = int(free - (1.0 - cfg.gpu_memory_utilization) * total) - (4 << 30)
            cap = max(64, budget // bpb)
            want = min(want, cap)
        return max(want, 16)

    # ------------------------------------------------------------------ public API
    def new_id(self) -> int:
        with self._id_lock:
            i = self._next_id
            self._next_id += 1
            return i

    def tokenize(self, text: str, add_bos: Optional[bool] = None) -> List[int]:
        return self.tokenizer.encode(text, add_bos=add_bos)

    def add_request(self, prompt, params: SamplingParams, callback: Callable[[Event], None],
                    req_id: Optional[int] = None, sink=None, images: Optional[Sequence] = None) -> int:
        """Queue a generation.  `callback(Event)` gets every text delta and the final event;
        with a native `sink` (native/_la_http SseSink) text deltas go straight to
        `sink.push(text, n_generated)` (no Python Event per token) and only the final event
        reaches `callback`."""
        rid = req_id if req_id is not None else self.new_id()
        if self.arrival_log is not None:
            self.arrival_log.append(time.perf_counter())
        if not self.healthy:  # dead device: refuse instead of queueing work nobody will run
            callback(Event(finished=True, finish_reason="error", error=f"backend unhealthy: {self.fatal_error}"))
            return rid
        if images and self.clip is not None and isinstance(prompt, str):
            # the vision tower runs on the engine thread (single GPU stream owner)
            params.resolved_seed()
            self._inbox.put(("mm", rid, prompt, list(images), params, callback, sink))
            self._wake.set()
            return rid
        toks = self.tokenize(prompt) if isinstance(prompt, str) else list(prompt)
        if not toks:
            toks = [self.tokenizer.bos_id if self.tokenizer.bos_id >= 0 else 0]
        toks = self._truncate(toks, params.n_keep)
        params.resolved_seed()
        stops = list(params.stop)
        r = Request(rid, toks, params, callback, n_prompt=len(toks), mu=2.0 * params.mirostat_tau)
        r.prompt_text = prompt if isinstance(prompt, str) else None
        if self.cfg.record_tokens:
            r.out_ids = []
            r.out_logits = [] if self.cfg.record_logits else None
        r.stream = core.TextStream(self.vocab, stops)
        if params.grammar:
            r.grammar = core.GrammarState(self._grammar(params.grammar), self.gvocab)
        r.sink = sink
        if sink is not None:
            sink.set_prompt_tokens(r.n_prompt)
        self._inbox.put(r)
        self._wake.set()
        return rid

    def _grammar(self, text: str):
        g = self._grammars.get(text)
        if g is None:
            g = core.Grammar(text)  # ValueError on a malformed grammar (surfaced to the caller)
            if len(self._grammars) > 64:
                self._grammars.clear()
            self._grammars[text] = g
        return g

    def abort(self, rid: int):
        self._inbox.put(("abort", rid))
        self._wake.set()

    def _truncate(self, toks: List[int], n_keep: int) -> List[int]:
        # grpc-server.cpp:1694-1720: keep n_keep, drop whole blocks of (n_ctx - n_keep)/2 from the middle
        n_ctx = self.ctx
        if len(toks) < n_ctx:
            return toks
        n_keep = min(max(n_keep, 0), n_ctx - 4)
        n_left = n_ctx - n_keep
        n_block = max(1, n_left // 2)
        erased = (len(toks) - n_keep - n_block) // n_block
        new = toks[:n_keep] + toks[n_keep + erased * n_block:]
        return new[-(n_ctx - 1):] if len(new) >= n_ctx else new

    def generate(self, prompt, params: SamplingParams, timeout: float = 600.0) -> dict:
        """Blocking helper (Predict RPC semantics)."""
        out = bytearray()
        done = threading.Event()
        res = {}

        def cb(ev: Event):
            out.extend(ev.text)
            if ev.finished:
                res.update(finish_reason=ev.finish_reason, prompt_tokens=ev.prompt_tokens,
                           completion_tokens=ev.completion_tokens, error=ev.error)
                if ev.token_ids is not None:
                    res["token_ids"] = ev.token_ids
                if ev.logits is not None:
                    res["logits"] = ev.logits
                done.set()

        self.add_request(prompt, params, cb)
        if self._thread is None:
            while not done.is_set():
                self.step()
        elif not done.wait(timeout):
            raise TimeoutError("generation timed out")
        res["text"] = out.decode("utf-8", errors="replace")
        return res

    def start(self):
        # the serving thread shares the GIL with the gateway's event loop.  Round 4 shortened the
        # switch interval to 1 ms; with burst admission + prefill-first the interpreter's default
        # 5 ms measures better (HTTP C=256 26.11-26.18 k vs 26.03-26.06 k tok/s, r5_kn_*.log)
        sw = float(os.environ.get("LOCALAI_AMD_GIL_SWITCH_MS", "5"))
        if sw > 0:
            import sys
            sys.setswitchinterval(min(sys.getswitchinterval(), sw / 1e3))
        if self._thread is None:
            self._stop = False
            self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
            self._thread.start()

    def shutdown(self):
        if self.tracer is not None:
            self.tracer.flush()
        if self.tp.world > 1 and self.leader and not self._stop:
            self._inbox.put(("stop",))  # followers leave run_follower() after this broadcast
            self._wake.set()
            if self._thread is not None:
                self._thread.join(timeout=30)
                self._thread = None
            else:
                self._drain_inbox()
            return
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None
        if self._gmask_bg is not None:
            self._gmask_bg.shutdown(wait=False, cancel_futures=True)
            self._gmask_bg = None

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while not self._stop:
            try:
                worked = self.step()
            except Exception as e:  # fail all in-flight requests, keep serving
                log.exception("engine step failed")
                self._fail_all(str(e))
                worked = False
                if self._is_fatal(e):
                    # a device fault leaves the GPU context unusable: stop taking work and let
                    # the model manager's health check respawn the backend (pkg/model/loader.go
                    # CheckIsLoaded semantics)
                    self.healthy = False
                    self.fatal_error = str(e)
                    self._stop = True
                    self._reject_inbox(str(e))
            if not worked:
                self._wake.wait(0.05)
                self._wake.clear()
                if self._admit_window_ms() > 0 and not self.requests and not self._inbox.empty():
                    self._admit_burst()

    def _admit_window_ms(self) -> float:
        return float(os.environ.get("LOCALAI_AMD_ADMIT_WINDOW_MS", self.cfg.admission_window_ms))

    def _admit_burst(self):
        """Idle -> busy: let a burst of arrivals land before scheduling (see EngineConfig)."""
        t_end = time.perf_counter() + self._admit_window_ms() / 1e3
        quiet = self.cfg.admission_quiet_ms / 1e3
        close = int(os.environ.get("LOCALAI_AMD_ADMIT_TOKENS", self.cfg.admission_close_tokens))
        if close < 0:
            close = max(1, self.cfg.max_batched_tokens // 2)
        n = self._inbox.qsize()
        while time.perf_counter() < t_end:
            time.sleep(quiet)
            m = self._inbox.qsize()
            if m == n or (close and self._inbox_tokens() >= close):
                break
            n = m
        if self.admit_log is not None:
            self.admit_log.append((time.perf_counter(), n))

    def _inbox_tokens(self) -> int:
        with self._inbox.mutex:
            return sum(len(r.prompt) for r in self._inbox.queue if isinstance(r, Request))

    @staticmethod
    def _is_fatal(e: Exception) -> bool:
        if isinstance(e, faults.InjectedFault):
            return True
        m = str(e).lower()
        return any(k in m for k in ("hip error", "hiperror", "device-side", "illegal memory", "gpu hang",
                                    "memory access fault", "unspecified launch failure"))

    def _reject_inbox(self, msg: str):
        while True:
            try:
                item = self._inbox.get_nowait()
            except queue.Empty:
                return
            if isinstance(item, Request):
                item.callback(Event(finished=True, finish_reason="error", error=msg))

    def _fail_all(self, msg: str):
        for rid in list(self.requests):
            self._finish(self.requests[rid], "error", error=msg)

    # ------------------------------------------------------------------ step
    def active_slot_stats(self) -> Optional[dict]:
        """The reference's GetMetrics view (grpc-server.cpp:2434-2457, llama.get_active_slot()):
        live numbers of one in-flight request -- the oldest one that is generating -- or None when
        nothing is in flight.  Read from the serving thread's dict without locking: a snapshot."""
        now = time.perf_counter()
        best = None
        for r in list(self.requests.values()):
            if r.done or r.cancelled:
                continue
            if best is None or r.arrival < best.arrival:
                best = r
        if best is None:
            return None
        gen_s = (now - best.first_token_t) if best.first_token_t else 0.0
        return {"id": best.id, "prompt_tokens": best.n_prompt or len(best.prompt), "completion_tokens": best.n_gen,
                "tokens_per_second": (best.n_gen / gen_s) if gen_s > 0 else 0.0,
                "prompt": best.prompt_text if best.prompt_text is not None else self.tokenizer.decode(best.prompt)}

    def has_work(self) -> bool:
        return bool(self.requests) or not self._inbox.empty()

    def step(self) -> bool:
        self._drain_inbox()
        if not self.requests or self._stop:
            return False
        if faults.hit("engine_step"):
            raise faults.InjectedFault("HIP error: memory access fault on the engine stream (injected fault)")
        self.busy = True
        spec_k = self._spec_k()
        K = 1 + spec_k if spec_k else self._lookahead()
        plan = self.sched.schedule(K, self._defer_decode())  # spec: reserves KV slots for the draft positions
        did = False
        tr = self.tracer
        p_ids = plan["p_ids"]
        if len(p_ids):
            t0 = time.perf_counter()
            with roctx("prefill"):
                self._run_prefill(plan)
            t1 = time.perf_counter()
            self.metrics["prefill_s"] += t1 - t0
            if tr is not None:
                tr.complete("prefill", t0, t1, seqs=len(p_ids), tokens=int(plan["p_cu"][-1]))
            did = True
        d_ids = plan["d_ids"]
        if len(d_ids):
            t0 = time.perf_counter()
            with roctx("decode"):
                if spec_k:
                    self._run_spec(plan, spec_k)
                else:
                    nc = sum(1 for i in d_ids if self.requests[int(i)].grammar is not None)
                    self.k_hist[(K, nc)] += 1
                    self.k_log.append((K, nc, len(d_ids), self.sched.num_waiting))
                    self._run_decode(plan, K)
            t1 = time.perf_counter()
            self.metrics["decode_s"] += t1 - t0
            # per-device-step time of decode runs (EMA), for the admission budget of _lookahead
            self._step_ms = 0.8 * self._step_ms + 0.2 * (t1 - t0) * 1e3 / max(1, K)
            if tr is not None:
                tr.complete("decode", t0, t1, batch=len(d_ids), device_steps=K)
            did = True
        if did and self.tp.car is not None and self.leader:
            # the custom all-reduce's error word, read after the step's token readback (no extra
            # sync, no collective): a timeout on any rank sets every rank's word, and the leader
            # hands the verdict to the group with the next step's control broadcast
            self._ar_err = int(self.tp.car.error_flag())
        if tr is not None:
            tr.counter("sequences", time.perf_counter(), running=self.sched.num_running,
                       waiting=self.sched.num_waiting)
        self.metrics["steps"] += 1
        self.busy = bool(self.requests)
        return did or bool(self.requests)

    def _drain_inbox(self):
        items = []
        if self.leader:
            while True:
                try:
                    items.append(self._inbox.get_nowait())
                except queue.Empty:
                    break
        if self.tp.world > 1:
            # replicated scheduling: every rank applies the leader's new work in the same order,
            # so all ranks build identical batches and sample identical tokens
            # one int per step over the gloo control group; the pickled items only when there are
            # any (most decode steps have none).  group_src: the leader is rank 0 of its replica's
            # group, not necessarily global rank 0 (data-parallel x tensor-parallel layouts)
            if self._shm is not None:
                # ranks of one node: one sequenced message through /dev/shm (parallel/shm_channel.py)
                # instead of a TCP broadcast on every token's latency path
                if self.leader:
                    ar_err = getattr(self, "_ar_err", 0)
                    msg = struct.pack("<qq", len(items), ar_err)
                    if items:
                        msg += pickle.dumps([self._to_wire(it) for it in items], protocol=pickle.HIGHEST_PROTOCOL)
                    self._shm.publish(raw=msg)
                else:
                    msg = self._shm.receive(raw=True)
                    n_items, ar_err = struct.unpack_from("<qq", msg)
                    if n_items:
                        items = [self._from_wire(w) for w in pickle.loads(msg[16:])]
            else:
                import torch.distributed as dist
                # [new work items, custom all-reduce error verdict of the last step]: ONE host
                # collective per step
                n = torch.tensor([len(items), getattr(self, "_ar_err", 0)], dtype=torch.int64)
                dist.broadcast(n, group_src=0, group=self.ctrl)
                ar_err = int(n[1].item())
                n = n[:1]
                if int(n.item()):
                    box = [[self._to_wire(it) for it in items] if self.leader else None]
                    dist.broadcast_object_list(box, group_src=0, group=self.ctrl)
                    if not self.leader:
                        items = [self._from_wire(w) for w in box[0]]
        mm = [it for it in items if isinstance(it, tuple) and it[0] == "mm"]
        if len(mm) > 1 and self.clip is not None:
            # every image that arrived this step goes through the vision tower in shared batches
            try:
                flat = [im for it in mm for im in it[3]]
                embs = self.clip.embed_images(flat)
                o = 0
                for k, it in enumerate(mm):
                    n = len(it[3])
                    self._mm_embs[id(it)] = embs[o:o + n]
                    o += n
            except Exception:  # a bad image: fall back to per-request encoding (errors per request)
                self._mm_embs.clear()
        for item in items:
            self._apply(item)
        self._mm_embs.clear()
        if self.tp.world > 1 and ar_err and self.tp.car is not None:
            from ..models.decoder import CustomAllReduceTimeout
            self._ar_err = 0
            self._graphs.clear()   # the captured decode graphs call the custom kernel
            self._graphs_tpg.clear()
            self._graphs_tps.clear()
            self.tp.drop_custom_ar()
            raise CustomAllReduceTimeout("tensor-parallel custom all-reduce timed out on a late peer rank: the last "
                                         "step's results are invalid; the group continues on RCCL")

    @staticmethod
    def _to_wire(item):
        if isinstance(item, tuple):
            if item[0] == "embed":
                return ("embed", item[1]["texts"], item[1]["pool"])
            if item[0] == "mm":
                _, rid, prompt, images, params, _cb, _sink = item
                return ("mm", rid, prompt, images, dataclasses.asdict(params))
            return item
        r: Request = item
        return ("req", r.id, list(r.prompt), dataclasses.asdict(r.params))

    def _from_wire(self, w):
        kind = w[0]
        if kind == "req":
            _, rid, prompt, prm = w
            params = SamplingParams(**prm)
            r = Request(rid, prompt, params, _noop_callback, n_prompt=len(prompt), mu=2.0 * params.mirostat_tau)
            r.stream = core.TextStream(self.vocab, list(params.stop))
            if params.grammar:
                r.grammar = core.GrammarState(self._grammar(params.grammar), self.gvocab)
            return r
        if kind == "embed":
            return ("embed", {"texts": w[1], "pool": w[2], "done": threading.Event()})
        if kind == "mm":
            _, rid, prompt, images, prm = w
            return ("mm", rid, prompt, images, SamplingParams(**prm), _noop_callback, None)
        return w

    def _apply(self, item):
        if isinstance(item, tuple) and item[0] == "stop":
            self._stop = True
            return
        if isinstance(item, tuple) and item[0] == "mm":
            try:
                item = self._build_mm_request(*item[1:], embs=self._mm_embs.get(id(item)))
            except Exception as e:  # bad image / too long: report to the caller
                log.exception("multimodal request failed")
                item[5](Event(finished=True, finish_reason="error", error=f"image processing failed: {e}"))
                return
        if isinstance(item, tuple) and item[0] == "embed":
            self._run_embed_job(item[1])
            return
        if isinstance(item, tuple) and item[0] == "abort":
            r = self.requests.get(item[1])
            if r is not None:
                r.cancelled = True
                self._finish(r, "cancelled")
            return
        r: Request = item
        if len(r.prompt) >= self.ctx:
            r.callback(Event(finished=True, finish_reason="error", error="prompt exceeds context"))
            return
        if r.params.prompt_cache_path and self.tp.world == 1:
            n = self._pcache.ensure_loaded(self, r.params.prompt_cache_path)
            if n:
                log.info("prompt cache %s: %d tokens of KV restored", r.params.prompt_cache_path, n)
        # burst membership (_defer_decode): the requests of an idle -> busy transition, and then
        # each one that arrived within burst_gap_ms of the burst's previous member
        if not self.requests:
            r.burst = True
        elif self._burst_last > 0 and r.arrival - self._burst_last <= self.cfg.burst_gap_ms / 1e3:
            r.burst = True
        if r.burst:
            self._burst_last = max(self._burst_last, r.arrival)
        self.requests[r.id] = r
        max_new = r.params.max_tokens if r.params.max_tokens > 0 else self.ctx
        self.sched.add(r.id, r.prompt, max_new)
        self.metrics["requests"] += 1
        if self.tracer is not None:
            self.tracer.instant("arrival", r.arrival, cat="request", tid=1, id=r.id,
                                correlation_id=r.params.correlation_id, prompt_tokens=r.n_prompt)

    IMG_MARK = re.compile(r"\[img-(\d+)\]")

    def _build_mm_request(self, rid, prompt, images, params, callback, sink, embs=None) -> Request:
        """Tokenise around `[img-N]` markers (LocalAI's multimodal template) and splice the
        projected CLIP embeddings of image N in.  Image positions carry placeholder token ids
        above the vocabulary, derived from the image hash so prefix caching never matches two
        different images."""
        V = self.hp.n_vocab
        if embs is None:
            embs = self.clip.embed_images(list(images))
        parts = self.IMG_MARK.split(prompt)
        used = {int(parts[i]) for i in range(1, len(parts), 2)}
        seq: List = [("img", i) for i in range(len(embs)) if i not in used]  # unreferenced: up front
        for i, ptxt in enumerate(parts):
            if i % 2 == 0:
                if ptxt:
                    seq.append(("txt", ptxt))
            elif int(ptxt) < len(embs):
                seq.append(("img", int(ptxt)))
        toks: List[int] = []
        if self.tokenizer.add_bos and self.tokenizer.bos_id >= 0:
            toks.append(self.tokenizer.bos_id)
        rows, mm_pos = [], {}
        for kind, v in seq:
            if kind == "txt":
                toks += self.tokenize(v, add_bos=False)
                continue
            e = embs[v]
            data = images[v].encode() if isinstance(images[v], str) else bytes(images[v])
            base = V + (int(hashlib.sha1(data).hexdigest()[:8], 16) % (1 << 18)) * 4096
            for j in range(e.shape[0]):
                mm_pos[len(toks)] = len(rows) + j
                toks.append(base + (j % 4096))
            rows.append(e)
        if len(toks) >= self.ctx:
            raise ValueError(f"prompt with images is {len(toks)} tokens, context is {self.ctx}")
        r = Request(rid, toks, params, callback, n_prompt=len(toks), mu=2.0 * params.mirostat_tau)
        if self.cfg.record_tokens:
            r.out_ids = []
            r.out_logits = [] if self.cfg.record_logits else None
        r.stream = core.TextStream(self.vocab, list(params.stop))
        if params.grammar:
            r.grammar = core.GrammarState(self._grammar(params.grammar), self.gvocab)
        r.sink = sink
        if sink is not None:
            sink.set_prompt_tokens(r.n_prompt)
        r.mm_pos = mm_pos
        r.mm_emb = torch.cat(rows, 0).float() if rows else None
        return r

    def run_follower(self):
        """Non-leader tensor-parallel rank: mirror the leader's steps until it broadcasts stop."""
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        while not self._stop:
            try:
                self.step()
            except Exception as e:  # noqa: BLE001 - mirror the leader's loop: fail the step, keep serving
                log.exception("follower step failed")
                self._fail_all(str(e))
                if self._is_fatal(e):
                    self.healthy = False
                    self.fatal_error = str(e)
                    raise

    def _dev(self, a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            return t.pin_memory().to(self.device, non_blocking=True)
        return t

    def _run_prefill(self, plan):
        ids = plan["p_ids"]
        cu = plan["p_cu"]
        last = plan["p_last"]
        qlens = plan["p_qlen"]
        rows = [int(cu[i + 1]) - 1 for i in range(len(ids)) if last[i]]
        tokens = plan["p_tokens"]
        inj_idx = inj_rows = None
        if self.clip is not None and (tokens >= self.hp.n_vocab).any():
            tokens = tokens.copy()
            pos = plan["p_pos"]
            idx, chunks = [], []
            for i, sid in enumerate(ids):
                r = self.requests[int(sid)]
                a, b = int(cu[i]), int(cu[i + 1])
                if r.mm_pos is None:
                    continue
                sel = [(t, r.mm_pos[int(pos[t])]) for t in range(a, b) if int(pos[t]) in r.mm_pos]
                if sel:
                    idx += [t for t, _ in sel]
                    chunks.append(r.mm_emb[torch.tensor([k for _, k in sel], device=r.mm_emb.device)])
            tokens[tokens >= self.hp.n_vocab] = 0
            if idx:
                inj_idx = torch.tensor(idx, dtype=torch.long, device=self.device)
                inj_rows = torch.cat(chunks, 0).to(self.device, torch.float32)
        fb = ForwardBatch(
            tokens=self._dev(tokens), pos=self._dev(plan["p_pos"]), slots=self._dev(plan["p_slots"]),
            decode=False, block_tables=self._dev(plan["p_bt"]), cu_q=self._dev(cu), ctx_lens=self._dev(plan["p_ctx"]),
            tiles=ops.prefill_tiles(qlens.tolist(), self.device) if self.device.type == "cuda" else None,
            logits_idx=self._dev(np.array(rows, dtype=np.int64)) if rows else None,
            inject_idx=inj_idx, inject_rows=inj_rows)
        self.metrics["prompt_tokens"] += int(cu[-1])
        if not rows:
            self.model.forward(fb, self.kv)  # intermediate chunk: KV only
            return
        logits = self.model.forward(fb, self.kv)
        seqs = [int(ids[i]) for i in range(len(ids)) if last[i]]
        self._sample_and_emit(seqs, logits)

    # ------------------------------------------------------------------ decode
    PEN_CAP = 256  # longest penalty window (repeat_last_n) the captured decode graphs keep on the device

    def _needs_host_sampling(self, r: Request) -> bool:
        """Sampler features the captured decode graph cannot run: mirostat v1, grammars, more logit
        biases than its table holds, or a penalty window longer than PEN_CAP tokens.  Penalties
        over shorter windows run in the graph (penalty ring), so they keep multi-step decode."""
        return bool(r.params.grammar) or self._needs_host_sampler(r)

    def _needs_host_sampler(self, r: Request) -> bool:
        """Sampler features the in-graph sampler cannot run (grammars aside): those force the whole
        batch onto the host sampler; a grammar alone only needs its own rows fixed up."""
        p = r.params
        pen = p.repeat_penalty != 1.0 or p.frequency_penalty != 0.0 or p.presence_penalty != 0.0
        window = p.repeat_last_n if p.repeat_last_n >= 0 else self.ctx
        return ((pen and window > self.PEN_CAP) or p.mirostat == 1
                or len(p.logit_bias) + len(self.tokenizer.eog) > self.cfg.bias_capacity)

    k1_reasons: "collections.Counter"   # why a decode step ran one device step (diagnostics)

    def _defer_decode(self) -> bool:
        """EngineConfig.prefill_first_ms: True while the burst that woke an idle engine is being
        prefilled (the native scheduler then plans prefill only, when any prefill work is left).
        Only members of that burst (EngineConfig.burst_gap_ms) keep it going: under steady open-
        loop arrivals a later request never extends the deferral, so the burst's rows start
        decoding as soon as the burst itself is prefilled (profiles/r6_arrivals.md)."""
        ms = float(os.environ.get("LOCALAI_AMD_PREFILL_FIRST_MS", self.cfg.prefill_first_ms))
        if ms <= 0 or self.tp.world > 1:
            return False
        oldest = None
        pending = False
        for r in self.requests.values():
            if r.n_gen == 0:
                pending = pending or r.burst
            elif r.n_gen > 1 or not r.first_token_t:
                return False  # a decoding stream: keep it moving
            elif oldest is None or r.first_token_t < oldest:
                oldest = r.first_token_t
        if not pending or oldest is None:
            return False
        return (time.perf_counter() - oldest) * 1e3 < ms

    def _lookahead(self) -> int:
        """Decode steps to run on the device before coming back to the host."""
        K = self.cfg.decode_steps
        if K <= 1 or not (self.cfg.use_graphs and self.device.type == "cuda"):
            return 1
        s = self.sched
        why = self.k1_reasons
        # new prompts waiting or mid-prefill: they are admitted at the next host round trip, so a
        # run is capped at admit_budget_ms of device steps (one step at the old default of 0):
        # under steady open-loop arrivals some prompt is nearly always waiting, and one device step
        # per round trip left the batch host-bound (profiles/r6_arrivals.md)
        budget = float(os.environ.get("LOCALAI_AMD_ADMIT_BUDGET_MS", self.cfg.admit_budget_ms))
        k_admit = max(1, min(K, int(budget / max(self._step_ms, 0.5)))) if budget > 0 else 1
        if s.num_waiting > 0 and s.num_running < self.cfg.max_num_seqs:
            why["admit"] += 1
            if k_admit <= 1:
                return 1  # admit new prompts promptly
            K = k_admit
        if len(self.requests) >= self.cfg.wide_batch and s.num_waiting == 0:
            K = max(K, self.cfg.decode_steps_wide)
        rem_tok, rem_ctx = 1, K
        riders = cons = unsure = 0
        for r in self.requests.values():
            if self._needs_host_sampler(r):
                why["host_sampler"] += 1
                return 1  # a host-side sampler feature
            if r.n_gen == 0:
                if k_admit <= 1:
                    why["prefill"] += 1
                    return 1  # prefill in flight
                K = min(K, k_admit)
                continue
            if r.grammar is not None and not self._grammar_ready(r):
                if not self._grammar_slot_cached(r):
                    why["grammar_no_mask"] += 1
                    return 1  # a parse state without a device mask: the host walks it first
                cons += 1
                if not self._gready(r):
                    riders += 1
                elif self._ghit.get(r.params.grammar, 0.0) < self.GRAMMAR_RUN_HIT:
                    unsure += 1  # learned state, but its grammar often parks rows at new successors
            n = r.n_prompt + r.n_gen
            rem_ctx = min(rem_ctx, self.ctx - n)
            mt = r.params.max_tokens
            rem_tok = max(rem_tok, (mt - r.n_gen) if mt > 0 else K)
        if cons:
            # constrained rows ride along a mostly-plain batch: the plain rows keep a multi-step
            # run, each constrained row takes at least its first (masked) token per run and parks
            # at its first unknown transition (_grammar_run).  Rows in a fully learned state
            # (_gready) do not shorten the run; unlearned ones cap it at GRAMMAR_MIXED_K.  A batch
            # that is mostly constrained stays at one step per round trip (rows park after a few
            # tokens: a long run would mostly compute discarded positions) unless run-ahead is on
            if cons > self.GRAMMAR_MIXED_FRAC * len(self.requests) and (riders or unsure):
                why["grammar_majority"] += 1
                return 1
            if riders:
                K = min(K, self.GRAMMAR_MIXED_K)
        return max(1, min(K, rem_ctx, rem_tok))

    # device steps per run while unlearned constrained rows ride along ...
    GRAMMAR_MIXED_K = int(os.environ.get("LOCALAI_AMD_GRAMMAR_MIXED_K", "4"))
    # ... when they are at most this fraction of the batch (above it: one step per round trip
    # unless every constrained row is in a fully learned, predictable state)
    GRAMMAR_MIXED_FRAC = float(os.environ.get("LOCALAI_AMD_GRAMMAR_MIXED_FRAC", "0.125"))

    def _grammar_slot_cached(self, r) -> bool:
        s = self._gmask_cache.get((r.params.grammar, r.grammar.key()))
        return s is not None and s >= 0

    SPEC_MAX_BATCH = 8   # speculation pays while decode streams weights (small batches)
    SPEC_MAX_DRAFT = 16
    DRAFT_DEFAULT_K = 8  # draft-model tokens per verify when the request sets no n_draft

    def _spec_k(self) -> int:
        """Draft length for an n-gram speculative step (engine/speculative.py), or 0: every
        running request asked for it (n_draft) and is plain greedy, the batch is small, and no
        prompt is still prefilling."""
        if not self.requests or len(self.requests) > self.SPEC_MAX_BATCH or self.sched.num_waiting:
            return 0
        k = 0
        for r in self.requests.values():
            p = r.params
            nd = p.n_draft if p.n_draft > 0 else (self.DRAFT_DEFAULT_K if self.drafter is not None else 0)
            if (nd <= 0 or r.n_gen == 0 or r.spec_off or r.grammar is not None or p.mirostat
                    or not (p.temperature <= 0.0 or p.top_k == 1) or p.logit_bias or p.repeat_penalty != 1.0
                    or p.frequency_penalty != 0.0 or p.presence_penalty != 0.0):
                return 0
            k = max(k, min(nd, self.SPEC_MAX_DRAFT))
        return k

    def _run_spec(self, plan, k: int):
        """Verify n-gram drafts for every decoding sequence in ONE forward pass (the chunked-
        prefill path: last token + draft at positions L-1 .. L-1+k), keep the longest prefix the
        greedy argmax agrees with plus the model's own next token."""
        ids = [int(x) for x in plan["d_ids"]]
        reqs = [self.requests[i] for i in ids]
        bm = self.sched.blocks()
        toks, pos, slots, cu, ctxl, drafts, tabs = [], [], [], [0], [], [], []
        seqs = [self.sched.tokens(r.id) for r in reqs]
        kk = [min(k, max(0, min(self.ctx - len(s), (r.params.max_tokens - r.n_gen) if r.params.max_tokens > 0
                                else self.ctx) - 1)) for r, s in zip(reqs, seqs)]
        dm = self.drafter.draft([r.id for r in reqs], seqs, kk) if self.drafter is not None else None
        for i, r in enumerate(reqs):
            seq = seqs[i]
            L = len(seq)
            d = dm[i] if dm is not None else ngram_draft(seq, kk[i])
            for j, t in enumerate([seq[-1]] + d):
                toks.append(t)
                pos.append(L - 1 + j)
                slots.append(bm.slot(r.id, L - 1 + j))
            cu.append(len(toks))
            ctxl.append(L + len(d))
            drafts.append(d)
            tabs.append(bm.table(r.id))
        if not any(drafts):  # nothing to verify: the ordinary (graph) decode step is cheaper
            self._run_decode(plan, 1)
            return
        bt = np.zeros((len(reqs), max(len(t) for t in tabs)), dtype=np.int32)
        for i, t in enumerate(tabs):
            bt[i, :len(t)] = t
        qlens = [cu[i + 1] - cu[i] for i in range(len(reqs))]
        i32 = lambda a: self._dev(np.asarray(a, dtype=np.int32))  # noqa: E731
        fb = ForwardBatch(tokens=i32(toks), pos=i32(pos), slots=i32(slots), decode=False, block_tables=self._dev(bt),
                          cu_q=i32(cu), ctx_lens=i32(ctxl),
                          tiles=ops.prefill_tiles(qlens, self.device) if self.device.type == "cuda" else None)
        logits = self.model.forward(fb, self.kv)  # [T, V]: every position verifies one draft token
        ban = [i for i, r in enumerate(reqs) if r.params.ignore_eos]
        if ban and self._eog_list:
            rows = torch.cat([torch.arange(cu[i], cu[i + 1]) for i in ban]).to(logits.device)
            cols = torch.tensor(self._eog_list, device=logits.device)
            logits[rows.unsqueeze(1), cols.unsqueeze(0)] = -math.inf
        am = logits.argmax(-1).cpu().numpy()
        now = time.perf_counter()
        self.metrics["spec_steps"] += 1
        for i, r in enumerate(reqs):
            d, row = drafts[i], am[cu[i]:cu[i + 1]]
            j = 0
            while j < len(d) and int(row[j]) == d[j]:
                j += 1
            self.metrics["spec_drafted"] += len(d)
            self.metrics["spec_accepted"] += j
            r.spec_drafted += len(d)
            r.spec_accepted += j
            if r.spec_drafted >= 32 and r.spec_accepted < 0.15 * r.spec_drafted:
                r.spec_off = True  # low acceptance: a verify pass costs more than it saves
            out = d[:j] + [int(row[j])]
            for t in out:
                self._on_token(r, t, now, append=False)
                if r.done:
                    break
            if not r.done:
                self.sched.append_run(r.id, out)

    def _run_decode(self, plan, K: int = 1):
        ids = [int(x) for x in plan["d_ids"]]
        B = len(ids)
        tok, pos, slots, lens, bt = plan["d_tokens"], plan["d_pos"], plan["d_slots"], plan["d_lens"], plan["d_bt"]
        Bp = len(tok)
        if not (self.cfg.use_graphs and self.device.type == "cuda"):
            fb = ForwardBatch(tokens=self._dev(tok), pos=self._dev(pos), slots=self._dev(slots), decode=True,
                              block_tables=self._dev(bt), seq_lens=self._dev(lens), max_len=int(plan["d_maxlen"]))
            logits = self.model.forward(fb, self.kv)
            self._sample_and_emit(ids, logits[:B])
            return
        reqs = [self.requests[i] for i in ids]
        device_sampling = not any(self._needs_host_sampling(r) for r in reqs)
        if device_sampling and self._tp_greedy_ok(reqs):
            g = self._graphs_tpg.get(Bp)
            if g is None:
                g = self._graphs_tpg[Bp] = self._capture(Bp, tp_greedy=True)
            graph, st, _ = g
            self._upload_step_inputs(st, reqs, Bp, tok, pos, slots, lens, bt, True)
            for _ in range(K):
                graph.replay()
            hist = st["hist"][:K, :B].cpu().numpy()
            rec = st.get("rec")
            if rec is not None:   # record_logits (tests): this rank's columns -> full rows, off the graph
                rec = self.model.tp.all_gather_cols(rec)
            self._emit_run(reqs, hist, K, rec)
            return
        if device_sampling and self._tp_sample_ok(reqs):
            miro = any(r.params.mirostat == 2 for r in reqs)
            g = self._graphs_tps.get((Bp, miro))
            if g is None:
                g = self._graphs_tps[(Bp, miro)] = self._capture(Bp, tp_sample=miro)
            graph, st, _ = g
            self._upload_step_inputs(st, reqs, Bp, tok, pos, slots, lens, bt, True)
            for _ in range(K):
                graph.replay()
            hist = st["hist"][:K, :B].cpu().numpy()
            if miro:
                muh = st["mu"][:B].cpu().numpy()
                for j, r in enumerate(reqs):
                    r.mu = float(muh[j])
            rec = st.get("rec")
            if rec is not None:
                rec = self.model.tp.all_gather_cols(rec)
            self._emit_run(reqs, hist, K, rec)
            return
        g = self._graphs.get(Bp)
        if g is None:
            g = self._graphs[Bp] = self._capture(Bp)
        graph, st, logits = g
        if not device_sampling and not any(self._needs_host_sampler(r) for r in reqs):
            # grammar rows only: one step with the in-graph sampler for EVERY row (penalties, bias,
            # mirostat 2 included), then the grammar rows' samples are checked on the host and
            # the rejected ones resampled from this step's logits restricted to grammar-valid
            # tokens (_apply_grammar); unconstrained rows take the native emitter as in a run
            # rows whose parse state has a cached device mask are masked inside the graph, so
            # their sample is valid as drawn; the rest are checked and fixed up after the step
            V = logits.shape[1]
            if self._gexp_pend:
                self._gexpand_poll(V)
            gslot = np.full(B, -1, dtype=np.int32)
            done_rows, grows = [], []
            epoch0 = self._gepoch
            for j, r in enumerate(reqs):
                if r.grammar is not None and not r.done:
                    grows.append(j)
                    sl = self._grammar_mask_slot(r, V, self.device)
                    if sl is not None and sl >= 0:
                        gslot[j] = sl
                        # learn the state's transitions at once (inline, or on the helper
                        # thread for permissive states): a row in a fully learned state rides
                        # multi-step runs without parking (_gready), at any batch mix
                        self._gexpand(r.params.grammar, r.grammar, sl, V)
                    elif sl is not None:
                        done_rows.append(j)
            if K > 1 and (done_rows or any(gslot[j] < 0 for j in grows) or epoch0 != self._gepoch):
                self.k1_reasons["grammar_demoted"] += 1
                K = 1  # a constrained row without a device mask (or a slot reused meanwhile) cannot run ahead
            self._gtrans_flush()
            self._upload_step_inputs(st, reqs, Bp, tok, pos, slots, lens, bt, True, gslot)
            if K > 1:
                self._grammar_run(graph, st, reqs, grows, gslot, K, V)
                return
            graph.replay()
            toks = st["hist"][0, :B].cpu().numpy().copy()
            toks[done_rows] = -1
            toks = self._apply_grammar(reqs, logits[:B], st["prm_np"], toks)
            if any(r.params.mirostat == 2 for r in reqs):
                muh = st["mu"][:B].cpu().numpy()
                for j, r in enumerate(reqs):
                    r.mu = float(muh[j])
            plain = [j for j, r in enumerate(reqs) if r.grammar is None]
            if plain:
                self._emit_run([reqs[j] for j in plain], toks[plain][None, :].astype(np.int32), 1)
            now = time.perf_counter()
            epoch = self._gepoch
            learn = self.cfg.grammar_run_ahead
            for j, r in enumerate(reqs):
                if r.grammar is not None:
                    t = int(toks[j])
                    self._on_token(r, t, now)
                    s0 = int(gslot[j])
                    if learn and s0 >= 0 and t >= 0 and not r.done:
                        # learn the transition and score whether a multi-step run would have
                        # known it (the hit rate gates running constrained rows ahead)
                        s2 = self._grammar_mask_slot(r, V, self.device)
                        self._grammar_hit(r, (s0, t) in self._gdev)
                        if (s0, t) not in self._gtrans and epoch == self._gepoch:
                            self._gtrans_learn(s0, t, s2)
            return
        self._upload_step_inputs(st, reqs, Bp, tok, pos, slots, lens, bt, device_sampling)
        if not device_sampling:  # long penalty windows / mirostat v1 / bias overflow: host sampling
            graph.replay()
            self._sample_and_emit(ids, logits[:B])
            return
        if K > 1 and STREAM_STEPS and st.get("rec") is None and self.device.type == "cuda":
            self._run_streamed(graph, st, reqs, K)
        else:
            for _ in range(K):
                graph.replay()
            hist = st["hist"][:K, :B].cpu().numpy()  # the only sync per K steps
            self._emit_run(reqs, hist, K, st.get("rec"))
        if any(r.params.mirostat == 2 for r in reqs):
            muh = st["mu"][:B].cpu().numpy()
            for j, r in enumerate(reqs):
                r.mu = float(muh[j])

    _REASONS = {1: ("stop", True), 2: ("stop", False), 3: ("length", True), 4: ("abort", True)}

    def _run_streamed(self, graph, st, reqs: List[Request], K: int):
        """A K-step device run whose tokens reach the clients step by step.  Every replay is
        followed by an async copy of its token row into pinned host memory and an event; the host
        emits step k (native detokenise / stop strings / SSE writes) as soon as that event fires,
        while the device computes steps k+1.., so the run still costs one host round trip but
        streams at the step interval: p99 inter-token latency is about one decode step instead of
        K of them (profiles/r6_arrivals.md).  Request bookkeeping (scheduler run, finish) happens
        once at the end of the run, as in _emit_run."""
        B = len(reqs)
        hist = st["hist"]
        pin = st.get("hist_pin")
        if pin is None or pin.shape != hist.shape:
            pin = st["hist_pin"] = torch.empty(hist.shape, dtype=hist.dtype, pin_memory=True)
            st["hist_ev"] = [torch.cuda.Event() for _ in range(hist.shape[0])]
        evs = st["hist_ev"]
        for k in range(K):
            graph.replay()
            pin[k].copy_(hist[k], non_blocking=True)
            evs[k].record()
        pn = pin.numpy()
        stt = np.zeros((B, 5), dtype=np.int32)
        for j, r in enumerate(reqs):
            stt[j] = (r.n_gen, r.params.max_tokens, r.n_prompt, 1 if r.params.ignore_eos else 0, 0 if r.done else 1)
        streams, sinks = [r.stream for r in reqs], [r.sink for r in reqs]
        tot = np.zeros(B, dtype=np.int32)
        why = np.zeros(B, dtype=np.int32)
        for k in range(K):
            evs[k].synchronize()   # releases the GIL while the device works on step k
            n_acc, reason, texts = core.emit_run(np.ascontiguousarray(pn[k:k + 1, :B]), 1, B, streams, sinks, stt,
                                                 self._eog_list, self.ctx)
            n_acc = np.asarray(n_acc, dtype=np.int32)
            reason = np.asarray(reason, dtype=np.int32)
            first = np.nonzero((tot == 0) & (n_acc > 0))[0]
            if len(first):
                now = time.perf_counter()
                for j in first:
                    r = reqs[j]
                    if r.first_token_t == 0.0 and not r.done:
                        r.first_token_t = now
                        if self.tracer is not None:
                            self.tracer.instant("first_token", now, cat="request", tid=1, id=r.id,
                                                correlation_id=r.params.correlation_id)
            tot += n_acc
            stt[:, 0] += n_acc
            ended = (reason != 0) & (why == 0)
            why[ended] = reason[ended]
            stt[reason != 0, 4] = 0
            for j, t in enumerate(texts):
                if t and not reqs[j].done:
                    reqs[j].callback(Event(text=t, token=-1))
            if not stt[:, 4].any():
                break   # every row has finished: the remaining steps carry nothing to emit
        for j, r in enumerate(reqs):
            n = int(tot[j])
            if r.done or n == 0:
                continue
            r.n_gen += n
            self.metrics["gen_tokens"] += n
            if r.out_ids is not None:
                r.out_ids.extend(int(t) for t in pn[:n, j])
            rs = int(why[j])
            if rs == 0:
                self.sched.append_run(r.id, pn[:n, j].tolist())
            else:
                why_s, flush = self._REASONS[rs]
                self._finish(r, why_s, flush=flush)
        if not evs[K - 1].query():
            evs[K - 1].synchronize()   # an early break: the run's last steps still finish first

    def _grammar_run(self, graph, st, reqs, grows, gslot, K: int, V: int):
        """K device steps with grammar rows masked in the graph: each row's mask slot follows the
        learned transition table (grammar_advance).  On the host, a constrained row keeps its
        tokens up to the first transition the table did not know yet -- that token was sampled
        under a valid mask, later ones were not -- and the transition is learned for the next
        runs; the row's dropped positions are recomputed next run (as with rejected drafts)."""
        B = len(reqs)
        for _ in range(K):
            graph.replay()
        hist = st["hist"][:K, :B].cpu().numpy()
        if any(r.params.mirostat == 2 for r in reqs):
            muh = st["mu"][:B].cpu().numpy()
            for j, r in enumerate(reqs):
                if r.grammar is None:
                    r.mu = float(muh[j])
        gset = set(grows)
        plain = [j for j in range(B) if j not in gset]
        if plain:
            self._emit_run([reqs[j] for j in plain], np.ascontiguousarray(hist[:, plain]), K)
        now = time.perf_counter()
        epoch = self._gepoch
        self.metrics["grammar_runs"] += 1
        self.metrics["grammar_run_rows"] += len(grows)
        gdev, gtrans, cache, skey = self._gdev, self._gtrans, self._gmask_cache, self._gslot_key
        for j in grows:
            r, s = reqs[j], int(gslot[j])
            kept = []
            followed = missed = False
            for i in range(K):
                t = int(hist[i, j])
                self._on_token(r, t, now, append=False)
                self.metrics["grammar_run_tokens"] += 1
                if r.done:
                    break
                kept.append(t)
                hit = (s, t) in gdev
                self._grammar_hit(r, hit)
                if not hit:
                    # the device parked this row after token t: learn the transition from the real
                    # state (not after a slot reuse: s may name another state)
                    s2 = self._grammar_mask_slot(r, V, self.device)
                    if (s, t) not in gtrans and epoch == self._gepoch:
                        self._gtrans_learn(s, t, s2)
                    missed = True
                    break
                # a learned transition within this epoch names the state's slot exactly (the table
                # was written from the real successor), so the host follows it without hashing the
                # parse state per token; the slot's mask stays recently used
                s = gtrans[(s, t)]
                followed = True
                k = skey.get(s)
                if k is not None and k in cache:
                    cache.move_to_end(k)
            if followed and not missed and not r.done and epoch == self._gepoch:
                self._grammar_verify(r, s)   # s and r.grammar both stand after the run's last token
            if kept and not r.done:
                # the device already wrote the KV of every kept token but the last (fed by the
                # next step): hand them over as a run, like the plain rows' _emit_run -- appending
                # them one by one marked them all uncomputed, and the row spent every other run
                # re-prefilling its own positions instead of decoding
                self.sched.append_run(r.id, kept)

    def _emit_run(self, reqs: List[Request], hist: np.ndarray, K: int, rec: Optional[torch.Tensor] = None):
        """Hand a [K, B] block of device-sampled tokens to the native emitter (detokenise, stop
        strings, EOS / length limits, SSE writes), then update Python-side request state once
        per row."""
        B = len(reqs)
        st = np.zeros((B, 5), dtype=np.int32)
        for j, r in enumerate(reqs):
            st[j] = (r.n_gen, r.params.max_tokens, r.n_prompt, 1 if r.params.ignore_eos else 0, 0 if r.done else 1)
        n_acc, reason, texts = core.emit_run(hist, K, B, [r.stream for r in reqs], [r.sink for r in reqs], st,
                                             self._eog_list, self.ctx)
        now = time.perf_counter()
        for j, r in enumerate(reqs):
            n = int(n_acc[j])
            if r.done or n == 0:
                continue
            if r.first_token_t == 0.0:
                r.first_token_t = now
                if self.tracer is not None:
                    self.tracer.instant("first_token", now, cat="request", tid=1, id=r.id,
                                        correlation_id=r.params.correlation_id)
            r.n_gen += n
            self.metrics["gen_tokens"] += n
            if r.out_ids is not None:
                r.out_ids.extend(int(t) for t in hist[:n, j])
                if r.out_logits is not None and rec is not None:
                    r.out_logits.extend(rec[k, j].clone() for k in range(n))
            if texts[j]:
                r.callback(Event(text=texts[j], token=-1))
            rs = int(reason[j])
            if rs == 0:
                self.sched.append_run(r.id, hist[:n, j].tolist())
            else:
                why, flush = self._REASONS[rs]
                self._finish(r, why, flush=flush)

    def _upload_step_inputs(self, st, reqs, Bp, tok, pos, slots, lens, bt, device_sampling: bool,
                            gslot: Optional[np.ndarray] = None):
        B = len(reqs)
        h = st["host"]  # one pinned staging block -> one H2D copy per run
        h["gslot"].fill_(-1)
        if gslot is not None:
            h["gslot"][:len(gslot)] = torch.from_numpy(gslot)
        h["tokens"][:] = torch.from_numpy(tok)
        h["pos"][:] = torch.from_numpy(pos)
        h["slots"][:] = torch.from_numpy(slots)
        h["lens"][:] = torch.from_numpy(lens)
        nb = bt.shape[1]
        h["bt"][:, :nb] = torch.from_numpy(bt)
        h["step"][0] = 0
        # the per-request sampling inputs (params, logit bias, penalty windows) depend only on the
        # batch's requests: an unchanged batch (the common multi-run case) refreshes just the
        # per-row counters instead of rebuilding ~256 rows in Python between two graph runs
        key = (device_sampling, tuple(r.id for r in reqs))
        same = st.get("in_key") == key
        st["in_key"] = key
        n_bias = st.get("in_nbias", 0) if same else 0
        if device_sampling:
            prm = st["prm_np"]
            if same:
                prm["counter"][:B] = [r.n_gen for r in reqs]
            else:
                prm[:] = 0  # padding rows: greedy
                for j, r in enumerate(reqs):
                    p = r.params
                    prm[j] = (p.temperature, p.top_p, p.min_p, p.typical_p, p.tfs_z, p.mirostat_tau, p.mirostat_eta,
                              p.top_k, 2 if p.mirostat == 2 else 0, 0, p.seed & 0xFFFFFFFFFFFFFFFF, r.n_gen)
            h["prm"][:] = torch.from_numpy(prm.view(np.uint8))
            if not same:
                rows, cols, vals = st["bias_np"]
                lo, hi = 0, self.hp.n_vocab
                if "tp_cols" in st:   # distributed-argmax graph: this rank's columns only
                    lo, hi = st["tp_cols"][0], st["tp_cols"][0] + st["tp_cols"][1]
                for j, r in enumerate(reqs):
                    ent = list(r.params.logit_bias.items())
                    if r.params.ignore_eos:
                        ent += [(t, -math.inf) for t in self.tokenizer.eog]
                    for t, b in ent:
                        if lo <= t < hi and n_bias < len(rows):
                            rows[n_bias], cols[n_bias], vals[n_bias] = j, t - lo, b
                            n_bias += 1
                h["bias_rows"][:] = torch.from_numpy(rows)
                h["bias_cols"][:] = torch.from_numpy(cols)
                h["bias_vals"][:] = torch.from_numpy(vals)
                st["in_nbias"] = n_bias
                st["in_miro"] = any(r.params.mirostat for r in reqs)
                st["in_pen"] = any(r.params.repeat_penalty != 1.0 or r.params.frequency_penalty != 0.0
                                   or r.params.presence_penalty != 0.0 for r in reqs)
            if st["in_miro"] or not same:
                mu = np.zeros(Bp, dtype=np.float32)
                for j, r in enumerate(reqs):
                    mu[j] = r.mu
                h["mu"][:] = torch.from_numpy(mu)
        if not (same and not (device_sampling and st.get("in_pen"))):
            # penalty windows: neutral unless a device-sampled row asks for penalties (rebuilt
            # every run while any row uses them: the windows slide)
            pen = np.zeros((Bp, 3), dtype=np.float32)
            pen[:, 0] = 1.0
            pcap = np.zeros(Bp, dtype=np.int32)
            pcnt = np.zeros(Bp, dtype=np.int32)
            pnl = np.ones(Bp, dtype=np.int32)
            if device_sampling:
                for j, r in enumerate(reqs):
                    p = r.params
                    if p.repeat_penalty == 1.0 and p.frequency_penalty == 0.0 and p.presence_penalty == 0.0:
                        continue
                    ln = p.repeat_last_n if p.repeat_last_n >= 0 else self.ctx
                    if ln <= 0:
                        continue
                    toks = self.sched.tokens(r.id)[-ln:]
                    pen[j] = (p.repeat_penalty, p.frequency_penalty, p.presence_penalty)
                    pcap[j] = ln
                    pcnt[j] = len(toks)
                    pnl[j] = 1 if p.penalize_nl else 0
                    if toks:
                        h["phist"][j, :len(toks)] = torch.tensor(toks, dtype=torch.int32)
            h["pen"][:] = torch.from_numpy(pen)
            h["pcap"][:] = torch.from_numpy(pcap)
            h["pcnt"][:] = torch.from_numpy(pcnt)
            h["phl"][:] = torch.from_numpy(np.minimum(pcnt, pcap))
            h["pnl"][:] = torch.from_numpy(pnl)
        h["bias_n"][0] = n_bias
        st["dev_block"].copy_(st["host_block"], non_blocking=True)

    TP_GREEDY = os.environ.get("LOCALAI_AMD_TP_GREEDY", "1") == "1"

    def _tp_greedy_ok(self, reqs) -> bool:
        """Tensor parallelism and every row plain greedy (temperature <= 0, no penalties, no
        mirostat, no grammar; logit bias and ignore_eos are fine): the batch can run the
        distributed-argmax graph.  Every rank decides alike (replicated request state)."""
        if self.tp.world < 2 or not self.TP_GREEDY:
            return False
        for r in reqs:
            p = r.params
            if (p.temperature > 0 or p.mirostat or r.grammar is not None or p.repeat_penalty != 1.0
                    or p.frequency_penalty != 0.0 or p.presence_penalty != 0.0):
                return False
        return True

    TP_SAMPLE = os.environ.get("LOCALAI_AMD_TP_SAMPLE", "1") == "1"

    def _tp_sample_ok(self, reqs) -> bool:
        """Tensor parallelism and every row within the distributed sampler's reach
        (TPInfo.sample_cols): greedy, mirostat 2, or the standard chain with 1 <= top_k <=
        TP_SAMPLE_C (tail-free / typical / top-p / min-p / temperature after it); penalties and
        logit bias are applied to each rank's own columns.  LocalAI's defaults (temperature 0.9,
        top-k 40, top-p 0.95, mirostat 2; core/config/backend_config.go:284-289) qualify.  Rows
        outside (top_k 0 without mirostat, grammars, mirostat 1) keep the full-row gather."""
        if self.tp.world < 2 or not self.TP_SAMPLE:
            return False
        for r in reqs:
            p = r.params
            if r.grammar is not None or p.mirostat == 1:
                return False
            if p.temperature > 0 and p.mirostat != 2 and not (1 <= p.top_k <= ops.TP_SAMPLE_C):
                return False
        return True

    def _capture(self, Bp: int, tp_greedy: bool = False, tp_sample: Optional[bool] = None):
        """One hipGraph per padded batch size: forward + logit bias + sampler + advance.
        tp_greedy: this rank's vocabulary columns only, logit bias on them, and the exact
        distributed argmax (TPInfo.argmax_cols) as the sampler.  tp_sample (True: with the
        mirostat-2 phases): this rank's columns, bias + penalties on them, and the distributed
        sampler (TPInfo.sample_cols)."""
        tp_local = tp_greedy or tp_sample is not None
        dev = self.device
        MB = self.max_blocks
        cap = max(1, Bp * self.cfg.bias_capacity)
        K = max(1, self.cfg.decode_steps, self.cfg.decode_steps_wide)
        # all per-run inputs live in one int32 block (uploaded with a single copy)
        prm_words = Bp * ops.SAMPLE_ROW_DTYPE.itemsize // 4
        PL = self.PEN_CAP
        layout = [("tokens", Bp), ("pos", Bp), ("slots", Bp), ("lens", Bp), ("bt", Bp * MB), ("step", 1),
                  ("prm", prm_words), ("bias_rows", cap), ("bias_cols", cap), ("bias_vals", cap), ("bias_n", 1),
                  ("mu", Bp), ("phist", Bp * PL), ("pcnt", Bp), ("phl", Bp), ("pcap", Bp), ("pen", Bp * 3),
                  ("pnl", Bp), ("gslot", Bp)]
        total = sum(n for _, n in layout)
        host_block = torch.zeros(total, dtype=torch.int32).pin_memory()
        dev_block = torch.zeros(total, dtype=torch.int32, device=dev)
        host, st, o = {}, {}, 0
        for name, n in layout:
            hv, dv = host_block[o:o + n], dev_block[o:o + n]
            if name == "bt":
                hv, dv = hv.view(Bp, MB), dv.view(Bp, MB)
            elif name == "phist":
                hv, dv = hv.view(Bp, PL), dv.view(Bp, PL)
            elif name == "pen":
                hv, dv = hv.view(torch.float32).view(Bp, 3), dv.view(torch.float32).view(Bp, 3)
            elif name in ("bias_vals", "mu"):
                hv, dv = hv.view(torch.float32), dv.view(torch.float32)
            elif name == "prm":
                hv, dv = hv.view(torch.uint8), dv.view(torch.uint8)
            host[name], st[name] = hv, dv
            o += n
        st["slots"].fill_(-1)
        st["lens"].fill_(1)
        st["gslot"].fill_(-1)
        st["host"], st["host_block"], st["dev_block"] = host, host_block, dev_block

        st["prm_np"] = np.zeros(Bp, dtype=ops.SAMPLE_ROW_DTYPE)
        st["bias_np"] = (np.zeros(cap, np.int32), np.zeros(cap, np.int32), np.zeros(cap, np.float32))
        st["next"] = torch.zeros(Bp, dtype=torch.int32, device=dev)
        st["hist"] = torch.zeros(K, Bp, dtype=torch.int32, device=dev)
        fb = ForwardBatch(tokens=st["tokens"], pos=st["pos"], slots=st["slots"], decode=True, block_tables=st["bt"],
                          seq_lens=st["lens"], max_len=self.ctx)
        ws = ops.decode_workspace(Bp, self.model.Hq, self.model.Hkv, self.model.Dh, self.ctx, dev,
                                  self.cfg.block_size)
        bs = self.cfg.block_size
        if tp_local:
            vl = self.model.vocab_local
            st["tp_cols"] = (self.model.tp.rank * vl, vl)   # bias entries are translated to these columns
        if tp_sample is not None:
            st["tpsw"] = self.model.tp.sample_workspace(Bp, dev)
        if self.cfg.record_logits:
            st["rec"] = torch.zeros(K, Bp, self.model.vocab_local if tp_local else self.model.hp.n_vocab,
                                    dtype=torch.float32, device=dev)

        def body_tpg():
            lg = self.model.forward(fb, self.kv, attn_workspace=ws, local_logits=True)
            if "rec" in st:
                st["rec"].index_copy_(0, st["step"][:1].long(), lg.float().unsqueeze(0))
            ops.logit_bias(lg, st["bias_rows"], st["bias_cols"], st["bias_vals"], st["bias_n"])
            st["next"].copy_(self.model.tp.argmax_cols(lg))
            ops.decode_advance(st["next"], st["tokens"], st["pos"], st["lens"], st["slots"], st["bt"], bs,
                               st["hist"], st["step"], st["prm"])
            return lg

        def body_tps():
            lg = self.model.forward(fb, self.kv, attn_workspace=ws, local_logits=True)
            if "rec" in st:
                st["rec"].index_copy_(0, st["step"][:1].long(), lg.float().unsqueeze(0))
            ops.logit_bias(lg, st["bias_rows"], st["bias_cols"], st["bias_vals"], st["bias_n"])
            ops.penalties(lg, st["phist"], st["phl"], st["pen"], self.tokenizer.nl_id, st["pnl"],
                          col0=st["tp_cols"][0])
            self.model.tp.sample_cols(lg, st["prm_np"], st["prm"], st["mu"], st["next"], st["tpsw"],
                                      mirostat=bool(tp_sample))
            ops.penalty_push(st["next"], st["phist"], st["pcnt"], st["phl"], st["pcap"])
            ops.decode_advance(st["next"], st["tokens"], st["pos"], st["lens"], st["slots"], st["bt"], bs,
                               st["hist"], st["step"], st["prm"])
            return lg

        def body():
            lg = self.model.forward(fb, self.kv, attn_workspace=ws)
            if "rec" in st:
                st["rec"].index_copy_(0, st["step"][:1].long(), lg.float().unsqueeze(0))
            ops.logit_bias(lg, st["bias_rows"], st["bias_cols"], st["bias_vals"], st["bias_n"])
            # repeat / frequency / presence penalties over each row's last-n window, kept on the
            # device across the run's steps (rows without penalties return at once)
            ops.penalties(lg, st["phist"], st["phl"], st["pen"], self.tokenizer.nl_id, st["pnl"])
            # grammar rows whose parse state has a cached mask sample only grammar-valid tokens
            ops.grammar_mask(lg, st["gslot"], self._gmask_pool_for(lg.shape[1], dev))
            ops.sample(lg, st["prm_np"], mu=st["mu"], params_dev=st["prm"], out=st["next"])
            ops.grammar_advance(st["next"], st["gslot"], self._gnext)
            ops.penalty_push(st["next"], st["phist"], st["pcnt"], st["phl"], st["pcap"])
            ops.decode_advance(st["next"], st["tokens"], st["pos"], st["lens"], st["slots"], st["bt"], bs,
                               st["hist"], st["step"], st["prm"])
            return lg

        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        if tp_greedy:
            body = body_tpg  # noqa: F811
        elif tp_sample is not None:
            body = body_tps  # noqa: F811
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up allocator / kernels outside the graph
                body()
                st["slots"].fill_(-1)
                st["pos"].zero_()
                st["lens"].fill_(1)
                st["step"].zero_()
        torch.cuda.current_stream(dev).wait_stream(s)
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self._graph_pool):
            logits = body()
        st["ws"] = ws
        return graph, st, logits

    def warmup(self, batch_sizes: Optional[Sequence[int]] = None):
        """Capture decode graphs ahead of serving (the reference's LoadToMemory eager path)."""
        if not (self.cfg.use_graphs and self.device.type == "cuda"):
            return
        tuning = self.cfg.blas_tune and ops.blas_tuning_start()
        try:
            for b in (batch_sizes or self.sched.buckets()):
                if b not in self._graphs:
                    self._graphs[b] = self._capture(b)
            if tuning and batch_sizes is None:
                self._tune_prefill()
        finally:
            if tuning:
                ops.blas_tuning_stop()
        torch.cuda.synchronize(self.device)

    def _tune_prefill(self):
        """Tune the library GEMMs of a FULL prefill chunk (M = max_batched_tokens), the shape a
        burst of prompts runs at: one throw-away step of equal prompts that pack the chunk
        exactly.  Measured on Llama-3-8B at M=8192: qkv 327->265 us, o 214->182 us, gate_up
        1313->1245 us, down 608->595 us per layer (-7% prefill GEMM time) for ~25 s of tuning.
        Partial chunks keep the library's default heuristic (tuning them inline would stall
        serving)."""
        if (self.tp.world > 1 or self._thread is not None or self.requests
                or os.environ.get("LOCALAI_AMD_PREFILL_TUNE", "1") == "0"):
            return
        n_tok = self.cfg.max_batched_tokens
        plen = next((p for p in range(min(512, self.ctx - 2), 15, -1) if n_tok % p == 0), 0)
        nreq = n_tok // plen if plen else 0
        if n_tok < 1024 or not plen or nreq > self.cfg.max_num_seqs:
            return
        rng = np.random.default_rng(0x7E57)
        left = [nreq]
        saved = dict(self.metrics)

        def cb(ev: Event):
            if ev.finished:
                left[0] -= 1

        for _ in range(nreq):  # distinct random prompts: no prefix-cache hit shortens the chunk
            toks = rng.integers(0, self.hp.n_vocab, size=plen).tolist()
            self.add_request(toks, SamplingParams(max_tokens=1, temperature=0.0), cb)
        while left[0] > 0:
            self.step()
        self.metrics = saved  # warm-up traffic is not served traffic

    # ------------------------------------------------------------------ sampling + output
    def _sample_and_emit(self, seq_ids: List[int], logits: torch.Tensor):
        raw = logits  # before bias / penalties (EngineConfig.record_logits)
        n = len(seq_ids)
        reqs = [self.requests[i] for i in seq_ids]
        prm = np.zeros(n, dtype=ops.SAMPLE_ROW_DTYPE)
        any_pen = any_bias = any_miro = False
        for j, r in enumerate(reqs):
            p = r.params
            prm[j] = (p.temperature, p.top_p, p.min_p, p.typical_p, p.tfs_z, p.mirostat_tau, p.mirostat_eta,
                      p.top_k, 2 if p.mirostat == 2 else (1 if p.mirostat == 1 else 0), 0,
                      p.seed & 0xFFFFFFFFFFFFFFFF, r.n_gen)
            if p.repeat_penalty != 1.0 or p.frequency_penalty != 0.0 or p.presence_penalty != 0.0:
                any_pen = True
            if p.logit_bias:
                any_bias = True
            if p.mirostat:
                any_miro = True
            if p.ignore_eos:
                any_bias = True
        if any_bias or any_pen:
            logits = logits.clone() if logits.is_cuda else logits
        if any_bias:
            rows, cols, vals = [], [], []
            for j, r in enumerate(reqs):
                for t, b in r.params.logit_bias.items():
                    if 0 <= t < logits.shape[1]:
                        rows.append(j); cols.append(t); vals.append(b)
                if r.params.ignore_eos:
                    for t in self.tokenizer.eog:
                        rows.append(j); cols.append(t); vals.append(-math.inf)
            if rows:
                ri = torch.tensor(rows, device=logits.device)
                ci = torch.tensor(cols, device=logits.device)
                logits[ri, ci] += torch.tensor(vals, device=logits.device, dtype=logits.dtype)
        if any_pen:
            L = max(1, max(max(0, r.params.repeat_last_n) if r.params.repeat_last_n >= 0 else self.ctx for r in reqs))
            hist = np.full((n, L), -1, dtype=np.int32)
            hl = np.zeros(n, dtype=np.int32)
            pen = np.zeros((n, 3), dtype=np.float32)
            for j, r in enumerate(reqs):
                p = r.params
                ln = p.repeat_last_n if p.repeat_last_n >= 0 else self.ctx
                toks = self.sched.tokens(r.id)[-ln:] if ln > 0 else []
                hist[j, :len(toks)] = toks
                hl[j] = len(toks)
                pen[j] = (p.repeat_penalty, p.frequency_penalty, p.presence_penalty)
            pnl = np.array([1 if r.params.penalize_nl else 0 for r in reqs], dtype=np.int32)
            ops.penalties(logits, self._dev(hist), self._dev(hl), self._dev(pen), self.tokenizer.nl_id,
                          self._dev(pnl))
        mu = None
        if any_miro:
            mu = torch.tensor([r.mu for r in reqs], dtype=torch.float32, device=logits.device)
        if any(r.params.mirostat == 1 for r in reqs):
            toks = self._sample_host_mirostat1(logits, reqs)
        else:
            toks = ops.sample(logits, prm, mu=mu).cpu().numpy()
        if any(r.grammar is not None for r in reqs):
            toks = self._apply_grammar(reqs, logits, prm, toks)
        if mu is not None:
            muh = mu.cpu().numpy()
            for j, r in enumerate(reqs):
                r.mu = float(muh[j])
        now = time.perf_counter()
        for j, r in enumerate(reqs):
            if r.out_logits is not None and not r.done:
                r.out_logits.append(raw[j].float().clone())
            self._on_token(r, int(toks[j]), now)

    GRAMMAR_TOPN = 1024
    GRAMMAR_MASK_BUDGET = 1500   # trie edges a first-sight whole-vocabulary mask walk may feed (~0.5 ms)
    GRAMMAR_MASK_SLOTS = 512     # device-resident masks (512 x 128 K vocabulary = 64 MB)

    def _gmask_pool_for(self, V: int, dev) -> torch.Tensor:
        """The device mask pool ([slots, V] bool); allocated once before the first graph capture
        (the captured grammar_mask kernel holds its address) and never reallocated on the GPU."""
        pool = self._gmask_pool
        if pool is None or pool.shape[1] != V or pool.device != torch.device(dev):
            if pool is not None and pool.is_cuda and self._graphs:
                raise RuntimeError("grammar mask pool shape changed after graph capture")
            pool = self._gmask_pool = torch.zeros(self.GRAMMAR_MASK_SLOTS, V, dtype=torch.bool, device=dev)
            # learned parse-state transitions for multi-step runs: next[slot, token] (-2 unknown)
            self._gnext = torch.full((self.GRAMMAR_MASK_SLOTS, V), -2, dtype=torch.int16, device=dev)
            self._gmask_free = list(range(self.GRAMMAR_MASK_SLOTS))
            self._gmask_cache.clear()
            self._gslot_key.clear()
            self._gtrans.clear()
            self._gtrans_in.clear()
            self._gpend.clear()
            self._gdev.clear()
            self._gexpanded.clear()
            self._gexp_pend.clear()
            self._gmask_np.clear()
        return pool

    def _gslot_release(self, slot: int):
        """A pool slot is being reused: forget every learned transition into or out of it."""
        self._gmask_free.append(slot)
        self._gepoch += 1
        self._gnext[slot].fill_(-2)
        self._gexpanded.discard(slot)
        self._gexp_pend.pop(slot, None)
        self._gmask_np.pop(slot, None)
        for st_t in self._gtrans_in.pop(slot, ()):
            self._gtrans.pop(st_t, None)
            if st_t in self._gdev:
                self._gdev.discard(st_t)
                self._gnext[st_t[0], st_t[1]] = -2
        self._gpend = [e for e in self._gpend if e[0] != slot and e[2] != slot]
        for k in [k for k in self._gtrans if k[0] == slot]:
            v = self._gtrans.pop(k)
            self._gdev.discard(k)
            if v is not None and v >= 0:
                self._gtrans_in.get(v, set()).discard(k)

    def _grammar_verify(self, r, s: int):
        """Once per row and run: the slot the host reached by following learned transitions must
        name the row's real parse state (one state hash per run, not per token).  A mismatch means
        a state key mapped two parse states with different successors; the slot is evicted (every
        transition into or out of it is forgotten) so later runs re-learn from real states."""
        key = (r.params.grammar, r.grammar.key())
        if self._gslot_key.get(s) == key:
            return
        self.metrics["grammar_drift"] += 1
        log.warning("grammar run-ahead: learned slot %d does not name the row's parse state; evicting it", s)
        old = self._gslot_key.get(s)
        if old is not None and self._gmask_cache.get(old) == s:
            del self._gmask_cache[old]
            self._gslot_key.pop(s, None)
            self._gslot_release(s)

    def _gtrans_learn(self, s: int, t: int, s2):
        """Record the transition (slot s, token t) -> s2 (a slot, -1 complete, None unmasked);
        only slot targets are written to the device table (the others keep the row on the host)."""
        self._gtrans[(s, t)] = s2
        if s2 is not None and s2 >= 0:
            self._gtrans_in.setdefault(s2, set()).add((s, t))
            self._gpend.append((s, t, s2))

    def _gtrans_flush(self):
        if self._gpend:
            self._gdev.update((a, b) for a, b, _ in self._gpend)
            a = torch.tensor(self._gpend, dtype=torch.int64)
            self._gnext[a[:, 0].to(self._gnext.device), a[:, 1].to(self._gnext.device)] = \
                a[:, 2].to(torch.int16).to(self._gnext.device)
            self._gpend.clear()

    GRAMMAR_RUN_HIT = 0.8   # learned-transition hit rate above which constrained rows run ahead

    def _grammar_hit(self, r, hit: bool):
        g = r.params.grammar
        self._ghit[g] = 0.95 * self._ghit.get(g, 0.0) + (0.05 if hit else 0.0)

    GRAMMAR_EXPAND_MAX = 20000   # allowed tokens up to which a state's transitions are learned inline
    # permissive states (`[a-z ]+`, the inside of a JSON string: 10^4-10^5 allowed tokens) are
    # expanded too, their successor keys computed on the helper thread (the native pass releases
    # the GIL) and applied in bulk when ready; until then the row learns per token as before
    GRAMMAR_EXPAND_BG = os.environ.get("LOCALAI_AMD_GRAMMAR_EXPAND_BG", "1") == "1"

    def _gexpand(self, gtext: str, gs, s: int, V: int):
        """Learn every transition out of slot s at once: the key of the state after each allowed
        token (one native pass), one mask per distinct successor.  A state like `[a-z ]+`
        (self-loop) or an enum position of a JSON schema is then fully known to the device
        table, so constrained rows do not park there (_gready: such a row is no rider)."""
        if s in self._gexpanded or s in self._gexp_pend:
            return
        m = self._gmask_np.get(s)
        if m is None:
            self._gexpanded.add(s)
            return
        toks = np.nonzero(m)[0].astype(np.int32)
        if len(toks) == 0:
            self._gexpanded.add(s)
            return
        if len(toks) > self.GRAMMAR_EXPAND_MAX:
            if self.GRAMMAR_EXPAND_BG and self.tp.world == 1:
                if self._gmask_bg is None:
                    import concurrent.futures
                    self._gmask_bg = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="gmask")
                g = gs.clone()
                self._gexp_pend[s] = (self._gmask_bg.submit(g.next_keys, toks), toks, gtext, g, self._gepoch)
            else:
                self._gexpanded.add(s)   # tensor-parallel ranks: per-token learning (same on every rank)
            return
        self._gexpand_apply(s, toks, gs.next_keys(toks), gtext, gs, self._gepoch, V)

    def _gexpand_poll(self, V: int):
        """Apply the background expansions that finished (called once per constrained step)."""
        for s in [s for s, e in self._gexp_pend.items() if e[0].done()]:
            fut, toks, gtext, gs, epoch = self._gexp_pend.pop(s)
            if epoch == self._gepoch:
                self._gexpand_apply(s, toks, fut.result(), gtext, gs, epoch, V)

    def _gexpand_apply(self, s: int, toks: np.ndarray, keys: np.ndarray, gtext: str, gs, epoch: int, V: int):
        """Every transition out of slot s, grouped by successor key: one successor slot per key,
        then the (s, t) -> s2 entries in bulk (host tables + one device index_put per key)."""
        uk, inv = np.unique(keys, return_inverse=True)
        for i, k in enumerate(uk.tolist()):
            if not k:
                continue
            ts = toks[inv == i]
            if (gtext, k) in self._gmask_cache:
                s2 = self._gmask_cache[(gtext, k)]
            else:
                g2 = gs.clone()
                if not g2.accept(int(ts[0])):
                    continue
                s2 = self._state_slot(gtext, g2, V, self.device, key=k)
            if epoch != self._gepoch:   # a slot was reused meanwhile: s may name another state
                return
            pairs = [(s, t) for t in ts.tolist()]
            self._gtrans.update(dict.fromkeys(pairs, s2))
            if s2 is not None and s2 >= 0:
                self._gtrans_in.setdefault(s2, set()).update(pairs)
                self._gdev.update(pairs)
                self._gnext[s, torch.from_numpy(ts.astype(np.int64)).to(self._gnext.device)] = s2
        self._gexpanded.add(s)

    def _gready(self, r) -> bool:
        """r's parse state has a device mask whose every transition is learned: it cannot park in
        this state, so it rides a multi-step run without shortening it (it may still park at a
        successor state it has not seen before)."""
        s = self._gmask_cache.get((r.params.grammar, r.grammar.key()))
        return s is not None and s >= 0 and s in self._gexpanded

    def _grammar_ready(self, r) -> bool:
        """r can run ahead inside a multi-step graph run: its parse state has a device mask and
        the transitions its grammar produces are mostly learned already (otherwise each row would
        park after about one token and waste the rest of the run)."""
        if not self.cfg.grammar_run_ahead or self._ghit.get(r.params.grammar, 0.0) < self.GRAMMAR_RUN_HIT:
            return False
        s = self._gmask_cache.get((r.params.grammar, r.grammar.key()))
        return s is not None and s >= 0

    def _grammar_mask_slot(self, r, V: int, dev):
        """Slot of r's current parse state in the device mask pool; -1 when nothing may follow
        (the grammar is complete); None when the state is too permissive for a cheap trie walk
        on first sight (the top-N filter handles it; if the state recurs its full mask is
        walked once and cached).
        Masks are keyed by (grammar text, parse-state hash), so the states a JSON schema's
        grammar revisits on every request and every row are walked once."""
        return self._state_slot(r.params.grammar, r.grammar, V, dev)

    def _state_slot(self, gtext: str, gs, V: int, dev, key: Optional[int] = None):
        """_grammar_mask_slot for a parse state object `gs` of grammar `gtext`."""
        key = (gtext, gs.key() if key is None else key)
        c = self._gmask_cache
        if key in c:
            c.move_to_end(key)
            return c[key]
        over = self._gmask_over
        pend = self._gmask_pending
        if key in pend:
            if not pend[key].done():
                return None             # the background walk is still running: top-N filter meanwhile
            m = pend.pop(key).result()
        elif key in over:
            # a permissive state seen again (e.g. `[a-z ]+`, or inside a string of a JSON
            # schema): walk the whole trie once and keep its mask.  A full walk can take tens of
            # ms, so a single-rank engine runs it on a helper thread (the native walk releases
            # the GIL) and keeps serving the state through the top-N filter until it is ready;
            # tensor-parallel ranks walk inline so every rank takes the same decisions
            del over[key]
            if self.tp.world == 1:
                if self._gmask_bg is None:
                    import concurrent.futures
                    self._gmask_bg = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="gmask")
                pend[key] = self._gmask_bg.submit(gs.clone().mask)
                return None
            m = gs.mask()
        else:
            m = gs.mask_limited(self.GRAMMAR_MASK_BUDGET)
            if m is None:
                if len(over) > 4096:
                    over.clear()
                over[key] = 1
                return None
        if not m.any():
            slot = -1
        else:
            pool = self._gmask_pool_for(V, dev)
            if not self._gmask_free:  # evict the least recently used state that owns a slot
                victim = next(k for k, v in c.items() if v is not None and v >= 0)
                self._gslot_release(c.pop(victim))
            slot = self._gmask_free.pop()
            n = min(len(m), V)
            pool[slot, :n].copy_(torch.from_numpy(m[:n].astype(bool)))
            self._gmask_np[slot] = m   # host copy: transitions out of the state can be expanded
        c[key] = slot
        if slot is not None and slot >= 0:
            self._gslot_key[slot] = key
        while len(c) > 4 * self.GRAMMAR_MASK_SLOTS:
            _, v = c.popitem(last=False)
            if v is not None and v >= 0:
                self._gslot_release(v)
        return slot

    def _apply_grammar(self, reqs, logits, prm, toks):
        """Constrained decoding: keep the device sample if the grammar accepts it (the common
        case); otherwise re-run the sampler chain on the logits restricted to grammar-valid
        tokens (llama.cpp resample path).  Rows whose parse state has a cached device mask are
        re-sampled together on the device in one masked pass; permissive states take the device
        top-N candidates the grammar accepts (whole-vocabulary scan if none is)."""
        toks = np.array(toks, copy=True)
        need = [j for j, r in enumerate(reqs)
                if r.grammar is not None and not r.done and not r.grammar.check(int(toks[j]))]
        if not need:
            return toks
        dev = logits.device
        masked, slots, filt = [], [], []
        for j in need:
            s = self._grammar_mask_slot(reqs[j], logits.shape[1], dev)
            if s is None:
                filt.append(j)
            elif s < 0:
                toks[j] = -1  # nothing can follow: the grammar is complete
            else:
                masked.append(j)
                slots.append(s)
        if masked:
            sub = logits[torch.tensor(masked, device=dev)].float()
            allow = self._gmask_pool[torch.tensor(slots, device=dev)]
            sub.masked_fill_(~allow, float("-inf"))
            toks[masked] = ops.sample(sub, prm[np.array(masked)]).cpu().numpy()
        if not filt:
            return toks
        # one batched top-N and one device->host copy for the permissive-state rows
        sub = logits[torch.tensor(filt, device=dev)].float()
        n = min(self.GRAMMAR_TOPN, sub.shape[1])
        vals, idx = torch.topk(sub, n, dim=-1)
        vals_h, idx_h = vals.cpu(), idx.cpu().numpy().astype(np.int32)
        rows_h = None
        for k, j in enumerate(filt):
            gs = reqs[j].grammar
            ok = gs.filter(idx_h[k]).astype(bool)
            if ok.any():
                cand_ids = idx_h[k][ok]
                cand_vals = vals_h[k][torch.from_numpy(ok)]
            else:
                mask = gs.mask().astype(bool)  # whole vocabulary (byte-trie walk in the native core)
                if not mask.any():
                    toks[j] = -1
                    continue
                if rows_h is None:
                    rows_h = sub.cpu()
                cand_ids = np.nonzero(mask)[0].astype(np.int32)
                cand_vals = rows_h[k][torch.from_numpy(cand_ids).long()]
            one = prm[j:j + 1].copy()
            c = int(ops.sample_ref(cand_vals.view(1, -1), one)[0])
            toks[j] = int(cand_ids[c])
        return toks

    def _sample_host_mirostat1(self, logits, reqs):
        """Mirostat v1 (rare): host implementation of llama_sampler_mirostat."""
        out = []
        lg = logits.float().cpu()
        V = lg.shape[1]
        for j, r in enumerate(reqs):
            p = r.params
            row = lg[j] / max(p.temperature, 1e-6)
            if p.mirostat != 1:
                out.append(int(torch.argmax(row)))
                continue
            probs, idx = torch.sort(torch.softmax(row, -1), descending=True)
            m = 100
            num = den = 0.0
            for i in range(min(m - 1, V - 1)):
                t_i = math.log((i + 2) / (i + 1))
                b_i = math.log(float(probs[i]) / float(probs[i + 1]))
                num += t_i * b_i
                den += t_i * t_i
            s_hat = num / den
            eps = s_hat - 1
            k = int(((eps * 2 ** r.mu) / (1 - V ** (-eps))) ** (1 / s_hat)) if eps > 0 else V
            k = max(1, min(k, V))
            q = probs[:k] / probs[:k].sum()
            g = torch.Generator().manual_seed(p.seed + r.n_gen)
            c = int(torch.multinomial(q, 1, generator=g))
            r.mu -= p.mirostat_eta * (-math.log2(float(q[c])) - p.mirostat_tau)
            out.append(int(idx[c]))
        return np.array(out, dtype=np.int32)

    def _on_token(self, r: Request, tok: int, now: float, append: bool = True):
        if r.done:
            return
        if r.grammar is not None:
            if tok < 0:
                self._finish(r, "stop")  # grammar complete, no token may follow
                return
            if not r.grammar.accept(tok):
                self._finish(r, "error", error="grammar rejected the sampled token")
                return
        if append:
            self.sched.append(r.id, tok)
        if r.out_ids is not None:
            r.out_ids.append(tok)
        r.n_gen += 1
        self.metrics["gen_tokens"] += 1
        if r.first_token_t == 0.0:
            r.first_token_t = now
            if self.tracer is not None:
                self.tracer.instant("first_token", now, cat="request", tid=1, id=r.id,
                                    correlation_id=r.params.correlation_id)
        p = r.params
        if self.tokenizer.is_eog(tok) and not p.ignore_eos:
            self._finish(r, "stop")
            return
        text, stopped = r.stream.push(tok)
        if stopped:
            if text:
                self._emit(r, text, tok)
            self._finish(r, "stop", flush=False)
            return
        if p.max_tokens > 0 and r.n_gen >= p.max_tokens:
            if text:
                self._emit(r, text, tok)
            self._finish(r, "length")
            return
        if r.n_prompt + r.n_gen >= self.ctx:
            if text:
                self._emit(r, text, tok)
            self._finish(r, "length")
            return
        if not self._emit(r, text, tok):
            self._finish(r, "abort")  # the client went away

    def _emit(self, r: Request, text: bytes, tok: int) -> bool:
        sink = r.sink
        if sink is not None:
            return sink.push(text, r.n_gen) if text else True
        r.callback(Event(text=text, token=tok))
        return True

    def _finish(self, r: Request, reason: str, flush: bool = True, error: str = ""):
        if r.done:
            return
        r.done = True
        tail = r.stream.flush() if (flush and r.stream is not None) else b""
        p = r.params
        if p.prompt_cache_path and not p.prompt_cache_ro and r.n_gen > 0 and self.tp.world == 1 \
                and self.sched.has(r.id):
            try:
                toks = self.sched.tokens(r.id)
                keep = len(toks) - 1 if p.prompt_cache_all else r.n_prompt  # tokens whose KV exists
                self._pcache.store(self, r.id, toks[:keep], p.prompt_cache_path)
            except Exception:
                log.exception("saving prompt cache %s", p.prompt_cache_path)
        self.sched.finish(r.id)
        self.requests.pop(r.id, None)
        if self.drafter is not None:
            self.drafter.release(r.id)
        end = time.perf_counter()
        ttft = (r.first_token_t - r.arrival) if r.first_token_t else 0.0
        gen_s = end - r.first_token_t if r.first_token_t else 0.0
        self.last_request_stats = {"id": r.id, "prompt_tokens": r.n_prompt, "completion_tokens": r.n_gen,
                                   "ttft_s": ttft, "gen_s": gen_s,
                                   "tokens_per_second": (r.n_gen - 1) / gen_s if gen_s > 0 and r.n_gen > 1 else 0.0}
        if self.tracer is not None:
            self.tracer.complete("request", r.arrival, end, cat="request", tid=1, id=r.id,
                                 correlation_id=r.params.correlation_id, prompt_tokens=r.n_prompt,
                                 completion_tokens=r.n_gen, ttft_ms=round(ttft * 1e3, 3), finish_reason=reason)
        if log.isEnabledFor(logging.DEBUG):
            log.debug("request %s [%s] done (%s): prompt %d tok, gen %d tok, ttft %.1f ms, %.1f tok/s",
                      r.id, r.params.correlation_id, reason, r.n_prompt, r.n_gen, ttft * 1e3,
                      self.last_request_stats["tokens_per_second"])
        try:
            r.callback(Event(text=tail, finished=True, finish_reason=reason, prompt_tokens=r.n_prompt,
                             completion_tokens=r.n_gen, error=error, token_ids=r.out_ids,
                             logits=r.out_logits))
        except Exception:
            log.exception("callback failed")

    # ------------------------------------------------------------------ embeddings
    def embed(self, texts: Sequence, pool: str = "mean", timeout: float = 600.0) -> List[List[float]]:
        """Final-layer hidden states pooled per input (mean by default).  Runs on the engine
        thread (the scheduler / KV pool are single-owner)."""
        job = {"texts": list(texts), "pool": pool, "done": threading.Event()}
        self._inbox.put(("embed", job))
        self._wake.set()
        if self._thread is None:
            self._drain_inbox()
        elif not job["done"].wait(timeout):
            raise TimeoutError("embedding timed out")
        if "error" in job:
            raise RuntimeError(job["error"])
        return job["result"]

    def _run_embed_job(self, job):
        try:
            out = []
            for t in job["texts"]:
                toks = self.tokenize(t) if isinstance(t, str) else list(t)
                toks = toks[: self.ctx - 1] or [0]
                h = self._hidden(toks)
                v = h.mean(0) if job["pool"] == "mean" else h[-1]
                out.append(v.float().cpu().tolist())
            job["result"] = out
        except Exception as e:  # report to the caller
            job["error"] = str(e)
        job["done"].set()

    def _hidden(self, toks: List[int]) -> torch.Tensor:
        sid = -self.new_id()
        bm = self.sched.blocks()
        bs = self.cfg.block_size
        if bm.allocate(sid, toks, len(toks)) < 0:
            raise RuntimeError("out of KV blocks for embedding")
        try:
            tab = bm.table(sid)
            T = len(toks)
            slots = np.array([tab[p // bs] * bs + p % bs for p in range(T)], dtype=np.int32)
            fb = ForwardBatch(tokens=self._dev(np.array(toks, dtype=np.int32)),
                              pos=self._dev(np.arange(T, dtype=np.int32)), slots=self._dev(slots), decode=False,
                              block_tables=self._dev(np.array([tab], dtype=np.int32)),
                              cu_q=self._dev(np.array([0, T], dtype=np.int32)),
                              ctx_lens=self._dev(np.array([T], dtype=np.int32)),
                              tiles=ops.prefill_tiles([T], self.device) if self.device.type == "cuda" else None)
            return self.model.forward(fb, self.kv, return_hidden=True)
        finally:
            bm.free_seq(sid)
