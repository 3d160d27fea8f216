"""Model manager: which backend serves which model, loaded lazily, health-checked, watched.

Reference: `pkg/model/{loader,initializers,process,watchdog}.go` (ModelLoader.LoadModel,
BackendLoader/GreedyLoader, startProcess, WatchDog) and `core/backend/options.go`
(ModelOptions / grpcModelOpts).

Backends:
  * our HIP engine (default for GGUF LLMs; aliases: llama-cpp, llama, llama-cpp-hipblas, ...):
      - "inprocess": an EngineServicer in this process, called directly (no sockets)
      - "process"  : `python -m localai_amd.worker --addr 127.0.0.1:<port>` per model, gRPC
  * "local-store": the GPU vector store (stores RPCs)
  * any external backend (`--external-grpc-backends name:host:port` or `name:/path/to/run.sh`)
    speaking the reference backend.proto (whisper/piper/diffusers/... Python backends).
Differences from the reference: per-model load locks instead of one global lock,
persistent gRPC channels (Q5), no per-model op mutex (Q7: the engine batches).
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, Optional

from ..config.backend_config import BackendConfig
from ..grpc import backend_pb as pb
from ..grpc.rpc import EmbeddedBackend, GRPCBackend

log = logging.getLogger("localai_amd.models")

ENGINE_BACKENDS = {"", "llama-cpp", "llama", "llama-cpp-hipblas", "llama-cpp-cuda", "llama-cpp-avx2",
                   "llama-cpp-avx", "llama-cpp-fallback", "llama-cpp-grpc", "llama-ggml", "localai-amd",
                   "vllm", "transformers", "autogptq",  # HF / GPTQ checkpoint directories (hf_checkpoint.py)
                   "whisper"}  # whisper.cpp GGML models run on the native worker (models/whisper.py)
STORE_BACKEND = "local-store"
HF_BACKENDS = {"huggingface", "langchain-huggingface"}  # remote Inference API (grpc/huggingface.py)
MAMBA_BACKEND = "mamba"  # selective state-space LMs (models/mamba.py, ops/csrc/mamba.hip)
RWKV_BACKEND = "rwkv"    # RWKV-4 recurrent LMs (models/rwkv.py)
SD_BACKENDS = {"diffusers", "stablediffusion", "tinydream"}  # Stable Diffusion 1.x / 2.x / XL pipelines (models/sd.py)
VITS_BACKENDS = {"piper", "vits", "mms-tts"}    # VITS text-to-speech voices (models/tts.py)
MUSICGEN_BACKENDS = {"transformers-musicgen", "musicgen"}  # text-to-music (models/musicgen.py)
BARK_BACKENDS = {"bark"}                         # text-to-speech/audio (models/bark.py)
PARLER_BACKENDS = {"parler-tts", "parler_tts"}   # description-conditioned TTS (models/parler.py)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@dataclass
class LoadedModel:
    id: str
    backend_name: str
    handle: object
    servicer: object = None
    process: Optional[subprocess.Popen] = None
    addr: str = ""
    last_used: float = field(default_factory=time.time)
    busy: int = 0
    busy_since: float = 0.0


def grpc_model_options(c: BackendConfig, app, model_path: str) -> pb.ModelOptions:
    """grpcModelOpts (core/backend/options.go:80-178)."""
    r = c.raw
    diff = r.get("diffusers") or {}
    threads = app.threads or int(r.get("threads") or 1)
    seed = c.resolved_seed()
    o = pb.ModelOptions(
        Model=c.model_file_name(), ModelFile=os.path.join(model_path, c.model_file_name()),
        ContextSize=int(r.get("context_size") or 1024), Seed=seed & 0x7FFFFFFF,
        NBatch=int(c.p("batch", 0) or 512), F16Memory=bool(r.get("f16")), MLock=bool(r.get("mmlock")),
        MMap=bool(r.get("mmap")), LowVRAM=bool(r.get("low_vram")), Embeddings=bool(r.get("embeddings")),
        NUMA=bool(r.get("numa")), NGPULayers=int(r.get("gpu_layers") or 9999999), MainGPU=str(r.get("main_gpu") or ""),
        TensorSplit=str(r.get("tensor_split") or ""), Threads=threads, RopeFreqBase=float(c.p("rope_freq_base", 0) or 0),
        RopeFreqScale=float(c.p("rope_freq_scale", 0) or 0), RMSNormEps=float(r.get("rms_norm_eps") or 0),
        NGQA=int(r.get("ngqa") or 0), CUDA=bool(r.get("cuda") or diff.get("cuda")),
        SchedulerType=str(diff.get("scheduler_type") or ""), PipelineType=str(diff.get("pipeline_type") or ""),
        CFGScale=float(diff.get("cfg_scale") or 0), IMG2IMG=bool(diff.get("img2img")),
        CLIPModel=str(diff.get("clip_model") or ""), CLIPSubfolder=str(diff.get("clip_subfolder") or ""),
        CLIPSkip=int(diff.get("clip_skip") or 0), ControlNet=str(diff.get("control_net") or ""),
        LoraBase=str(r.get("lora_base") or ""), LoraAdapter=str(r.get("lora_adapter") or ""),
        LoraScale=float(r.get("lora_scale") or 0), NoMulMatQ=bool(r.get("no_mulmatq")),
        DraftModel=str(r.get("draft_model") or ""), AudioPath=str(((r.get("vall-e") or {}).get("audio_path")) or ""),
        Quantization=str(r.get("quantization") or ""), GPUMemoryUtilization=float(r.get("gpu_memory_utilization") or 0),
        TrustRemoteCode=bool(r.get("trust_remote_code")), EnforceEager=bool(r.get("enforce_eager")),
        SwapSpace=int(r.get("swap_space") or 0), MaxModelLen=int(r.get("max_model_len") or 0),
        TensorParallelSize=int(r.get("tensor_parallel_size") or 0), MMProj=c.mmproj_file_name(),
        FlashAttention=bool(r.get("flash_attention")), NoKVOffload=bool(r.get("no_kv_offloading")),
        YarnExtFactor=float(r.get("yarn_ext_factor") or 0), YarnAttnFactor=float(r.get("yarn_attn_factor") or 0),
        YarnBetaFast=float(r.get("yarn_beta_fast") or 0), YarnBetaSlow=float(r.get("yarn_beta_slow") or 0),
        RopeScaling=str(r.get("rope_scaling") or ""), Type=str(r.get("type") or ""),
        Tokenizer=str(c.p("tokenizer", "") or ""), LibrarySearchPath="")
    return o


class _ReplicaServicers:
    """The in-process servicers of a replicated model, shut down together."""

    def __init__(self, servicers):
        self.servicers = list(servicers)
        self.engine = servicers[0].engine if servicers and hasattr(servicers[0], "engine") else None

    def shutdown(self):
        for sv in self.servicers:
            sv.shutdown()


class _ProcessGroup:
    """The worker processes of a replicated model: poll() reports the first one that died."""

    def __init__(self, procs):
        self.procs = [p for p in procs if p is not None]
        self.returncode = None

    def poll(self):
        for p in self.procs:
            rc = p.poll()
            if rc is not None:
                self.returncode = rc
                return rc
        return None

    def terminate(self):
        for p in self.procs:
            p.terminate()

    def kill(self):
        for p in self.procs:
            p.kill()

    def wait(self, timeout=None):
        for p in self.procs:
            p.wait(timeout)


class ModelManager:
    def __init__(self, app_config, models_path: str):
        self.app = app_config
        self.models_path = models_path
        self.models: Dict[str, LoadedModel] = {}
        self._locks: Dict[str, asyncio.Lock] = {}
        self._global = asyncio.Lock()
        self._watchdog_task = None
        self._next_gpu = 0

    # ------------------------------------------------------------------ lookup
    def list_loaded(self):
        return list(self.models.values())

    def get(self, model_id: str) -> Optional[LoadedModel]:
        return self.models.get(model_id)

    def _lock(self, mid: str) -> asyncio.Lock:
        if mid not in self._locks:
            self._locks[mid] = asyncio.Lock()
        return self._locks[mid]

    def register(self, model_id: str, backend_name: str, handle, servicer=None):
        """Attach an already-running backend (used by tests / the benchmark harness)."""
        self.models[model_id] = LoadedModel(model_id, backend_name, handle, servicer=servicer)

    # ------------------------------------------------------------------ loading
    async def load(self, cfg: BackendConfig) -> LoadedModel:
        mid = cfg.name or cfg.model
        lm = self.models.get(mid)
        if lm is not None and await self._check_alive(lm):
            lm.last_used = time.time()
            return lm
        async with self._lock(mid):
            lm = self.models.get(mid)
            if lm is not None and await self._check_alive(lm):
                return lm
            if self.app.single_active_backend:
                for other in list(self.models):
                    if other != mid:
                        await self.shutdown(other)
            lm = await self._start(mid, cfg)
            self.models[mid] = lm
            return lm

    async def _check_alive(self, lm: LoadedModel) -> bool:
        """CheckIsLoaded: health-check; drop dead process backends so they respawn."""
        if lm.process is not None and lm.process.poll() is not None:
            log.warning("backend for %s died (rc=%s); respawning", lm.id, lm.process.returncode)
            self.models.pop(lm.id, None)
            return False
        if hasattr(lm.handle, "health") and not await lm.handle.health(timeout=120):
            log.warning("backend for %s is unhealthy; respawning", lm.id)
            self.models.pop(lm.id, None)
            try:
                if isinstance(lm.servicer, _ReplicaServicers):
                    lm.servicer.shutdown()  # every replica engine, not just the first
                elif lm.servicer is not None and getattr(lm.servicer, "engine", None) is not None:
                    lm.servicer.engine.shutdown()
                if lm.process is not None:
                    lm.process.kill()
            except Exception:
                log.exception("tearing down the unhealthy backend of %s", lm.id)
            return False
        return True

    def _pick_device(self, cfg: BackendConfig) -> Optional[str]:
        mg = str(cfg.raw.get("main_gpu") or "")
        try:
            import torch
            if not torch.cuda.is_available():
                return "cpu"
            if mg.isdigit():
                return f"cuda:{int(mg)}"
            env = os.environ.get("LOCAL_RANK")
            if env is not None:
                return f"cuda:{int(env)}"
            n = torch.cuda.device_count()
            d = self._next_gpu % max(1, n)
            self._next_gpu += 1
            return f"cuda:{d}"
        except Exception:
            return "cpu"

    async def _start(self, mid: str, cfg: BackendConfig) -> LoadedModel:
        backend = cfg.backend
        ext = self.app.external_grpc_backends
        if backend in ext:
            return await self._start_external(mid, backend, ext[backend], cfg)
        if backend in HF_BACKENDS:
            from ..grpc.huggingface import HuggingFaceServicer
            sv = HuggingFaceServicer()
            res = await sv.LoadModel(grpc_model_options(cfg, self.app, self.models_path), None)
            if not res.success:
                raise RuntimeError(f"could not load model: {res.message}")
            return LoadedModel(mid, "huggingface", EmbeddedBackend(sv), servicer=sv)
        if backend in (MAMBA_BACKEND, RWKV_BACKEND):
            from ..grpc.mamba_servicer import MambaServicer, RwkvServicer
            sv = (MambaServicer if backend == MAMBA_BACKEND else RwkvServicer)(device=self._pick_device(cfg))
            res = await sv.LoadModel(grpc_model_options(cfg, self.app, self.models_path), None)
            if not res.success:
                raise RuntimeError(f"could not load model: {res.message}")
            return LoadedModel(mid, backend, EmbeddedBackend(sv), servicer=sv)
        if backend in SD_BACKENDS:
            from ..grpc.diffusers_servicer import DiffusersServicer
            sv = DiffusersServicer(device=self._pick_device(cfg))
            res = await sv.LoadModel(grpc_model_options(cfg, self.app, self.models_path), None)
            if not res.success:
                raise RuntimeError(f"could not load model: {res.message}")
            return LoadedModel(mid, backend, EmbeddedBackend(sv), servicer=sv)
        if backend in VITS_BACKENDS | MUSICGEN_BACKENDS | BARK_BACKENDS | PARLER_BACKENDS:
            from ..grpc import audio_servicer as au
            cls = (au.VitsServicer if backend in VITS_BACKENDS else
                   au.MusicgenServicer if backend in MUSICGEN_BACKENDS else
                   au.ParlerServicer if backend in PARLER_BACKENDS else au.BarkServicer)
            sv = cls(device=self._pick_device(cfg))
            res = await sv.LoadModel(grpc_model_options(cfg, self.app, self.models_path), None)
            if not res.success:
                raise RuntimeError(f"could not load model: {res.message}")
            return LoadedModel(mid, backend, EmbeddedBackend(sv), servicer=sv)
        if backend == STORE_BACKEND:
            from ..grpc.servicer import EngineServicer
            sv = EngineServicer(device=self._pick_device(cfg))
            return LoadedModel(mid, backend, EmbeddedBackend(sv), servicer=sv)
        if backend not in ENGINE_BACKENDS:
            raise RuntimeError(f"backend {backend!r} is not available (register it with --external-grpc-backends)")
        opts = grpc_model_options(cfg, self.app, self.models_path)
        from ..models.hf_checkpoint import is_hf_checkpoint
        if not (os.path.isfile(opts.ModelFile) or is_hf_checkpoint(opts.ModelFile)):
            raise RuntimeError(f"could not load model: model file {opts.ModelFile} not found")
        tp = int(cfg.raw.get("tensor_parallel_size") or 0)
        dp = int(cfg.raw.get("data_parallel_size") or cfg.raw.get("replicas") or 0)
        if dp > 1:
            return await self._start_replicas(mid, cfg, opts, dp, tp)
        if tp > 1:
            return await self._start_tp_group(mid, cfg, opts, tp)
        if self.app.engine_mode == "process":
            port = free_port()
            addr = f"127.0.0.1:{port}"
            dev = self._pick_device(cfg)
            cmd = [sys.executable, "-m", "localai_amd.worker", "--addr", addr]
            env = dict(os.environ)
            if dev and dev.startswith("cuda:"):
                env["LOCALAI_DEVICE"] = dev
            proc = subprocess.Popen(cmd, env=env)
            h = GRPCBackend(addr)
            await self._wait_healthy(h, cfg, proc)
            res = await h.LoadModel(opts, timeout=3600)
            if not res.success:
                proc.terminate()
                raise RuntimeError(f"could not load model: {res.message}")
            return LoadedModel(mid, "localai-amd", h, process=proc, addr=addr)
        from ..grpc.servicer import EngineServicer
        sv = EngineServicer(device=self._pick_device(cfg))
        res = await sv.LoadModel(opts)
        if not res.success:
            raise RuntimeError(res.message)
        return LoadedModel(mid, "localai-amd", EmbeddedBackend(sv), servicer=sv)

    def _replica_devices(self, cfg: BackendConfig, n: int, per: int) -> list:
        """Devices of n replicas of `per` GPUs each: consecutive GPUs from main_gpu (default 0);
        every replica on the CPU when there is no GPU."""
        try:
            import torch
            ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
        except Exception:
            ngpu = 0
        if ngpu == 0:
            return ["cpu"] * n
        mg = str(cfg.raw.get("main_gpu") or "0")
        base = int(mg) if mg.isdigit() else 0
        if base + n * per > ngpu:
            raise RuntimeError(f"data_parallel_size {n} x {per} GPU(s) from GPU {base} needs {base + n * per} GPUs, "
                               f"{ngpu} visible")
        return [f"cuda:{base + i * per}" for i in range(n)]

    async def _start_replicas(self, mid: str, cfg: BackendConfig, opts, dp: int, tp: int) -> LoadedModel:
        """data_parallel_size = N > 1: N engine replicas of the model (one per GPU, or one per
        tensor-parallel group of tensor_parallel_size GPUs), served through ONE handle that sends
        each request to the least-busy replica, preferring the replica that holds the request's
        prompt prefix in its cache (parallel/replicas.py)."""
        from ..parallel.replicas import ReplicaBackend
        per = max(1, tp)
        devs = self._replica_devices(cfg, dp, per)
        handles, procs, servicers, names = [], [], [], []
        try:
            for i, dev in enumerate(devs):
                if per > 1:
                    first = int(dev.split(":")[1])
                    vis = ",".join(str(first + j) for j in range(per))
                    lm = await self._start_tp_group(f"{mid}#{i}", cfg, opts, per, visible=vis)
                    handles.append(lm.handle)
                    procs.append(lm.process)
                    names.append(f"{lm.addr}[gpus {vis}]")
                elif self.app.engine_mode == "process":
                    addr = f"127.0.0.1:{free_port()}"
                    env = dict(os.environ)
                    if dev.startswith("cuda:"):
                        env["LOCALAI_DEVICE"] = dev
                    proc = subprocess.Popen([sys.executable, "-m", "localai_amd.worker", "--addr", addr], env=env)
                    procs.append(proc)
                    h = GRPCBackend(addr)
                    await self._wait_healthy(h, cfg, proc)
                    res = await h.LoadModel(opts, timeout=3600)
                    if not res.success:
                        raise RuntimeError(f"could not load model: {res.message}")
                    handles.append(h)
                    names.append(f"{addr}[{dev}]")
                else:
                    from ..grpc.servicer import EngineServicer
                    sv = EngineServicer(device=dev)
                    res = await sv.LoadModel(opts)
                    if not res.success:
                        raise RuntimeError(res.message)
                    servicers.append(sv)
                    handles.append(EmbeddedBackend(sv))
                    names.append(f"embedded[{dev}]#{i}")
        except Exception:
            for sv in servicers:
                sv.shutdown()
            for h in handles:
                if isinstance(h, GRPCBackend):
                    await h.close()
            for p in procs:
                if p is not None:
                    p.terminate()
            raise
        rb = ReplicaBackend(handles, names, affinity_chars=int(cfg.raw.get("replica_affinity_chars") or 512))
        log.info("model %s: %d replicas %s", mid, dp, names)
        return LoadedModel(mid, f"localai-amd-dp{dp}" + (f"xtp{per}" if per > 1 else ""), rb,
                           servicer=_ReplicaServicers(servicers) if servicers else None,
                           process=_ProcessGroup(procs) if procs else None, addr=rb.addr)

    async def _start_tp_group(self, mid: str, cfg: BackendConfig, opts, tp: int, visible: str = "") -> LoadedModel:
        """tensor_parallel_size > 1: one process per GPU via torch.distributed.run (RCCL over xGMI);
        rank 0 serves backend.proto and the gateway talks to it like any other backend.
        `visible`: the group's GPUs (HIP_VISIBLE_DEVICES) when several groups share a node."""
        port, mport = free_port(), free_port()
        addr = f"127.0.0.1:{port}"
        ctx = int(cfg.raw.get("context_size") or opts.ContextSize or 4096)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={tp}",
               "--master-addr", "127.0.0.1", "--master-port", str(mport), "-m", "localai_amd.parallel.worker",
               "--model", opts.ModelFile, "--addr", addr, "--context", str(ctx),
               "--max-num-seqs", os.environ.get("LOCALAI_MAX_NUM_SEQS", "256")]
        if opts.EnforceEager:
            cmd.append("--eager")
        if cfg.raw.get("expert_parallel"):  # model-config extension (not in the reference schema)
            cmd.append("--expert-parallel")
        env = dict(os.environ)
        if visible:
            env["HIP_VISIBLE_DEVICES"] = visible
        proc = subprocess.Popen(cmd, env=env)
        h = GRPCBackend(addr)
        g = dict(cfg.raw.get("grpc") or {})
        g.setdefault("attempts", 300)  # sharded load of a 70B model takes a while
        cfg.raw["grpc"] = g
        await self._wait_healthy(h, cfg, proc)
        res = await h.LoadModel(opts, timeout=3600)
        if not res.success:
            proc.terminate()
            raise RuntimeError(f"could not load model: {res.message}")
        return LoadedModel(mid, f"localai-amd-tp{tp}", h, process=proc, addr=addr)

    async def _wait_healthy(self, h: GRPCBackend, cfg: BackendConfig, proc=None):
        g = cfg.raw.get("grpc") or {}
        attempts = int(g.get("attempts") or 20)
        sleep = float(g.get("attempts_sleep_time") or 2)
        for _ in range(attempts):
            if proc is not None and proc.poll() is not None:
                raise RuntimeError("backend process exited during startup")
            if await h.health(timeout=2):
                return
            await asyncio.sleep(sleep)
        raise RuntimeError("grpc service not ready")

    async def _start_external(self, mid, name, uri, cfg):
        if os.path.exists(uri):
            port = free_port()
            addr = f"127.0.0.1:{port}"
            proc = subprocess.Popen([uri, "--addr", addr])
            h = GRPCBackend(addr)
            await self._wait_healthy(h, cfg, proc)
        else:
            proc, addr = None, uri
            h = GRPCBackend(addr)
        opts = grpc_model_options(cfg, self.app, self.models_path)
        try:
            res = await h.LoadModel(opts, timeout=3600)
            if not res.success:
                raise RuntimeError(res.message)
        except Exception as e:
            if proc is not None:
                proc.terminate()
            raise RuntimeError(f"could not load model: {e}")
        return LoadedModel(mid, name, h, process=proc, addr=addr)

    # ------------------------------------------------------------------ lifecycle
    def mark_busy(self, mid: str, busy: bool):
        lm = self.models.get(mid)
        if lm is None:
            return
        if busy:
            lm.busy += 1
            if lm.busy == 1:
                lm.busy_since = time.time()
        else:
            lm.busy = max(0, lm.busy - 1)
            lm.last_used = time.time()

    async def shutdown(self, mid: str, force: bool = False) -> bool:
        lm = self.models.get(mid)
        if lm is None:
            return False
        # wait while busy (pkg/model/loader.go:143-168), forced after retries
        retries = 0
        while lm.busy and not force:
            retries += 1
            if retries > 10 and os.environ.get("LOCALAI_FORCE_BACKEND_SHUTDOWN") == "true":
                break
            await asyncio.sleep(min(2 ** retries * 0.05, 2.0))
        self.models.pop(mid, None)
        if lm.servicer is not None:
            lm.servicer.shutdown()
        if isinstance(lm.handle, GRPCBackend):
            await lm.handle.close()
        if lm.process is not None:
            lm.process.terminate()
            try:
                lm.process.wait(10)
            except Exception:
                lm.process.kill()
        return True

    async def stop_all(self):
        for mid in list(self.models):
            await self.shutdown(mid, force=True)

    def start_watchdog(self, interval: float = 30.0):
        if not (self.app.watchdog_idle or self.app.watchdog_busy) or self._watchdog_task is not None:
            return

        async def run():
            while True:
                await asyncio.sleep(interval)
                now = time.time()
                for mid, lm in list(self.models.items()):
                    if self.app.watchdog_busy and lm.busy and now - lm.busy_since > self.app.watchdog_busy_timeout:
                        log.warning("watchdog: %s busy for too long, stopping", mid)
                        await self.shutdown(mid, force=True)
                    elif self.app.watchdog_idle and not lm.busy and now - lm.last_used > self.app.watchdog_idle_timeout:
                        log.warning("watchdog: %s idle for too long, stopping", mid)
                        await self.shutdown(mid, force=True)
        self._watchdog_task = asyncio.get_event_loop().create_task(run())
