#!/usr/bin/env python3
"""Headline benchmark: output tokens/s + p50 TTFT of streaming /v1/chat/completions on a
random-init Llama-3-8B-Instruct GGUF (Q4_K_M mix) -- BASELINE.json's metric and config.

One "step" = one wave of `--concurrency` concurrent streaming chat completions per GPU,
each with a synthetic ~`--prompt-len`-token user message and `--max-tokens` generated
tokens (ignore_eos, temperature 0, mirostat 0 -- SURVEY §6 / BASELINE.md).  W untimed
warm-up waves, then exactly K timed waves bracketed by barrier + synchronize.

Multi-GPU: one process per GPU over RCCL.  `python bench.py --gpus N` starts the N ranks
itself (a torch.distributed.run child launched BEFORE this process touches the GPU) unless it
already runs under torchrun (RANK / WORLD_SIZE set).  --tp T groups consecutive ranks into
tensor-parallel replicas of T GPUs (BASELINE config 3: --preset llama3-70b --tp 8); the
N / T replicas are data-parallel (weak scaling: fixed load per replica), aggregate tokens/s =
sum over replicas / max wall time over replicas.

--mode http   : requests go through the real gateway (FastAPI app on the native C++ HTTP
                server, or uvicorn with --server uvicorn) from out-of-process aiohttp SSE
                clients (localai_amd/utils/loadgen.py) -> gateway -> engine (default)
--mode engine : requests are fed to the engine directly (no HTTP), for kernel work

--dp-mode gateway (http): the deployment shape of a LocalAI user with `data_parallel_size: N` --
ONE gateway process (rank 0) takes concurrency x N streams and spreads them over the N engines
(rank 0's in-process, ranks 1..N-1 over gRPC: parallel/replicas.py least-in-flight + prefix
affinity); tokens/s is what that single gateway delivers.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "output tokens/sec + p50 TTFT, /v1/chat/completions Llama-3-8B GGUF, 1/2/4/8 GPU"


def _metric(preset: str) -> str:
    """BASELINE.json's headline metric for the headline model; the same measurement named after
    the model for the other presets (Mixtral, 70B ...)."""
    if preset == "llama3-8b":
        return METRIC
    return METRIC.replace("Llama-3-8B GGUF", MODEL_NAMES.get(preset, preset))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tp", type=int, default=int(os.environ.get("BENCH_TP", 1)),
                    help="tensor-parallel degree per replica (consecutive ranks); replicas = gpus / tp")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=int(os.environ.get("BENCH_CONCURRENCY", 256)))
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--preset", default=os.environ.get("BENCH_PRESET", "llama3-8b"))
    ap.add_argument("--mode", default=os.environ.get("BENCH_MODE", "http"), choices=["http", "engine"])
    ap.add_argument("--context", type=int, default=2048)
    ap.add_argument("--batch-tokens", type=int, default=int(os.environ.get("BENCH_BATCH_TOKENS", 0)),
                    help="prefill tokens per engine step (0: max(8192, 8 prompts))")
    ap.add_argument("--decode-steps", type=int, default=int(os.environ.get("BENCH_DECODE_STEPS", 0)),
                    help="device decode steps per host round trip (0: engine default)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--arrival-rate", type=float, default=float(os.environ.get("BENCH_ARRIVAL_RATE", 0)),
                    help="open-loop Poisson arrivals at this many requests/s (HTTP mode) instead of "
                         "synchronised waves; reports tok/s, p50/p99 TTFT and p50/p99 inter-token latency")
    ap.add_argument("--requests", type=int, default=int(os.environ.get("BENCH_REQUESTS", 0)),
                    help="requests of the open-loop run (default: concurrency x steps)")
    ap.add_argument("--server", default=os.environ.get("BENCH_SERVER", "native"), choices=["native", "uvicorn"])
    ap.add_argument("--clients", type=int, default=int(os.environ.get("BENCH_CLIENTS", 4)),
                    help="load-generator processes (separate from the server process)")
    ap.add_argument("--cache-dir", default=os.environ.get("LOCALAI_AMD_CACHE", "/tmp/localai_amd_cache"))
    ap.add_argument("--dp-mode", default=os.environ.get("BENCH_DP_MODE", "ranks"), choices=["ranks", "gateway"],
                    help="ranks: every rank serves its own gateway + load (summed); gateway: rank 0's ONE "
                         "gateway serves all N GPUs (data_parallel_size: N behind parallel/replicas.py), the "
                         "other ranks' engines answer it over backend.proto gRPC")
    ap.add_argument("--n-draft", type=int, default=0,
                    help="engine mode: n-gram speculative draft length (model-config n_draft); 0 = off")
    return ap.parse_args()


def user_messages(tok, n, plen, seed=0):
    import random
    rnd = random.Random(seed)
    words = ["the", "model", "server", "token", "request", "graph", "kernel", "memory", "stream", "batch",
             "latency", "context", "python", "value", "system", "answer", "question", "data", "quick", "brown"]
    out = []
    for i in range(n):
        ws = []
        while len(tok.encode(" ".join(ws), add_bos=False)) < plen - 24:
            ws.extend(rnd.choice(words) for _ in range(8))
        out.append(f"Request {i}: " + " ".join(ws))
    return out


def percentile(xs, p):
    xs = sorted(xs)
    if not xs:
        return 0.0
    k = (len(xs) - 1) * p / 100.0
    f = int(k)
    c = min(f + 1, len(xs) - 1)
    return xs[f] + (xs[c] - xs[f]) * (k - f)


def spawn_ranks(args) -> int:
    """Start N ranks (torch.distributed.run, 127.0.0.1 rendezvous) as a CHILD process and return
    its exit code.  Called before this process imports torch or touches a GPU."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, BENCH_SPAWNED="1"))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    loadgen = None
    tp_env = max(1, args.tp)
    gw = args.dp_mode == "gateway" and args.gpus > 1
    if gw and (args.mode != "http" or tp_env > 1):
        raise SystemExit("--dp-mode gateway needs --mode http and --tp 1")
    if args.mode == "http" and int(os.environ.get("RANK", "0")) % tp_env == 0 and \
            (not gw or int(os.environ.get("RANK", "0")) == 0):
        # client processes are started before this process touches the GPU (no fork/exec
        # from a GPU-initialised process)
        from localai_amd.utils.loadgen import LoadGen
        loadgen = LoadGen(args.clients * (args.gpus if gw else 1))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share
    # devices round-robin); the real run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)
    if args.gpus > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    tp = max(1, args.tp)
    if world % tp:
        raise SystemExit(f"--tp {tp} does not divide the {world} ranks")
    if not torch.cuda.is_available():
        backend = "gloo"  # CPU rehearsal of the multi-rank path
    if world > 1:
        if torch.cuda.is_available():
            torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        else:
            dist.init_process_group(backend)
    dev = f"cuda:{gpu}" if torch.cuda.is_available() else "cpu"  # cpu: dev smoke runs only
    red_dev = dev if backend == "nccl" else "cpu"  # gloo reduces host tensors
    # replica = tp consecutive ranks; its first rank ("leader") drives the load and the timing
    replica, tp_rank = rank // tp, rank % tp
    leader = tp_rank == 0
    tp_group = ctrl = None
    leaders = None
    if world > 1:
        for r0 in range(0, world, tp):   # new_group is collective: every rank creates every group
            g = dist.new_group(list(range(r0, r0 + tp))) if tp > 1 else None
            c = dist.new_group(list(range(r0, r0 + tp)), backend="gloo") if tp > 1 else None
            if r0 == replica * tp:
                tp_group, ctrl = g, c
        leaders = dist.new_group(list(range(0, world, tp)), backend="gloo")
    n_rep = world // tp

    def sync():
        if dev != "cpu":
            torch.cuda.synchronize()

    from localai_amd.models import synth

    os.makedirs(args.cache_dir, exist_ok=True)
    path = os.path.join(args.cache_dir, f"{args.preset}.gguf")
    t_gen = time.time()
    if rank == 0 and not os.path.exists(path):
        synth.write_model(path + f".partial{os.getpid()}", args.preset)
        os.replace(path + f".partial{os.getpid()}", path)
    if world > 1:
        dist.barrier()
    t_gen = time.time() - t_gen

    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.models.decoder import TPInfo

    tpi = None
    if tp > 1:
        tpi = TPInfo(rank=tp_rank, world=tp, group=tp_group)
        if dev != "cpu":
            from localai_amd.parallel.custom_ar import maybe_create
            tpi.car = maybe_create(tp_group, tp_rank, tp, dev)
    t0 = time.time()
    extra = {"decode_steps": args.decode_steps, "decode_steps_wide": args.decode_steps} if args.decode_steps else {}
    cfg = EngineConfig(model_path=path, device=dev, context_size=args.context,
                       max_num_seqs=max(args.concurrency, 1),
                       max_batched_tokens=args.batch_tokens or max(8192, args.prompt_len * 8),
                       use_graphs=not args.no_graphs,
                       max_kv_tokens=args.concurrency * (args.prompt_len + args.max_tokens + 64) + 4096, **extra)
    eng = LLMEngine(cfg, tp=tpi, ctrl_group=ctrl)
    t_load = time.time() - t0
    t0 = time.time()
    eng.warmup()
    t_capture = time.time() - t0
    if os.environ.get("BENCH_DUMP_GEMM") and rank == 0:
        from localai_amd import ops
        for k, v in sorted(ops._GEMM_CHOICE.items(), key=str):
            print(f"gemm choice M={k[0]} K={k[1]} ws={k[2]} -> {v}", file=sys.stderr)

    if not leader:
        # tensor-parallel follower: mirror the leader's steps until its engine shuts down
        eng.run_follower()
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        if loadgen is not None:
            loadgen.close()
        return

    if gw:
        return gateway_dp(args, eng, loadgen, rank, world, leaders, t_gen, t_load, t_capture)
    msgs = user_messages(eng.tokenizer, args.concurrency, args.prompt_len, seed=replica)
    if args.mode == "http":
        runner = HttpRunner(eng, args, loadgen)
    else:
        runner = EngineRunner(eng, args)

    arrivals = os.environ.get("BENCH_ARRIVALS") == "1"

    def wave(w):
        # the wave tag leads the message: no prompt shares more than the chat-template header with a
        # prompt of an earlier wave, so every wave prefills its 256 prompts in full (a trailing tag
        # would let the engine's prefix cache skip ~90 % of the prefill of every repeated wave)
        if arrivals:
            eng.arrival_log, eng.admit_log = [], []
            tw = time.perf_counter()
        r = runner.wave([f"(wave {w}) " + m for m in msgs])
        if arrivals:  # server-side view of the burst (diagnostics on stderr, outside the JSON line)
            a_ = eng.arrival_log
            ad = eng.admit_log[0] if eng.admit_log else (float("nan"), 0)
            print(f"bench: wave {w} arrivals {len(a_)}: first +{(a_[0] - tw) * 1e3:.1f} ms, spread "
                  f"{(a_[-1] - a_[0]) * 1e3:.1f} ms (p50 +{(a_[len(a_) // 2] - a_[0]) * 1e3:.1f}); admission closed "
                  f"+{(ad[0] - a_[0]) * 1e3:.1f} ms with {ad[1]} waiting; p50 ttft "
                  f"{percentile(r[0], 50) * 1e3:.1f} ms", file=sys.stderr, flush=True)
        return r

    def lbarrier():
        if leaders is not None:
            dist.barrier(group=leaders)

    for w in range(args.warmup):
        wave(-1 - w)
    if args.arrival_rate > 0 and args.mode == "http" and n_rep == 1 and rank == 0:
        return open_loop(args, eng, runner, msgs)
    sync()
    lbarrier()
    sync()
    t0 = time.perf_counter()
    ttfts, tokens = [], 0
    ev0 = getattr(runner, "events", None)
    for k in ("merged", "bad", "short", "split", "tail"):   # counters at the start of the timed waves
        setattr(runner, f"_{k}0", getattr(runner, k, 0))
    for s_ in range(args.steps):
        tt, nt = wave(s_)
        ttfts += tt
        tokens += nt
    sync()
    lbarrier()
    sync()
    elapsed = time.perf_counter() - t0
    # the token count is the server's usage report; check it against the stream itself: ignore_eos
    # fixes every request at max_tokens, and each generated token with non-empty text arrives as
    # its own SSE event (counted by the clients on the wire)
    stream_check = None
    stream_bad = False
    if ev0 is not None:
        # per request, on the wire: every chunk carries the running usage, so the events plus the
        # tokens whose text arrived inside a later event (held-back partial UTF-8) must add up to
        # the reported count, and each request must report exactly max_tokens (ignore_eos)
        expect = args.steps * len(msgs) * args.max_tokens
        events = runner.events - ev0
        merged = getattr(runner, "merged", 0) - getattr(runner, "_merged0", 0)
        d = {k: getattr(runner, k, 0) - getattr(runner, f"_{k}0", 0) for k in ("bad", "short", "split", "tail")}
        stream_check = {"expected_tokens": expect, "reported_tokens": tokens, "streamed_events": events,
                        "merged_tokens": merged, "split_events": d["split"], "tail_tokens": d["tail"],
                        "bad_streams": d["bad"], "short_requests": d["short"]}
        stream_bad = (tokens != expect or events - d["split"] + merged + d["tail"] != tokens or d["bad"]
                      or d["short"])
        if stream_bad:
            print(f"bench: stream check FAILED {stream_check}", file=sys.stderr, flush=True)

    all_ttft, tot_tokens, max_el = ttfts, tokens, elapsed
    if leaders is not None and n_rep > 1:
        el = torch.tensor([elapsed])
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=leaders)
        nt = torch.tensor([float(tokens)])
        dist.all_reduce(nt, group=leaders)
        gathered = [None] * n_rep
        dist.all_gather_object(gathered, ttfts, group=leaders)
        all_ttft = [x for g in gathered for x in g]
        max_el, tot_tokens = float(el.item()), int(nt.item())
    runner.close()
    if tp > 1 and args.mode == "engine":
        eng.shutdown()   # releases the followers (HttpRunner.close already did)
    if rank == 0:
        value = tot_tokens / max_el
        seq = args.prompt_len + args.max_tokens
        par = f"dp{n_rep}" + (f"xtp{tp}" if tp > 1 else "")
        out = {
            "metric": _metric(args.preset),
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_el / args.steps * 1000, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "p50_ttft_ms": round(percentile(all_ttft, 50) * 1000, 2),
            "p90_ttft_ms": round(percentile(all_ttft, 90) * 1000, 2),
            "config": {"model": MODEL_NAMES.get(args.preset, args.preset),
                       "global_batch": args.concurrency * n_rep, "seq_len": seq,
                       "prompt_tokens": args.prompt_len, "max_tokens": args.max_tokens,
                       "parallelism": par, "endpoint": "/v1/chat/completions (stream)",
                       "mode": args.mode, "sampling": "greedy, mirostat 0, ignore_eos",
                       **({"n_draft": args.n_draft} if args.n_draft else {})},
            "setup_s": {"model_gen": round(t_gen, 1), "load": round(t_load, 1), "graph_capture": round(t_capture, 1)},
        }
        if dev != "cpu":  # weights + resident copies + KV cache + workspaces of this rank
            out["device_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 1)
        if stream_check is not None:
            out["stream_check"] = stream_check
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if stream_bad:
        sys.exit(3)


def gateway_dp(args, eng, loadgen, rank, world, ctl, t_gen, t_load, t_capture):
    """--dp-mode gateway: rank 0 serves ONE gateway over all N engines; ranks 1..N-1 expose their
    engine over backend.proto gRPC until rank 0 is done."""
    import asyncio
    import socket

    import torch.distributed as dist
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.rpc import GRPCBackend, serve
    from localai_amd.grpc.servicer import EngineServicer

    eng.start()
    addr = ""
    loop = server = None
    if rank > 0:
        sv = EngineServicer(device=str(eng.device))
        sv.engine, sv.model_name, sv.state = eng, "llama3-8b-instruct", pb.StatusResponse.READY
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        addr = f"127.0.0.1:{port}"
        loop = asyncio.new_event_loop()
        threading.Thread(target=loop.run_forever, daemon=True).start()
        server = asyncio.run_coroutine_threadsafe(serve(sv, addr), loop).result(60)
    addrs = [None] * world
    dist.all_gather_object(addrs, addr, group=ctl)
    if rank > 0:
        dist.barrier(group=ctl)          # rank 0 ran every wave
        asyncio.run_coroutine_threadsafe(server.stop(1), loop).result(30)
        loop.call_soon_threadsafe(loop.stop)
        eng.shutdown()
        dist.barrier()
        dist.destroy_process_group()
        return
    remote = [GRPCBackend(a) for a in addrs[1:]]
    runner = HttpRunner(eng, args, loadgen, replicas=remote)
    n = args.concurrency * world
    msgs = user_messages(eng.tokenizer, n, args.prompt_len, seed=0)

    def wave(w):
        return runner.wave([f"(wave {w}) " + m for m in msgs])

    for w in range(args.warmup):
        wave(-1 - w)
    t0 = time.perf_counter()
    ttfts, tokens = [], 0
    ev0 = getattr(runner, "events", None)
    for k in ("merged", "bad", "short", "split", "tail"):   # counters at the start of the timed waves
        setattr(runner, f"_{k}0", getattr(runner, k, 0))
    for s_ in range(args.steps):
        tt, nt = wave(s_)
        ttfts += tt
        tokens += nt
    elapsed = time.perf_counter() - t0
    served = runner.replica_stats()
    runner.close()
    dist.barrier(group=ctl)
    out = {
        "metric": _metric(args.preset), "value": round(tokens / elapsed, 2), "unit": "tokens/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000, 2),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "p50_ttft_ms": round(percentile(ttfts, 50) * 1000, 2), "p90_ttft_ms": round(percentile(ttfts, 90) * 1000, 2),
        "config": {"model": MODEL_NAMES.get(args.preset, args.preset), "global_batch": n,
                   "seq_len": args.prompt_len + args.max_tokens, "prompt_tokens": args.prompt_len,
                   "max_tokens": args.max_tokens, "parallelism": f"dp{world}-gateway",
                   "endpoint": "/v1/chat/completions (stream)", "mode": "http",
                   "sampling": "greedy, mirostat 0, ignore_eos", "replica_requests": served},
        "setup_s": {"model_gen": round(t_gen, 1), "load": round(t_load, 1), "graph_capture": round(t_capture, 1)},
    }
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


MODEL_NAMES = {"llama3-8b": "Llama-3-8B-Instruct GGUF Q4_K_M (random-init)",
               "llama3-70b": "Llama-3-70B-Instruct GGUF Q4_K_M (random-init)",
               "mixtral-8x7b": "Mixtral-8x7B GGUF Q4_K_M (random-init)"}


class EngineRunner:
    """Feeds chat-templated prompts straight into the engine (no HTTP)."""

    def __init__(self, eng, args):
        self.eng, self.args = eng, args
        from localai_amd.engine.sampling_params import SamplingParams
        self.SP = SamplingParams

    def wave(self, contents):
        eng = self.eng
        ttft, ntok = [], [0]
        done = [0]
        lock = threading.Lock()
        t_start = {}
        for i, c in enumerate(contents):
            prompt = ("<|begin_of_text|><|start_header_id|>user<|end_header_id|>\n\n" + c +
                      "<|eot_id|>\n<|start_header_id|>assistant<|end_header_id|>")
            first = [True]
            t0 = time.perf_counter()

            def cb(ev, first=first, t0=t0):
                with lock:
                    if first[0] and (ev.text or ev.finished):
                        first[0] = False
                        ttft.append(time.perf_counter() - t0)
                    if ev.finished:
                        ntok[0] += ev.completion_tokens
                        done[0] += 1

            eng.add_request(prompt, self.SP(max_tokens=self.args.max_tokens, temperature=0.0, ignore_eos=True,
                                            mirostat=0, repeat_penalty=1.0, n_draft=self.args.n_draft), cb)
        while done[0] < len(contents):
            eng.step()
        return ttft, ntok[0]

    def close(self):
        pass


def open_loop(args, eng, runner, msgs):
    """Open-loop serving measurement: requests arrive as a Poisson process at args.arrival_rate
    (seeded), each with its own prompt; tokens/s over the whole run, TTFT and per-token
    inter-token-latency percentiles (SURVEY §3.2 TTFT; the reference streams one SSE event per
    token, core/http/endpoints/openai/chat.go:463-508)."""
    import numpy as np
    n = args.requests or args.concurrency * max(1, args.steps)
    rng = np.random.default_rng(20261018)
    offs = np.cumsum(rng.exponential(1.0 / args.arrival_rate, size=n)).tolist()
    contents = [f"(arrival {i}) " + msgs[i % len(msgs)] for i in range(n)]
    t0 = time.perf_counter()
    ttft, tokens = runner.wave(contents, offsets=offs)
    el = time.perf_counter() - t0
    w = runner.lg.last_wire
    gaps = sorted(w["gaps_ms"])
    out = {"metric": "open-loop Poisson arrivals, streamed /v1/chat/completions", "rate_rps": args.arrival_rate,
           "requests": n, "tokens_per_s": round(tokens / el, 1), "elapsed_s": round(el, 2),
           "p50_ttft_ms": round(percentile(ttft, 50) * 1e3, 1), "p99_ttft_ms": round(percentile(ttft, 99) * 1e3, 1),
           "p50_itl_ms": round(percentile(gaps, 50), 2) if gaps else None,
           "p99_itl_ms": round(percentile(gaps, 99), 2) if gaps else None,
           "stream_check": {"reported_tokens": tokens, "expected_tokens": n * args.max_tokens,
                            "streamed_events": w["events"], "merged_tokens": w["merged"],
                            "split_events": w["split"], "tail_tokens": w["tail"], "bad_streams": w["bad"]},
           "heuristics": {"admission_window_ms": float(os.environ.get("LOCALAI_AMD_ADMIT_WINDOW_MS",
                                                                      eng.cfg.admission_window_ms)),
                          "prefill_first_ms": float(os.environ.get("LOCALAI_AMD_PREFILL_FIRST_MS",
                                                                   eng.cfg.prefill_first_ms))},
           "config": {"model": MODEL_NAMES.get(args.preset, args.preset), "prompt_tokens": args.prompt_len,
                      "max_tokens": args.max_tokens}}
    print(json.dumps(out), flush=True)
    runner.close()


class HttpRunner:
    """Real gateway over HTTP: the FastAPI app on the native server (or uvicorn), driven by
    out-of-process aiohttp SSE clients."""

    def __init__(self, eng, args, loadgen, replicas=None):
        import socket
        from localai_amd.gateway.app import create_app_for_engine
        self.args = args
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        self.port = s.getsockname()[1]
        s.close()
        self.eng = eng
        eng.start()  # engine loop thread: the servicer only enqueues requests
        self.app, self.model_name = create_app_for_engine(eng, name="llama3-8b-instruct", replicas=replicas)
        if args.server == "native":
            from localai_amd.gateway.native_server import NativeHTTPServer
            self.server = NativeHTTPServer(self.app, "127.0.0.1", 0)
            self.port = self.server.port
        else:
            import uvicorn
            cfg = uvicorn.Config(self.app, host="127.0.0.1", port=self.port, log_level="warning", loop="asyncio",
                                 http="h11", access_log=False)
            self.server = uvicorn.Server(cfg)
        self.th = threading.Thread(target=self.server.run, daemon=True)
        self.th.start()
        for _ in range(600):
            if self.server.started:
                break
            time.sleep(0.05)
        self.lg = loadgen
        self.url = f"http://127.0.0.1:{self.port}/v1/chat/completions"

    def wave(self, contents, offsets=None):
        r = self.lg.wave(self.url, self.model_name, contents, self.args.max_tokens,
                         extra={"temperature": 0, "ignore_eos": True, "mirostat": 0}, offsets=offsets)
        self.events = getattr(self, "events", 0) + getattr(self.lg, "last_events", 0)
        w = getattr(self.lg, "last_wire", None) or {}
        for k in ("merged", "bad", "split", "tail"):
            setattr(self, k, getattr(self, k, 0) + w.get(k, 0))
        # ignore_eos: every request must stream exactly max_tokens
        self.short = getattr(self, "short", 0) + sum(1 for v in getattr(self.lg, "last_per", [])
                                                      if v != self.args.max_tokens)
        return r

    def replica_stats(self):
        """Requests each replica served (gateway DP mode), from the ReplicaBackend."""
        h = getattr(self.app.state, "bench_handle", None)
        return list(h.served) if h is not None and hasattr(h, "served") else None

    def close(self):
        self.lg.close()
        if hasattr(self.server, "shutdown"):
            self.server.shutdown()
        else:
            self.server.should_exit = True
        self.th.join(timeout=10)
        self.eng.shutdown()


if __name__ == "__main__":
    main()
