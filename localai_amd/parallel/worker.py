"""Tensor-parallel engine worker group (replaces the reference's llama.cpp RPC workers /
`local-ai worker llama-cpp-rpc` and vLLM's tensor_parallel_size).

Launch one process per GPU (torchrun sets RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m localai_amd.parallel.worker --model llama3-70b.gguf --addr 127.0.0.1:50051

Every rank loads its shard (column-parallel QKV / gate|up, row-parallel o / down, vocab-parallel
lm_head) and builds the same scheduler.  Rank 0 serves backend.proto over gRPC (or the whole HTTP
API with --http) and broadcasts new requests / aborts to the followers each step over a gloo
group; activations are all-reduced over RCCL ("nccl" backend on ROCm).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import sys


def init_distributed():
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        if use_gpu:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    ctrl = dist.new_group(backend="gloo") if world > 1 else None
    dev = f"cuda:{local}" if use_gpu else "cpu"
    return rank, world, dev, ctrl


def build_engine(args, rank, world, dev, ctrl):
    import torch.distributed as dist
    from ..engine.llm_engine import EngineConfig, LLMEngine
    from ..models.decoder import TPInfo
    tp = TPInfo(rank=rank, world=world, group=dist.group.WORLD if world > 1 else None,
                ep=bool(getattr(args, "expert_parallel", False)))
    if world > 1:
        from .custom_ar import maybe_create
        tp.car = maybe_create(dist.group.WORLD, rank, world, dev)
    cfg = EngineConfig(model_path=args.model, device=dev, context_size=args.context, max_num_seqs=args.max_num_seqs,
                       max_batched_tokens=args.max_batched_tokens, use_graphs=not args.eager,
                       decode_steps=args.decode_steps)
    return LLMEngine(cfg, tp=tp, ctrl_group=ctrl)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("localai_amd.parallel.worker")
    ap.add_argument("--model", required=True)
    ap.add_argument("--addr", default="127.0.0.1:50051", help="gRPC (backend.proto) address served by rank 0")
    ap.add_argument("--http", default="", help="serve the full HTTP API from rank 0 instead (host:port)")
    ap.add_argument("--name", default="", help="model name under --http")
    ap.add_argument("--context", type=int, default=4096)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-batched-tokens", type=int, default=8192)
    ap.add_argument("--decode-steps", type=int, default=8)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--expert-parallel", action="store_true",
                    default=os.environ.get("LOCALAI_AMD_EP", "0") == "1",
                    help="MoE models: each rank holds whole experts (E / world) instead of an F slice of every expert")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s tp-worker %(message)s")
    rank, world, dev, ctrl = init_distributed()
    eng = build_engine(a, rank, world, dev, ctrl)
    eng.warmup()
    if rank != 0:
        eng.run_follower()
        return 0
    eng.start()
    if a.http:
        from ..gateway.app import create_app_for_engine
        from ..gateway.native_server import NativeHTTPServer
        host, _, port = a.http.rpartition(":")
        app, _ = create_app_for_engine(eng, name=a.name or os.path.basename(a.model))
        srv = NativeHTTPServer(app, host or "0.0.0.0", int(port))
        logging.info("TP=%d HTTP API on %s", world, a.http)
        try:
            srv.run()
        finally:
            eng.shutdown()
        return 0
    from ..grpc import backend_pb as pb
    from ..grpc.rpc import serve
    from ..grpc.servicer import EngineServicer
    sv = EngineServicer(device=dev)
    sv.engine, sv.model_name, sv.state = eng, os.path.basename(a.model), pb.StatusResponse.READY
    sv.loaded_path = os.path.abspath(a.model)

    async def run():
        server = await serve(sv, a.addr)
        logging.info("TP=%d gRPC backend on %s", world, a.addr)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sgn in (signal.SIGTERM, signal.SIGINT):
            try:
                loop.add_signal_handler(sgn, stop.set)
            except NotImplementedError:
                pass
        await stop.wait()
        await server.stop(2)
    try:
        asyncio.run(run())
    finally:
        eng.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
