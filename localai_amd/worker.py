"""Backend worker process: serves backend.proto for one model on one GPU.

The reference spawns one `grpc-server` binary per model (`pkg/model/initializers.go:startProcess`,
`backend/cpp/llama/grpc-server.cpp`).  Ours is `python -m localai_amd.worker --addr host:port`
hosting an EngineServicer (HIP engine + vector store) bound to `LOCALAI_DEVICE` (or
`--device`).  Exits when stdin closes if `--die-with-parent` is given.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("localai_amd.worker")
    ap.add_argument("--addr", default="127.0.0.1:50051")
    ap.add_argument("--device", default=os.environ.get("LOCALAI_DEVICE"))
    ap.add_argument("--die-with-parent", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if os.environ.get("LOCALAI_DEBUG") == "true" else logging.INFO,
                        format="%(asctime)s %(levelname)s worker[%(process)d] %(message)s")
    os.environ["LOCALAI_AMD_WORKER"] = "1"  # arms the worker-only fault sites (utils/faults.py)
    import torch  # noqa: F401  (loads the HIP runtime before our kernels)
    from .grpc.rpc import serve
    from .grpc.servicer import EngineServicer

    sv = EngineServicer(device=a.device)

    async def run():
        server = await serve(sv, a.addr)
        logging.getLogger("localai_amd.worker").info("listening on %s (device=%s)", a.addr, a.device)
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGTERM, signal.SIGINT):
            try:
                loop.add_signal_handler(s, stop.set)
            except NotImplementedError:
                pass
        if a.die_with_parent:
            loop.add_reader(sys.stdin.fileno(), lambda: (sys.stdin.read(), stop.set()))
        await stop.wait()
        sv.shutdown()
        await server.stop(2)

    asyncio.run(run())
    return 0


if __name__ == "__main__":
    sys.exit(main())
