"""In-server data parallelism (parallel/replicas.py + ModelManager data_parallel_size): least-busy
dispatch, prefix affinity, stateful RPCs pinned to one replica, and end-to-end generation through
two CPU engine replicas matching a single engine."""
import asyncio
import shutil

from localai_amd.grpc import backend_pb as pb
from localai_amd.parallel.replicas import ReplicaBackend


class _Fake:
    def __init__(self, name):
        self.name, self.calls, self.addr = name, [], name
        self.gate = None

    def __getattr__(self, rpc):
        if rpc.startswith("_"):
            raise AttributeError(rpc)

        if rpc == "PredictStream":
            async def gen(req, timeout=None):
                self.calls.append((rpc, req.Prompt))
                if self.gate is not None:
                    await self.gate.wait()
                yield pb.Reply(message=self.name.encode())
            return gen

        async def call(req, timeout=None):
            self.calls.append((rpc, getattr(req, "Prompt", "")))
            if rpc == "LoadModel":
                return pb.Result(success=True, message=self.name)
            return pb.Reply(message=self.name.encode())
        return call

    async def health(self, timeout=5.0):
        return True


def test_least_busy_dispatch_and_release():
    a, b = _Fake("a"), _Fake("b")
    rb = ReplicaBackend([a, b], affinity_chars=10_000)  # prompts too short for affinity

    async def run():
        ev = asyncio.Event()
        a.gate = b.gate = ev
        gens = [rb.PredictStream(pb.PredictOptions(Prompt=f"p{i}")) for i in range(4)]
        tasks = [asyncio.ensure_future(g.__anext__()) for g in gens]
        await asyncio.sleep(0.01)
        assert sorted(rb.inflight) == [2, 2]  # 4 open streams spread 2/2
        ev.set()
        for t in tasks:
            await t
        for g in gens:
            async for _ in g:
                pass
        assert rb.inflight == [0, 0]
        r = await rb.Predict(pb.PredictOptions(Prompt="x"))
        assert r.message in (b"a", b"b") and rb.inflight == [0, 0]
    asyncio.run(run())


def test_pick_native_local_and_pinned_remote():
    """The gateway's native SSE path (openai_routes._native_stream): an in-process replica is
    returned with its servicer; a remote pick is pinned so the next streaming RPC of the same
    task lands on it, counted once."""
    from localai_amd.grpc.rpc import EmbeddedBackend

    class _Sv:
        engine = object()

    local, remote = EmbeddedBackend(_Sv()), _Fake("r")
    rb = ReplicaBackend([local, remote], affinity_chars=10_000)

    async def run():
        i, sv = rb.pick_native(pb.PredictOptions(Prompt="a"))
        assert i == 0 and isinstance(sv, _Sv) and rb.inflight == [1, 0]
        j, sv2 = rb.pick_native(pb.PredictOptions(Prompt="b"))  # least busy: the remote
        assert j == 1 and sv2 is None and rb.inflight == [1, 0] and rb.served == [1, 0]
        # the local replica is now idle: an unpinned pick would choose it, the pin must win
        rb._done(0)
        async for rep in rb.PredictStream(pb.PredictOptions(Prompt="b")):
            assert rep.message == b"r"
        assert rb.served == [1, 1] and rb.inflight == [0, 0] and remote.calls == [("PredictStream", "b")]
    asyncio.run(run())


def test_prefix_affinity_and_sticky_stores():
    a, b, c = _Fake("a"), _Fake("b"), _Fake("c")
    rb = ReplicaBackend([a, b, c], affinity_chars=64)
    sys_prompt = "You are a helpful assistant. " * 4

    async def run():
        first = await rb.Predict(pb.PredictOptions(Prompt=sys_prompt + "question one"))
        for q in ("two", "three", "four"):
            r = await rb.Predict(pb.PredictOptions(Prompt=sys_prompt + q))
            assert r.message == first.message  # same 64-char prefix -> same replica
        for _ in range(3):
            await rb.StoresSet(pb.StoresSetOptions())
        assert [x[0] for x in a.calls].count("StoresSet") == 3  # stateful RPCs on replica 0 only
        res = await rb.LoadModel(pb.ModelOptions(Model="m"))
        assert res.success and all(any(x[0] == "LoadModel" for x in f.calls) for f in (a, b, c))
        assert await rb.health()
    asyncio.run(run())


def test_affinity_yields_to_load():
    a, b = _Fake("a"), _Fake("b")
    rb = ReplicaBackend([a, b], affinity_chars=16, affinity_slack=1)
    p = "shared prefix shared prefix"
    i0 = rb.pick(pb.PredictOptions(Prompt=p))
    i1 = rb.pick(pb.PredictOptions(Prompt=p))   # affine replica 1 ahead: within slack
    assert i1 == i0
    i2 = rb.pick(pb.PredictOptions(Prompt=p))   # 2 ahead of the other: goes elsewhere
    assert i2 != i0


def test_model_manager_two_cpu_replicas(tiny_model_path, tmp_path):
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.model_manager import ModelManager
    shutil.copy(tiny_model_path, tmp_path / "tiny.gguf")
    mm = ModelManager(ApplicationConfig(models_path=str(tmp_path)), str(tmp_path))
    cfg = BackendConfig({"name": "tiny", "backend": "localai-amd", "context_size": 256, "data_parallel_size": 2,
                         "parameters": {"model": "tiny.gguf"}})

    async def collect(h, prompt):
        out = b""
        async for rep in h.PredictStream(pb.PredictOptions(Prompt=prompt, Tokens=6, Temperature=0.0, IgnoreEOS=True)):
            out += rep.message
        return out

    async def run():
        lm = await mm.load(cfg)
        rb = lm.handle
        assert isinstance(rb, ReplicaBackend) and len(rb.replicas) == 2
        assert lm.backend_name == "localai-amd-dp2"
        prompts = [f"replica test prompt {i}" for i in range(6)]
        outs = await asyncio.gather(*(collect(rb, p) for p in prompts))
        assert all(rb.served) and sum(rb.served) == 6  # both replicas took requests
        assert rb.inflight == [0, 0]
        # every replica computes the same greedy continuation as replica 0 alone
        for p, o in zip(prompts, outs):
            alone = await collect(rb.replicas[0], p)
            assert o == alone, (p, o, alone)
        await mm.stop_all()
    asyncio.run(run())


def test_model_manager_process_replicas_over_grpc(tiny_model_path, tmp_path):
    """engine_mode=process: each replica is its own worker process (one per GPU on a node) behind a
    persistent gRPC channel; the replica handle spreads concurrent streams over both."""
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.model_manager import ModelManager
    shutil.copy(tiny_model_path, tmp_path / "tiny.gguf")
    ac = ApplicationConfig(models_path=str(tmp_path))
    ac.engine_mode = "process"
    mm = ModelManager(ac, str(tmp_path))
    cfg = BackendConfig({"name": "tiny", "backend": "localai-amd", "context_size": 256, "replicas": 2,
                         "parameters": {"model": "tiny.gguf"}})

    async def collect(h, prompt):
        out = b""
        async for rep in h.PredictStream(pb.PredictOptions(Prompt=prompt, Tokens=5, Temperature=0.0, IgnoreEOS=True)):
            out += rep.message
        return out

    async def run():
        lm = await mm.load(cfg)
        try:
            rb = lm.handle
            assert isinstance(rb, ReplicaBackend) and len(rb.replicas) == 2 and lm.process is not None
            outs = await asyncio.gather(*(collect(rb, f"process replica {i}") for i in range(4)))
            assert all(outs) and all(rb.served)
            assert await mm._check_alive(lm)
        finally:
            await mm.stop_all()
    asyncio.run(run())
