"""Failure detection / respawn under injected faults: a fatal engine step error,
a failed KV allocation (hipMalloc), a dropped gRPC stream, all on the CPU engine.  The model
manager health-checks the backend before reuse and respawns an unhealthy one, like the
reference's CheckIsLoaded (pkg/model/loader.go:170-206)."""
import asyncio
import os
import shutil

import pytest

from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.utils import faults


@pytest.fixture
def fault_env(monkeypatch):
    def arm(spec):
        monkeypatch.setenv("LOCALAI_AMD_FAULT", spec)
        faults.reset()
    yield arm
    monkeypatch.delenv("LOCALAI_AMD_FAULT", raising=False)
    faults.reset()


def test_fault_spec_fires_once_on_nth_hit(fault_env):
    fault_env("a:3,b")
    assert [faults.hit("a") for _ in range(5)] == [False, False, True, False, False]
    assert faults.hit("b") and not faults.hit("b")
    assert not faults.hit("c") and not faults.armed("c") and faults.armed("a")


def _engine(path):
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    return LLMEngine(EngineConfig(model_path=path, device="cpu", context_size=256, max_num_seqs=4, use_graphs=False))


def test_kv_alloc_failure_is_a_load_error(tiny_model_path, fault_env):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    fault_env("kv_alloc")
    sv = EngineServicer(device="cpu")
    res = asyncio.run(sv.LoadModel(pb.ModelOptions(ModelFile=tiny_model_path, ContextSize=256)))
    assert not res.success and "hipMalloc" in res.message


def test_fatal_step_fails_requests_and_marks_unhealthy(tiny_model_path, fault_env):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    fault_env("engine_step:2")
    eng = _engine(tiny_model_path)
    eng.start()
    try:
        res = eng.generate("hello", SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True))
        assert res.get("finish_reason") == "error" or res.get("error"), res
        assert not eng.healthy and "injected" in eng.fatal_error
        sv = EngineServicer(device="cpu")
        sv.engine = eng
        assert asyncio.run(sv.Health(pb.HealthMessage())).message.startswith(b"unhealthy")
        # new work is refused instead of hanging on a dead device
        res2 = eng.generate("again", SamplingParams(max_tokens=2, temperature=0.0))
        assert res2.get("error")
    finally:
        eng.shutdown()


def test_dropped_stream_frees_the_sequence(tiny_model_path, fault_env):
    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.servicer import EngineServicer
    fault_env("grpc_stream_drop")
    eng = _engine(tiny_model_path)
    eng.start()
    sv = EngineServicer(device="cpu")
    sv.engine = eng

    async def run():
        got = []
        with pytest.raises(faults.InjectedFault):
            async for rep in sv.PredictStream(pb.PredictOptions(Prompt="stream", Tokens=32, IgnoreEOS=True,
                                                                 Temperature=0.0)):
                got.append(rep)
        return got

    try:
        got = asyncio.run(run())
        assert len(got) == 1
        for _ in range(200):  # the abort is applied by the engine thread
            if not eng.requests:
                break
            asyncio.run(asyncio.sleep(0.01))
        assert not eng.requests
        assert eng.healthy  # a client-side failure is not an engine failure
    finally:
        eng.shutdown()


def test_model_manager_respawns_unhealthy_backend(tiny_model_path, tmp_path, fault_env):
    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.model_manager import ModelManager
    shutil.copy(tiny_model_path, tmp_path / "tiny.gguf")
    mm = ModelManager(ApplicationConfig(models_path=str(tmp_path)), str(tmp_path))
    cfg = BackendConfig({"name": "tiny", "backend": "localai-amd", "context_size": 256,
                         "parameters": {"model": "tiny.gguf"}})

    async def run():
        lm1 = await mm.load(cfg)
        assert await mm.load(cfg) is lm1  # healthy: reused
        fault_env("engine_step")
        eng = lm1.servicer.engine
        res = eng.generate("x", SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True))
        assert not eng.healthy, res
        lm2 = await mm.load(cfg)  # health check fails -> torn down and respawned
        assert lm2 is not lm1 and lm2.servicer.engine.healthy
        res = lm2.servicer.engine.generate("y", SamplingParams(max_tokens=3, temperature=0.0, ignore_eos=True))
        assert res["completion_tokens"] == 3
        await mm.stop_all()

    asyncio.run(run())
