"""Stable Diffusion pipeline (models/sd.py) and the diffusers backend.

Oracles: the CLIP text encoder against transformers' CLIPTextModel on the same weights (exact,
with and without clip-skip); the DDIM / Euler schedulers against closed form (a denoiser that
returns the true noise must land on the clean latent).  The UNet / VAE have no oracle in this
image (diffusers is not installed): parity unpinned -- they are checked for strict weight-name
coverage on load, shapes, determinism under a seed, and CFG / scheduler plumbing.
"""
import asyncio
import base64
import io
import math
import os

import pytest
import torch
import torch.nn.functional as F

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import synth
from localai_amd.models.sd import Scheduler, StableDiffusion


@pytest.fixture(scope="module")
def pipe_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("sd") / "sd-tiny"
    synth.write_sd_pipeline(str(d))
    return str(d)


@pytest.mark.parametrize("skip", [0, 1])
def test_text_encoder_matches_transformers(pipe_dir, skip):
    import transformers as tf
    p = StableDiffusion(pipe_dir, "cpu", clip_skip=skip)
    te = tf.CLIPTextModel.from_pretrained(os.path.join(pipe_dir, "text_encoder")).eval()
    ids = p.tok(["a red fox in the snow", "x"], padding="max_length", max_length=77, truncation=True,
                return_tensors="pt").input_ids
    with torch.no_grad():
        tm = getattr(te, "text_model", te)
        hs = te(ids, output_hidden_states=True).hidden_states
        ref = tm.final_layer_norm(hs[-(skip + 1)])
        got = p.text(ids, skip)
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("kind", ["ddim", "euler"])
@pytest.mark.parametrize("pred", ["epsilon", "v_prediction"])
def test_scheduler_recovers_clean_latent_with_oracle_denoiser(kind, pred):
    s = Scheduler({"set_alpha_to_one": True, "prediction_type": pred}, kind)
    g = torch.Generator().manual_seed(0)
    x0, eps = torch.randn(1, 4, 8, 8, generator=g), torch.randn(1, 4, 8, 8, generator=g)
    ts = s.timesteps(10)
    assert ts[0] == 901 and ts[-1] == 1 and len(ts) == 10
    a = float(s.ac[ts[0]])
    # the noisy latent in each scheduler's own parameterisation
    x = math.sqrt(a) * x0 + math.sqrt(1 - a) * eps if kind == "ddim" else x0 + math.sqrt((1 - a) / a) * eps
    for i, t in enumerate(ts):
        at = float(s.ac[t])
        out = eps if pred == "epsilon" else math.sqrt(at) * eps - math.sqrt(1 - at) * x0
        x = s.step(out, t, ts[i + 1] if i + 1 < len(ts) else None, x)
    torch.testing.assert_close(x, x0, atol=1e-5, rtol=1e-5)


def test_pipeline_shapes_determinism_and_guidance(pipe_dir):
    p = StableDiffusion(pipe_dir, "cpu")
    a = p("a cat", "blurry", 64, 48, steps=3, guidance_scale=7.0, seed=5)
    assert a.shape == (48, 64, 3) and a.dtype == torch.uint8
    assert torch.equal(a, p("a cat", "blurry", 64, 48, steps=3, guidance_scale=7.0, seed=5))
    assert not torch.equal(a, p("a cat", "blurry", 64, 48, steps=3, guidance_scale=7.0, seed=6))
    assert not torch.equal(a, p("a cat", "blurry", 64, 48, steps=3, guidance_scale=1.0, seed=5))
    p.sched = Scheduler(p.sched_cfg, "euler")
    assert p("a cat", "", 32, 32, steps=2, seed=1).shape == (32, 32, 3)


def test_unet_rejects_missing_weights(pipe_dir, tmp_path):
    import shutil

    from safetensors.torch import load_file, save_file
    d = tmp_path / "broken"
    shutil.copytree(pipe_dir, d)
    f = d / "unet" / "diffusion_pytorch_model.safetensors"
    sd = load_file(str(f))
    sd.pop(next(k for k in sd if "attn2.to_k" in k))
    save_file(sd, str(f))
    with pytest.raises(RuntimeError, match="Missing key"):
        StableDiffusion(str(d), "cpu")


def test_servicer_generate_image(pipe_dir, tmp_path):
    from PIL import Image

    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    sv = DiffusersServicer(device="cpu")
    dst = str(tmp_path / "out.png")

    async def go():
        assert (await sv.LoadModel(pb.ModelOptions(ModelFile=pipe_dir, CFGScale=5.0, SchedulerType="euler"))).success
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a boat", negative_prompt="", width=40,
                                                           height=32, step=2, seed=3, dst=dst))
        assert r.success
        # EnableParameters=none: pipeline defaults (sample_size * 2 px for the two-level toy VAE)
        await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a boat", width=40, height=32, step=1,
                                                       EnableParameters="none", seed=3, dst=dst + ".2.png"))
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a boat", src="in.png", dst=dst + ".3.png"))
        assert not r.success and "No such file" in r.message
        # img2img from a real source keeps the source's size (no width / height asked)
        Image.new("RGB", (24, 16), (200, 30, 30)).save(tmp_path / "src.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a boat", src=str(tmp_path / "src.png"),
                                                           step=4, seed=1, dst=dst + ".4.png"))
        assert r.success, r.message
    asyncio.run(go())
    assert sv.cfg_scale == 5.0 and sv.pipe.sched_name == "euler" and sv.pipe.ksampler is not None
    assert Image.open(dst + ".4.png").size == (24, 16)
    assert Image.open(dst).size == (40, 32)
    px = sv.pipe.unet_sample_size * sv.pipe.vae_scale
    assert Image.open(dst + ".2.png").size == (px, px)


def test_gateway_images_endpoint(pipe_dir, tmp_path):
    import shutil

    from fastapi.testclient import TestClient
    from PIL import Image

    from localai_amd.config.app_config import ApplicationConfig
    from localai_amd.config.backend_config import BackendConfig
    from localai_amd.gateway.app import create_app
    from localai_amd.gateway.state import AppState
    mdir = tmp_path / "models"
    shutil.copytree(pipe_dir, mdir / "sd-tiny")
    ac = ApplicationConfig(models_path=str(mdir), upload_dir=str(tmp_path / "up"), config_dir=str(tmp_path / "cfg"),
                           image_dir=str(tmp_path / "img"), audio_dir=str(tmp_path / "aud"))
    st = AppState(ac)
    bc = BackendConfig({"name": "sd", "backend": "diffusers", "parameters": {"model": "sd-tiny"},
                        "diffusers": {"cfg_scale": 6, "scheduler_type": "ddim"}})
    bc.set_defaults()
    st.configs.add(bc)
    with TestClient(create_app(st)) as c:
        r = c.post("/v1/images/generations", json={"model": "sd", "prompt": "a lighthouse|fog", "size": "32x32",
                                                   "step": 2, "response_format": "b64_json"})
        assert r.status_code == 200, r.text
        img = Image.open(io.BytesIO(base64.b64decode(r.json()["data"][0]["b64_json"])))
        assert img.size == (32, 32)
        assert "diffusers" in c.get("/system").json()["backends"]
        # default response_format (url): the returned URL is served (core/http/routes/openai.go:75)
        r = c.post("/v1/images/generations", json={"model": "sd", "prompt": "a lighthouse", "size": "32x32",
                                                   "step": 1})
        assert r.status_code == 200, r.text
        url = r.json()["data"][0]["url"]
        path = url[url.index("/generated-images/"):]
        got = c.get(path)
        assert got.status_code == 200 and Image.open(io.BytesIO(got.content)).size == (32, 32)
        assert c.get("/generated-images/../../etc/passwd").status_code == 404
        assert c.get("/generated-audio/nope.wav").status_code == 404


@pytest.mark.gpu
def test_pipeline_on_gpu_matches_cpu_layout(pipe_dir):
    """bf16 on the GPU vs fp32 on the CPU: same seed, same scheduler -> close images."""
    a = StableDiffusion(pipe_dir, "cpu")("a cat", "", 32, 32, steps=2, seed=7).float()
    b = StableDiffusion(pipe_dir, "cuda:0")("a cat", "", 32, 32, steps=2, seed=7).float()
    assert (a - b).abs().mean() < 4.0


@pytest.mark.gpu
@pytest.mark.parametrize("shape,groups", [((2, 320, 64, 64), 32), ((2, 1280, 8, 8), 32), ((1, 128, 96, 80), 32),
                                          ((2, 640, 16, 16), 32), ((1, 96, 5, 7), 8), ((3, 2048, 4, 4), 64)])
@pytest.mark.parametrize("silu", [False, True])
def test_groupnorm_nhwc_kernel_matches_fp32(shape, groups, silu):
    from localai_amd import ops
    torch.manual_seed(0)
    C = shape[1]
    x = (torch.randn(shape, device="cuda") * 3 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.rand(C, device="cuda") + 0.5).to(torch.bfloat16)
    b = torch.randn(C, device="cuda").to(torch.bfloat16)
    ref = F.group_norm(x.float(), groups, w.float(), b.float(), 1e-5)
    ref = F.silu(ref) if silu else ref
    got = ops.groupnorm_nhwc(x, groups, w, b, 1e-5, silu)
    assert got.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(got.float(), ref, atol=3e-2, rtol=2e-2)
    got = ops.groupnorm_nhwc(x, groups, None, None, 1e-5, silu)  # affine-free
    ref = F.group_norm(x.float(), groups, None, None, 1e-5)
    torch.testing.assert_close(got.float(), F.silu(ref) if silu else ref, atol=3e-2, rtol=2e-2)
    # fixed-order statistics (no float atomics): repeated launches are bit-identical
    for _ in range(3):
        assert torch.equal(ops.groupnorm_nhwc(x, groups, None, None, 1e-5, silu), got)


@pytest.mark.gpu
def test_unet_on_gpu_matches_fp32_forward(pipe_dir):
    """Every UNet evaluation of a GPU run (bf16, NHWC, our GroupNorm kernels, graph capture and
    replays) against the same UNet weights in fp32 PyTorch on the CPU, on the same inputs."""
    from conftest import compare_to_fp32, record_calls
    gpu = StableDiffusion(pipe_dir, "cuda:0")
    calls = record_calls(gpu, "_unet")
    gpu("a cat", "blurry", 32, 32, steps=3, seed=11)
    assert gpu._graphs
    cpu = StableDiffusion(pipe_dir, "cpu")
    compare_to_fp32(calls, cpu._unet)


@pytest.mark.gpu
def test_unet_graph_replay_matches_eager(pipe_dir):
    p = StableDiffusion(pipe_dir, "cuda:0")
    assert p.use_graphs and p.channels_last
    a = p("a cat", "blurry", 32, 32, steps=3, seed=11)  # first step eager + capture, then replays
    assert p._graphs, "UNet step was not captured"
    p.use_graphs = False
    b = p("a cat", "blurry", 32, 32, steps=3, seed=11)
    assert (a.float() - b.float()).abs().max() <= 2


@pytest.mark.parametrize("w,h", [(520, 72), (40, 24), (72, 56)])
def test_pipeline_any_multiple_of_8(pipe_dir, w, h):
    """Sides that are not a multiple of the UNet's total downsampling: the up path lands on each
    skip's size (diffusers forward_upsample_size) instead of crashing at the concat."""
    p = StableDiffusion(pipe_dir, "cpu")
    img = p("a cat", "", w, h, steps=1, seed=3)
    assert img.shape == (h, w, 3)


@pytest.mark.gpu
def test_unet_graph_cache_is_bounded(pipe_dir, monkeypatch):
    monkeypatch.setenv("LOCALAI_AMD_SD_GRAPH_CACHE", "2")
    p = StableDiffusion(pipe_dir, "cuda:0")
    for side in (32, 40, 48, 56):
        p("a cat", "", side, side, steps=2, seed=1)
    assert len(p._graphs) == 2
    # the two most recent latent sizes (side / the VAE's downscale)
    assert [k[0][-1] for k in p._graphs] == [48 // p.vae_scale, 56 // p.vae_scale]


@pytest.mark.parametrize("name", ["pndm", "heun", "unipc", "euler_a", "lms", "dpm_2", "dpm_2_a", "dpmpp_2m",
                                  "dpmpp_sde", "dpmpp_2m_sde", "k_dpmpp_2m", "k_lms"])
def test_every_reference_scheduler_runs_the_pipeline(pipe_dir, name):
    """Each SchedulerType of the reference's mapping drives the pipeline end to end; seeded runs are
    reproducible; unknown names are refused at load."""
    p = StableDiffusion(pipe_dir, "cpu", scheduler=name)
    a = p("a lighthouse", "", 32, 32, steps=3, seed=5)
    b = p("a lighthouse", "", 32, 32, steps=3, seed=5)
    assert a.shape == (32, 32, 3) and torch.equal(a, b)


def test_unknown_scheduler_refused(pipe_dir):
    with pytest.raises(ValueError, match="Invalid scheduler"):
        StableDiffusion(pipe_dir, "cpu", scheduler="k_bogus")


def test_img2img_strength(pipe_dir, tmp_path):
    """img2img: strength 0 returns (a VAE round trip of) the source; full strength ignores it."""
    from PIL import Image
    p = StableDiffusion(pipe_dir, "cpu", scheduler="ddim")
    src = Image.new("RGB", (32, 32), (10, 200, 40))
    lo = p("x", "", 32, 32, steps=4, seed=2, image=src, strength=0.0)
    hi = p("x", "", 32, 32, steps=4, seed=2, image=src, strength=1.0)
    txt = p("x", "", 32, 32, steps=4, seed=2)
    assert lo.shape == hi.shape == (32, 32, 3)
    assert not torch.equal(lo, hi) and not torch.equal(lo, txt)


@pytest.mark.gpu
def test_k_sampler_and_img2img_on_gpu(pipe_dir):
    """Sigma-space sampler (fractional timesteps through the captured UNet graph) and img2img on
    the device: seeded runs reproduce, and match the CPU pipeline's layout."""
    from PIL import Image
    g = StableDiffusion(pipe_dir, "cuda:0", scheduler="k_dpmpp_2m")
    a = g("a cat", "", 32, 32, steps=4, seed=7)
    b = g("a cat", "", 32, 32, steps=4, seed=7)
    assert torch.equal(a, b)
    c = StableDiffusion(pipe_dir, "cpu", scheduler="k_dpmpp_2m")("a cat", "", 32, 32, steps=4, seed=7)
    assert (a.float() - c.float()).abs().mean() < 4.0
    src = Image.new("RGB", (32, 32), (10, 200, 40))
    i2i = g("a cat", "", 32, 32, steps=4, seed=7, image=src, strength=0.6)
    assert i2i.shape == (32, 32, 3)


def test_controlnet(pipe_dir, tmp_path):
    """ControlNetModel (diffusers layout) conditioning the UNet: a fresh ControlNet (zero output
    convolutions) leaves the image unchanged exactly; a trained-looking one (random output convs)
    changes it, and the control image matters; weight names follow diffusers
    (controlnet_cond_embedding.*, controlnet_down_blocks.N, controlnet_mid_block)."""
    from PIL import Image

    from localai_amd.models.sd import ControlNet
    ctrl = tmp_path / "ctrl.png"
    Image.fromarray((torch.rand(32, 32, 3) * 255).to(torch.uint8).numpy()).save(ctrl)
    ctrl2 = tmp_path / "ctrl2.png"
    Image.fromarray((torch.rand(32, 32, 3) * 255).to(torch.uint8).numpy()).save(ctrl2)
    base = StableDiffusion(pipe_dir, "cpu")("a cat", "", 32, 32, steps=2, seed=3)
    zdir = synth.write_controlnet(str(tmp_path / "cn-zero"), pipe_dir, zero=True)
    pz = StableDiffusion(pipe_dir, "cpu", controlnet=zdir)
    names = set(pz.controlnet.state_dict())
    n_skips = sum(1 for k in names if k.startswith("controlnet_down_blocks.") and k.endswith(".weight"))
    assert n_skips == 1 + 2 + 1  # conv_in + (resnet, downsampler) + resnet of the 2-level toy UNet
    assert {"controlnet_mid_block.weight", "controlnet_cond_embedding.conv_out.weight"} <= names
    assert not any(k.startswith("up_blocks") for k in names)
    assert torch.equal(pz("a cat", "", 32, 32, steps=2, seed=3, control_image=str(ctrl)), base)
    rdir = synth.write_controlnet(str(tmp_path / "cn-rand"), pipe_dir, zero=False, seed=5)
    pr = StableDiffusion(pipe_dir, "cpu", controlnet=rdir)
    a = pr("a cat", "", 32, 32, steps=2, seed=3, control_image=str(ctrl))
    b = pr("a cat", "", 32, 32, steps=2, seed=3, control_image=str(ctrl2))
    assert not torch.equal(a, base) and not torch.equal(a, b)
    pr.cn_scale = 0.0
    assert torch.equal(pr("a cat", "", 32, 32, steps=2, seed=3, control_image=str(ctrl)), base)
    with pytest.raises(ValueError, match="ControlNet"):
        StableDiffusion(pipe_dir, "cpu")("a cat", "", 32, 32, steps=1, seed=3, control_image=str(ctrl))
    assert isinstance(pr.controlnet, ControlNet)


def test_controlnet_through_backend(pipe_dir, tmp_path):
    from PIL import Image

    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    synth.write_controlnet(os.path.join(os.path.dirname(pipe_dir), "cn-backend"), pipe_dir, zero=False, seed=2)
    ctrl = tmp_path / "pose.png"
    Image.fromarray((torch.rand(32, 32, 3) * 255).to(torch.uint8).numpy()).save(ctrl)
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=pipe_dir, ControlNet="cn-backend"), None)
        assert r.success, r.message
        dst = str(tmp_path / "out.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a dancer", width=32, height=32, step=2,
                                                           seed=4, src=str(ctrl), dst=dst), None)
        assert r.success, r.message
        assert Image.open(dst).size == (32, 32)  # control image, not img2img: the requested size
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=pipe_dir, ControlNet="no-such-controlnet"), None)
        assert not r.success and "ControlNet" in r.message
    asyncio.run(go())


@pytest.mark.gpu
def test_controlnet_on_gpu_graph(pipe_dir, tmp_path):
    from PIL import Image
    cdir = synth.write_controlnet(str(tmp_path / "cn"), pipe_dir, zero=False, seed=5)
    ctrl = tmp_path / "ctrl.png"
    Image.fromarray((torch.rand(32, 32, 3) * 255).to(torch.uint8).numpy()).save(ctrl)
    # deterministic convolution solvers: replays and eager differ only by what the graph changes
    # (MIOpen's default solvers alone moved a pixel by 4 between two otherwise identical runs)
    p = StableDiffusion(pipe_dir, "cuda:0", controlnet=cdir, deterministic=True)
    a = p("a cat", "", 32, 32, steps=3, seed=3, control_image=str(ctrl))
    b = p("a cat", "", 32, 32, steps=3, seed=3, control_image=str(ctrl))
    assert p._graphs and (a.float() - b.float()).abs().max() <= 3
    p.use_graphs = False
    c = p("a cat", "", 32, 32, steps=3, seed=3, control_image=str(ctrl))
    assert (b.float() - c.float()).abs().max() <= 3


def test_depth2img_pipeline(tmp_path):
    """StableDiffusionDepth2ImgPipeline (backend.py:196-198): the DPT depth of the source image,
    on the latent grid and scaled to [-1, 1], is the UNet's fifth input channel; the depth map
    changes the result; no source image is an error; the backend path works."""
    import asyncio

    from PIL import Image

    from localai_amd.grpc import backend_pb as pb
    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    d = synth.write_sd_pipeline(str(tmp_path / "depth"), depth=True)
    p = StableDiffusion(d, "cpu")
    assert p.depth is not None and p.extra_ch == 1 and p.latent_ch == 4
    src = tmp_path / "src.png"
    Image.fromarray((torch.rand(32, 32, 3) * 255).to(torch.uint8).numpy()).save(src)
    dm = p._estimate_depth(str(src), 4, 4)
    assert dm.shape == (1, 1, 4, 4) and float(dm.min()) == -1.0 and float(dm.max()) == 1.0
    a = p("a room", "", 32, 32, steps=3, seed=1, image=str(src), strength=0.9)
    b = p("a room", "", 32, 32, steps=3, seed=1, image=str(src), strength=0.9)
    assert a.shape == (32, 32, 3) and torch.equal(a, b)
    # the depth channel matters: zeroing the estimator's output changes the image
    est = p._estimate_depth
    p._estimate_depth = lambda *a_: torch.zeros_like(est(*a_))
    c = p("a room", "", 32, 32, steps=3, seed=1, image=str(src), strength=0.9)
    assert not torch.equal(a, c)
    p._estimate_depth = est
    with pytest.raises(ValueError, match="source image"):
        p("a room", "", 32, 32, steps=2, seed=1)
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=d, PipelineType="StableDiffusionDepth2ImgPipeline"), None)
        assert r.success, r.message
        dst = str(tmp_path / "o.png")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a room", src=str(src), step=2, seed=3,
                                                           dst=dst), None)
        assert r.success, r.message
        assert Image.open(dst).size == (32, 32)
    asyncio.run(go())


@pytest.mark.gpu
def test_llm_graph_capture_after_diffusion_graphs(pipe_dir, tiny_model_path):
    """A diffusion pipeline's hipGraph captures must leave the CUDA generator usable for later
    captures outside them (an inference_mode capture turned its graph-state tensors into inference
    tensors and every later LLM decode-graph capture in the process failed)."""
    import torch
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    p = StableDiffusion(pipe_dir, "cuda:0")
    p("a cat", "", 32, 32, steps=2, seed=1)
    assert p._graphs
    eng = LLMEngine(EngineConfig(model_path=tiny_model_path, device="cuda:0", context_size=128, max_num_seqs=2,
                                 max_batched_tokens=128, decode_steps=4))
    res = eng.generate("after the unet", SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))
    assert res["completion_tokens"] == 6 and eng._graphs
    torch.randn(4, device="cuda:0")  # the default generator is not left mid-capture
