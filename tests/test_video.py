"""Text-to-video (models/video.py, the reference's VideoDiffusionPipeline path,
backend/python/diffusers/backend.py:223-226 / 445-448) on a random-init UNet3DConditionModel
pipeline from synth.write_t2v_pipeline: every tensor loads strictly under its diffusers name,
frames are deterministic per seed and coupled through the temporal layers (a frame's content
depends on its neighbours), the video files are readable, and the diffusers servicer serves it.
Parity with diffusers' TextToVideoSDPipeline is unpinned (diffusers is not installed)."""
import asyncio
import os

import pytest
import torch

from localai_amd.grpc import backend_pb as pb
from localai_amd.models import synth
from localai_amd.models.video import TextToVideo, export_video, is_video_pipeline, read_avi_frames


@pytest.fixture(scope="module")
def t2v_dir(tmp_path_factory):
    return synth.write_t2v_pipeline(str(tmp_path_factory.mktemp("t2v") / "t2v-tiny"))


def test_frames_deterministic_and_temporally_coupled(t2v_dir):
    assert is_video_pipeline(t2v_dir)
    p = TextToVideo(t2v_dir, "cpu")
    a = p("a red car", "", 64, 64, num_frames=5, steps=2, guidance_scale=9.0, seed=3)
    b = p("a red car", "", 64, 64, num_frames=5, steps=2, guidance_scale=9.0, seed=3)
    assert a.shape == (5, 64, 64, 3) and a.dtype == torch.uint8 and torch.equal(a, b)
    # the temporal convolutions / attentions couple the frames: with the temporal layers zeroed the
    # same latents give different frames
    with torch.no_grad():
        for n, prm in p.unet.named_parameters():
            if (".temp_convs." in n and ".conv4.3." in n) or (".temp_attentions." in n and "proj_out" in n) \
                    or n.startswith("transformer_in.proj_out"):
                prm.zero_()
    c = p("a red car", "", 64, 64, num_frames=5, steps=2, guidance_scale=9.0, seed=3)
    assert not torch.equal(a, c)


def test_video_files(t2v_dir, tmp_path):
    from PIL import Image
    v = torch.randint(0, 255, (4, 32, 48, 3), dtype=torch.uint8)
    export_video(v, str(tmp_path / "v.gif"), 7)
    assert Image.open(str(tmp_path / "v.gif")).n_frames == 4
    export_video(v, str(tmp_path / "v.mp4"), 7)
    data = open(str(tmp_path / "v.mp4"), "rb").read()
    assert data[:4] == b"RIFF" and data[8:12] == b"AVI "
    jpgs = read_avi_frames(str(tmp_path / "v.mp4"))
    assert len(jpgs) == 4 and all(j[:2] == b"\xff\xd8" for j in jpgs)
    import io
    assert Image.open(io.BytesIO(jpgs[2])).size == (48, 32)


def test_servicer_video_diffusion_pipeline(t2v_dir, tmp_path, monkeypatch):
    from localai_amd.grpc.diffusers_servicer import DiffusersServicer
    monkeypatch.setenv("FRAMES", "3")
    sv = DiffusersServicer(device="cpu")

    async def go():
        r = await sv.LoadModel(pb.ModelOptions(ModelFile=t2v_dir, PipelineType="VideoDiffusionPipeline"), None)
        assert r.success, r.message
        dst = str(tmp_path / "out.gif")
        r = await sv.GenerateImage(pb.GenerateImageRequest(positive_prompt="a lighthouse", width=32, height=32, step=2,
                                                           seed=5, dst=dst), None)
        assert r.success, r.message
        from PIL import Image
        im = Image.open(dst)
        assert im.n_frames == 3 and im.size == (32, 32)
        bad = await sv.LoadModel(pb.ModelOptions(ModelFile=str(tmp_path), PipelineType="VideoDiffusionPipeline"), None)
        assert not bad.success
    asyncio.run(go())


@pytest.mark.gpu
def test_unet3d_gpu_bf16_matches_cpu_fp32(t2v_dir):
    """One UNet3D evaluation on the GPU (bf16, the fused GroupNorm kernels on the 2-D layers) vs
    the fp32 CPU module: relative L2 of the noise prediction."""
    gpu, cpu = TextToVideo(t2v_dir, "cuda:0"), TextToVideo(t2v_dir, "cpu")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 5, 8, 8, generator=g)
    ctx = torch.randn(2, 77, 32, generator=g)
    t = torch.tensor([500.0, 500.0])
    a = gpu.unet(x.cuda().to(torch.bfloat16), t.cuda(), ctx.cuda().to(torch.bfloat16)).float().cpu()
    b = cpu.unet(x, t, ctx)
    rel = float((a - b).norm() / b.norm())
    assert rel < 5e-2, rel
    v = gpu("a red car", "", 64, 64, num_frames=4, steps=2, guidance_scale=9.0, seed=3)
    assert v.shape == (4, 64, 64, 3)
