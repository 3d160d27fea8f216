"""`diffusers` / `stablediffusion` backend servicer (backend.proto LoadModel + GenerateImage) over
the native Stable Diffusion 1.x / 2.x / XL pipeline (models/sd.py), FLUX.1 (models/flux.py,
`pipeline_type: FluxPipeline` or a FluxPipeline model_index.json) and Stable Diffusion 3
(models/sd3.py, `pipeline_type: StableDiffusion3Pipeline`), text-to-video
(models/video.py, `pipeline_type: VideoDiffusionPipeline` or a TextToVideoSDPipeline
model_index.json) and image-to-video (models/svd.py, `pipeline_type: StableVideoDiffusionPipeline`).

Mirrors `backend/python/diffusers/backend.py`: LoadModel keeps `CFGScale` (7 when unset),
`CLIPSkip` and `SchedulerType`; GenerateImage uses `step` (1 when unset), width / height,
`negative_prompt`, seeds its generator when `seed > 0`, and honours `EnableParameters` (a comma
list naming which of negative_prompt / width / height / num_inference_steps reach the pipeline,
"none" for none of them -- the rest take the pipeline defaults: sample_size * 8 pixels, 50 steps).
`src` makes the call img2img (strength 0.8, the diffusers default) -- or, when LoadModel named a
`ControlNet` (a ControlNetModel directory, relative to the pipeline's parent directory), the
control image of a ControlNet-conditioned txt2img (backend.py:292-296, 403-405); `LoraAdapter` (relative to
the model file's directory) is merged into the UNet / text encoders at load (models/sd_lora.py,
backend.py:300-314; `LoraScale` when set, else 1); `SchedulerType` takes every
scheduler name of the reference's mapping (models/schedulers.py).  One image at a time (the
reference runs one gRPC worker per backend).
"""
from __future__ import annotations

import asyncio
import os
import threading

from . import backend_pb as pb


class DiffusersServicer:
    def __init__(self, device: str = ""):
        self.device = device
        self.pipe = None
        self.cfg_scale = 7.0
        self.state = pb.StatusResponse.UNINITIALIZED
        self._lock = threading.Lock()

    async def Health(self, request, context=None):
        return pb.Reply(message=b"OK")

    async def Status(self, request, context=None):
        return pb.StatusResponse(state=self.state)

    async def LoadModel(self, request, context=None):
        from ..models.flux import FluxPipeline, is_flux_pipeline
        from ..models.sd import StableDiffusion, is_sd_pipeline
        from ..models.sd3 import SD3Pipeline, is_sd3_pipeline
        path = request.ModelFile or request.Model
        from ..models import sd_single_file as ssf
        flux_file = None
        if str(request.PipelineType or "") == "FluxTransformer2DModel":
            # backend.py:255-269: the transformer from the single file, everything else from
            # BFL_REPO (here a local diffusers FLUX directory: there is no hub to fetch from)
            base = os.environ.get("BFL_REPO", "")
            if not os.path.isabs(base) and base:
                base = os.path.join(os.path.dirname(os.path.abspath(path)), base)
            if not ssf.is_single_file(path):
                return pb.Result(success=False, message=f"FluxTransformer2DModel needs a single-file transformer: {path}")
            if not (base and is_flux_pipeline(base)):
                return pb.Result(success=False, message="FluxTransformer2DModel: set BFL_REPO to a local diffusers "
                                                        f"FLUX pipeline directory (got {base!r})")
            flux_file, path = path, base
        elif ssf.is_single_file(path):
            # backend.py:184-191: a local file is a from_single_file checkpoint (SD 1.x / 2.x / XL)
            clip = str(request.CLIPModel or "")
            if clip and not os.path.isabs(clip):
                clip = os.path.join(os.path.dirname(os.path.abspath(path)), clip)
            try:
                path = await asyncio.get_running_loop().run_in_executor(
                    None, lambda: ssf.convert(path, tokenizer_dir=clip if os.path.isdir(clip) else None))
            except Exception as e:  # noqa: BLE001
                return pb.Result(success=False, message=f"single-file checkpoint: {e}")
        flux = is_flux_pipeline(path) or str(request.PipelineType or "").startswith("Flux")
        sd3 = is_sd3_pipeline(path) or str(request.PipelineType or "") == "StableDiffusion3Pipeline"
        from ..models.svd import StableVideoDiffusion, is_svd_pipeline
        from ..models.video import TextToVideo, is_video_pipeline
        # backend.py:223-226: VideoDiffusionPipeline = a text-to-video DiffusionPipeline
        t2v = is_video_pipeline(path) or str(request.PipelineType or "") == "VideoDiffusionPipeline"
        if t2v and not is_video_pipeline(path):
            return pb.Result(success=False, message=f"VideoDiffusionPipeline needs a TextToVideoSDPipeline directory: {path}")
        # backend.py:199-205: StableVideoDiffusionPipeline (img2vid)
        i2v = is_svd_pipeline(path) or str(request.PipelineType or "") == "StableVideoDiffusionPipeline"
        if i2v and not is_svd_pipeline(path):
            return pb.Result(success=False, message=f"StableVideoDiffusionPipeline directory expected: {path}")
        if not (t2v or i2v or is_sd_pipeline(path) or ((flux or sd3) and os.path.isdir(path))):
            return pb.Result(success=False, message=f"not a diffusers pipeline directory: {path}")
        dev = self.device
        if not dev:
            import torch
            dev = "cuda:0" if torch.cuda.is_available() else "cpu"
        cn = str(request.ControlNet or "")
        if cn and not os.path.isabs(cn) and not os.path.isdir(cn):
            cn = os.path.join(os.path.dirname(os.path.normpath(path)), cn)  # next to the pipeline directory
        if cn and not os.path.isfile(os.path.join(cn, "config.json")):
            return pb.Result(success=False, message=f"ControlNet model not found: {request.ControlNet}")
        lora = str(request.LoraAdapter or "")
        if lora and not os.path.isabs(lora):
            # backend.py:300-305: relative to the model file's directory
            lora = os.path.join(os.path.dirname(request.ModelFile or path.rstrip("/")), lora)
        if lora and not os.path.exists(lora):
            return pb.Result(success=False, message=f"LoRA adapter not found: {request.LoraAdapter}")
        if lora and (flux or sd3):
            return pb.Result(success=False, message="LoRA adapters are supported for SD 1.x / 2.x / XL pipelines")
        try:
            if t2v:
                p = await asyncio.get_running_loop().run_in_executor(None, lambda: TextToVideo(path, dev))
            elif i2v:
                p = await asyncio.get_running_loop().run_in_executor(None, lambda: StableVideoDiffusion(path, dev))
            elif flux:  # backend.py:247-251: FluxPipeline; GenerateImage adds max_sequence_length=256
                p = await asyncio.get_running_loop().run_in_executor(
                    None, lambda: FluxPipeline(path, dev, max_sequence_length=256, transformer_file=flux_file))
            elif sd3:  # backend.py:235-246: StableDiffusion3Pipeline
                p = await asyncio.get_running_loop().run_in_executor(
                    None, lambda: SD3Pipeline(path, dev, clip_skip=int(request.CLIPSkip or 0)))
            else:
                p = await asyncio.get_running_loop().run_in_executor(
                    None, lambda: StableDiffusion(path, dev, request.SchedulerType, int(request.CLIPSkip or 0),
                                                  controlnet=cn, lora=lora,
                                                  lora_scale=float(request.LoraScale) if request.LoraScale else 1.0))
        except Exception as e:  # noqa: BLE001 - reported to the caller like the reference
            return pb.Result(success=False, message=f"Unexpected {e!r}")
        self.pipe, self.state = p, pb.StatusResponse.READY
        self.cfg_scale = float(request.CFGScale) if request.CFGScale else 7.0
        return pb.Result(success=True, message="Model loaded successfully")

    def shutdown(self):
        self.pipe, self.state = None, pb.StatusResponse.UNINITIALIZED

    def _generate(self, request):
        p = self.pipe
        if p is None:
            raise RuntimeError("no model loaded")
        from ..models.svd import StableVideoDiffusion
        from ..models.video import TextToVideo, export_video
        if isinstance(p, StableVideoDiffusion):
            # backend.py:435-443: src resized to 1024 x 576, guidance cfg_scale (the top of the
            # per-frame ramp), decode_chunk_size CHUNK_SIZE (8), export_to_video at FPS (7)
            if not request.src:
                raise ValueError("StableVideoDiffusionPipeline needs a source image (src)")
            fps = int(os.environ.get("FPS", "7"))
            with self._lock:
                v = p(request.src, request.width or 1024, request.height or 576, steps=int(request.step or 25),
                      max_guidance_scale=self.cfg_scale, fps=fps,
                      decode_chunk_size=int(os.environ.get("CHUNK_SIZE", "8")),
                      seed=request.seed if request.seed > 0 else None)
                export_video(v, request.dst, fps)
            return
        if isinstance(p, TextToVideo):
            # backend.py:445-448: num_frames = FRAMES (64), num_inference_steps = step, guidance
            # cfg_scale; export_to_video at FPS (7)
            frames = int(os.environ.get("FRAMES", "64"))
            fps = int(os.environ.get("FPS", "7"))
            with self._lock:
                v = p(request.positive_prompt, request.negative_prompt or "", request.width or 256,
                      request.height or 256, num_frames=frames, steps=int(request.step or 25),
                      guidance_scale=self.cfg_scale, seed=request.seed if request.seed > 0 else None)
                export_video(v, request.dst, fps)
            return
        default_px = p.unet_sample_size * p.vae_scale
        options = {"negative_prompt": request.negative_prompt, "width": request.width, "height": request.height,
                   "num_inference_steps": request.step if request.step else 1}
        keys = list(options)
        if request.EnableParameters:
            keys = [] if request.EnableParameters == "none" else [k.strip() for k in request.EnableParameters.split(",")]
        kw = {k: options[k] for k in keys if k in options}
        w = int(kw.get("width") or default_px)
        h = int(kw.get("height") or default_px)
        image = request.src or None   # backend.py: options["image"] = Image.open(request.src) -> img2img
        control = None
        if image is not None and getattr(p, "controlnet", None) is not None:
            control, image = image, None  # backend.py:403: with a ControlNet, src is the control image
        if image is not None:
            # the reference passes width / height only when asked; img2img keeps the source's size otherwise
            w = int(kw["width"]) if kw.get("width") else 0
            h = int(kw["height"]) if kw.get("height") else 0
        with self._lock:
            extra = {"image": image, "control_image": control} if image is not None or control is not None else {}
            img = p(request.positive_prompt, kw.get("negative_prompt", ""), w, h,
                    steps=int(kw.get("num_inference_steps", 50)), guidance_scale=self.cfg_scale,
                    seed=request.seed if request.seed > 0 else None, **extra)
            p.save(img, request.dst)

    async def GenerateImage(self, request, context=None):
        try:
            await asyncio.get_running_loop().run_in_executor(None, self._generate, request)
        except (ValueError, OSError) as e:
            return pb.Result(success=False, message=f"Unexpected {e!r}")
        return pb.Result(message="Media generated", success=True)
