"""Model gallery endpoints (`core/http/endpoints/localai/gallery.go`, routes/localai.go:22-34)."""
from __future__ import annotations

from fastapi import APIRouter, Request
from fastapi.responses import JSONResponse

from .. import gallery as gal
from ..config.loader import LoadOptions


def build_router(state) -> APIRouter:
    r = APIRouter()

    def reload():
        state.configs.load_from_path(state.models_path, state.load_options())
        try:
            state.configs.preload(state.models_path)
        except Exception:
            pass

    svc = gal.GalleryService(state.cfg, on_change=reload)
    state.gallery = svc

    async def apply(request: Request):
        b = await request.json()
        req = gal.GalleryModel.from_dict(b)
        op = gal.GalleryOp(id=gal.new_op_id(), gallery_model_name=b.get("id", ""),
                           config_url=b.get("config_url", "") or b.get("url", ""),
                           req=req, galleries=list(state.cfg.galleries))
        svc.submit(op)
        base = str(request.base_url).rstrip("/")
        return {"uuid": op.id, "status": f"{base}/models/jobs/{op.id}"}

    async def delete(name: str, request: Request):
        op = gal.GalleryOp(id=gal.new_op_id(), gallery_model_name=name, delete=True)
        svc.submit(op)
        state.configs.remove(name)
        base = str(request.base_url).rstrip("/")
        return {"uuid": op.id, "status": f"{base}/models/jobs/{op.id}"}

    async def available():
        models = gal.available_models(state.cfg.galleries, state.models_path)
        return [m.to_json() for m in models]

    async def list_galleries():
        return state.cfg.galleries

    async def add_gallery(request: Request):
        g = await request.json()
        if any(x.get("name") == g.get("name") for x in state.cfg.galleries):
            return JSONResponse({"error": {"message": "gallery already exists", "code": 500}}, status_code=500)
        state.cfg.galleries.append({"name": g.get("name", ""), "url": g.get("url", "")})
        return state.cfg.galleries

    async def remove_gallery(request: Request):
        g = await request.json()
        before = len(state.cfg.galleries)
        state.cfg.galleries[:] = [x for x in state.cfg.galleries if x.get("name") != g.get("name")]
        if len(state.cfg.galleries) == before:
            return JSONResponse({"error": {"message": "gallery not found", "code": 500}}, status_code=500)
        return state.cfg.galleries

    async def job(uuid: str):
        st = svc.get(uuid)
        if st is None:
            return JSONResponse({"error": {"message": "could not find any status for ID", "code": 500}},
                                status_code=500)
        return st

    async def jobs():
        return svc.all()

    r.add_api_route("/models/apply", apply, methods=["POST"])
    r.add_api_route("/models/delete/{name}", delete, methods=["POST"])
    r.add_api_route("/models/available", available, methods=["GET"])
    r.add_api_route("/models/galleries", list_galleries, methods=["GET"])
    r.add_api_route("/models/galleries", add_gallery, methods=["POST"])
    r.add_api_route("/models/galleries", remove_gallery, methods=["DELETE"])
    r.add_api_route("/models/jobs/{uuid}", job, methods=["GET"])
    r.add_api_route("/models/jobs", jobs, methods=["GET"])
    return r
