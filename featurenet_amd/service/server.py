"""REST task service (reference Flask app, ``ui/back/main.py:145-230``).

Routes (same paths and payloads as the reference, port 9999):

* ``POST   /sample/``                               ``{"data": {dataset, max_sampling_time,
  nb_initial_config, max_nb_cells, max_nb_blocks, nb_training_iterations, task_name}}``
  -> creates the task and starts a worker process
* ``GET    /sample/``                               all tasks (+ ``nb_valid_elements``)
* ``GET    /sample/{id}[?full=1]``                  one task (+ ``models`` from the
  ``{N}products.json`` vector list when ``full``)
* ``GET    /sample/{id}/product/{pId}/graph|model`` the candidate's graph (SVG) or
  checkpoint (``.fnk``)
* ``DELETE /sample/``                               drop all tasks
* ``GET    /``                                      a static dashboard (replaces the React SPA)

Built on FastAPI (installed) instead of Flask (not installed); workers are
separate processes (``python -m featurenet_amd.service.worker``).
"""

import json
import os
import re
import subprocess
import sys
from pathlib import Path

from .store import TaskStore

STATIC = Path(__file__).parent / "static"


def _valid_elements(task: dict, count_only: bool = True) -> dict:
    path = task.get("products")
    files = sorted(f for f in os.listdir(path) if f.endswith(".fnk")) if path and os.path.isdir(path) else []
    if count_only:
        task["nb_valid_elements"] = len(files)
    else:
        task["valid_elements"] = files
    return task


def _models(task: dict):
    path, n = task.get("products"), task.get("nb_initial_config")
    f = Path(f"{path}/{n}products.json")
    if not path or not f.is_file():
        return None

    def fmt(v):
        s = v[1][1]
        return {"accuracy": v[0], "name": v[1][0], "nb_blocks": s[0], "nb_layers": s[1], "nb_params": s[2],
                "nb_flops": s[3], "robustness": v[1][2][0]}

    return [fmt(v) for v in json.loads(f.read_text())]


def _file_endswith(folder: str, suffix: str):
    if not folder or not os.path.isdir(folder):
        return None
    for f in sorted(os.listdir(folder)):
        if f.endswith(suffix):
            return os.path.join(folder, f)
    return None


def create_app(db_path: str = "samples.db", base_path: str = "products", devices: str | None = None,
               spawn_workers: bool = True, max_workers: int = 2, cors_origins: list[str] | None = None):
    """``max_workers`` caps concurrently running worker processes (each trains on the
    GPUs); ``cors_origins`` enables CORS for those origins only (default: same origin)."""
    from fastapi import FastAPI, Request
    from fastapi.responses import FileResponse, HTMLResponse, JSONResponse, Response

    from . import fm_builder

    store = TaskStore(db_path)
    app = FastAPI(title="featurenet_amd NAS service")
    if cors_origins:
        from fastapi.middleware.cors import CORSMiddleware

        app.add_middleware(CORSMiddleware, allow_origins=list(cors_origins), allow_methods=["GET", "POST", "DELETE"],
                           allow_headers=["Content-Type"])
    app.state.store = store
    app.state.workers = {}

    def running() -> int:
        return sum(1 for p in app.state.workers.values() if p.poll() is None)

    def start_worker(task_id: str):
        cmd = [sys.executable, "-m", "featurenet_amd.service.worker", task_id, "--db", db_path, "--base", base_path]
        if devices:
            cmd += ["--devices", devices]
        log = open(Path(base_path) / f"worker_{task_id}.log", "w")
        app.state.workers[task_id] = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT,
                                                      cwd=os.getcwd(), start_new_session=True)

    def stop_workers() -> int:
        n = 0
        for p in app.state.workers.values():
            if p.poll() is None:
                p.terminate()                     # the worker's own process only (its session)
                n += 1
        for p in app.state.workers.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        app.state.workers.clear()
        return n

    app.state.stop_workers = stop_workers
    Path(base_path).mkdir(parents=True, exist_ok=True)

    @app.delete("/sample/")
    def sample_delete_all():
        stop_workers()
        return store.delete_all()

    @app.get("/sample/")
    def sample_all():
        return [_valid_elements(t) for t in store.all()]

    @app.get("/sample/{task_id}/product/{pid}/{content}")
    def model_get(task_id: str, pid: str, content: str):
        task = store.get(task_id)
        if task is None:
            return JSONResponse({}, status_code=404)
        if not re.fullmatch(r"[A-Za-z0-9_.-]{1,128}", pid) or ".." in pid:
            return JSONResponse({"error": "bad product id"}, status_code=400)
        if content == "graph":
            f, mime = _file_endswith(task.get("products"), f"{pid}.svg"), "image/svg+xml"
        else:
            f, mime = _file_endswith(task.get("products"), f"{pid}.fnk"), "application/octet-stream"
        if f is None:
            return JSONResponse({})
        return FileResponse(f, media_type=mime)

    @app.get("/sample/{task_id}")
    def sample_get(task_id: str, full: str | None = None):
        task = store.get(task_id)
        if task is None:
            return JSONResponse({}, status_code=404)
        if full:
            task["models"] = _models(task)
        return task

    @app.post("/sample/")
    async def sample_post(request: Request):
        body = await request.json()
        data = body.get("data", body) if isinstance(body, dict) else {}
        if spawn_workers and running() >= max_workers:
            return JSONResponse({"error": f"{max_workers} tasks already running; retry later"}, status_code=429)
        task = store.create(data)
        if spawn_workers:
            start_worker(task["task_id"])
        return task

    @app.get("/fm/catalogue")
    def fm_catalogue():
        """Checkable cell-feature tree of the FM builder (reference ``ui/src/util.js``)."""
        return fm_builder.catalogue()

    @app.post("/fm/build")
    async def fm_build(request: Request):
        """SPLOT XML of the checked cell features (reference ``buildTree``, ``ui/src/pages/fm.js:112-118``)."""
        body = await request.json()
        checked = body.get("checked", []) if isinstance(body, dict) else []
        if not isinstance(checked, list) or not all(isinstance(k, str) for k in checked):
            return JSONResponse({"error": "checked must be a list of catalogue keys"}, status_code=400)
        xml = fm_builder.build_fm(checked)
        return Response(xml, media_type="application/xml",
                        headers={"Content-Disposition": 'attachment; filename="fm.xml"'})

    @app.get("/", response_class=HTMLResponse)
    def index():
        return (STATIC / "index.html").read_text()

    return app


def serve(host: str = "127.0.0.1", port: int = 9999, db_path: str = "samples.db", base_path: str = "products",
          devices: str | None = None, max_workers: int = 2, cors_origins: list[str] | None = None) -> None:
    """Bind to localhost by default: the service has no authentication (as the reference's)."""
    import uvicorn

    uvicorn.run(create_app(db_path, base_path, devices, max_workers=max_workers, cors_origins=cors_origins),
                host=host, port=port)
