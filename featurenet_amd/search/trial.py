"""Candidate trials and the trial-per-GPU scheduler.

Reference: a candidate is trained by ``TensorflowGenerator`` (build -> train ->
evaluate -> robustness, ``tensorflow_generator.py:97-136``); invalid
architectures, >20M-parameter models and OOM are "dropped" candidates
(``model/keras_model.py:127-156``, ``helpers.py:172-174``).  The reference
trains candidates strictly one after another in one process (its
``multiprocessing`` code is commented out: ``full_mnist.py:37-39``).

Here a trial is a pure function ``run_trial(spec, cfg, device) -> spec`` and
the :class:`TrialScheduler` runs trials concurrently, one worker process per
GPU (8 concurrent candidates on an 8x MI355X node), with

* a per-trial watchdog: a hung or crashed trial kills only its worker, the
  trial is marked ``failed`` and the worker is restarted;
* invalid-candidate semantics: compile errors -> ``status="invalid"``,
  accuracy 0; OOM / non-finite loss -> ``status="failed"``;
* fault-injection hooks for tests (``cfg.inject = {spec_name: "build" | "oom" |
  "hang" | "crash" | "device"}``; "device": a HIP runtime error that poisons the
  worker's context -- the trial fails and the worker is replaced).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import time
import traceback
from dataclasses import asdict, dataclass, field

from ..ir.spec import ModelSpec


@dataclass
class TrialConfig:
    dataset: str = "cifar"
    epochs: int = 12
    batch_size: int = 64
    lr: float = 1e-3
    attacks: list = field(default_factory=list)
    robustness_set_size: int = 500
    clever_samples: int | None = 20
    augment: bool = False
    compat: bool = True
    fill_defaults: bool = False
    save_dir: str | None = None
    save_prefix: str = ""
    seed: int = 0
    synthetic_sizes: tuple = (6000, 1000)
    verbose: int = 0
    inject: dict = field(default_factory=dict)
    graph: bool = True          # hipGraph-captured training steps on GPU (launch-bound small candidates)

    def to_dict(self) -> dict:
        return asdict(self)


def run_trial(spec: ModelSpec, cfg: TrialConfig, device=None) -> ModelSpec:
    """Train + evaluate one candidate in this process; never raises."""
    import torch

    from ..ir.compile import CompileError, compile_model
    from ..training.callbacks import reference_callbacks
    from ..training.data import load_dataset
    from ..training.trainer import Trainer, TrainingFailed

    spec = spec.clone()
    t0 = time.time()
    fault = cfg.inject.get(spec.name) if cfg.inject else None
    try:
        if fault == "hang":
            time.sleep(3600)
        if fault == "crash":
            os._exit(17)
        ds = load_dataset(cfg.dataset, synthetic_sizes=tuple(cfg.synthetic_sizes), seed=cfg.seed)
        torch.manual_seed(cfg.seed)
        if fault == "build":
            raise CompileError("injected build failure")
        model = compile_model(spec, ds.input_shape, ds.num_classes, compat=cfg.compat,
                              fill_defaults=cfg.fill_defaults)
        spec.nb_params, spec.nb_layers, spec.nb_flops = model.nb_params, model.nb_layers, model.flops_per_sample
        if fault == "oom":
            raise TrainingFailed("out of device memory: injected")
        if fault == "device":
            raise RuntimeError("HIP error: an illegal memory access was encountered (injected)")
        trainer = Trainer(model, lr=cfg.lr, device=device, graph=cfg.graph, meta={"model_kind": "candidate", "spec": spec.to_dict(),
                                                                  "input_shape": list(ds.input_shape),
                                                                  "num_classes": ds.num_classes,
                                                                  "compat": cfg.compat,
                                                                  "fill_defaults": cfg.fill_defaults})
        packed = ds.input_shape[0] if ds.packed else None
        hist = trainer.fit(ds.x_train, ds.y_train, epochs=cfg.epochs, batch_size=cfg.batch_size,
                           validation_data=(ds.x_test, ds.y_test), callbacks=reference_callbacks(False),
                           augment=cfg.augment, packed_size=packed, verbose=cfg.verbose, seed=cfg.seed)
        loss, acc = trainer.evaluate(ds.x_test, ds.y_test, packed_size=packed)
        spec.accuracy = float(acc)
        spec.history = {k: [float(v) for v in vs] for k, vs in hist.history.items()}
        spec.status = "trained"
        if cfg.attacks and acc >= 0.5:
            from ..robust.evaluate import eval_robustness

            r = eval_robustness(model, ds, list(cfg.attacks), set_size=cfg.robustness_set_size,
                                clever_samples=cfg.clever_samples)
            spec.robustness_score = float(r.get("score", 0.0))
            for k in ("clever", "fgsm", "pgd", "cw"):
                if r.get(k) is not None:
                    setattr(spec, f"{k}_score", list(r[k]) if isinstance(r[k], tuple) else r[k])
        if cfg.save_dir:
            os.makedirs(cfg.save_dir, exist_ok=True)
            trainer.meta["spec"] = spec.to_dict()
            trainer.save(os.path.join(cfg.save_dir, f"{cfg.save_prefix}{spec.name}.fnk"))
            from ..utils.graph import to_svg

            with open(os.path.join(cfg.save_dir, f"{cfg.save_prefix}{spec.name}.svg"), "w") as f:
                f.write(to_svg(model))
    except CompileError as e:
        spec.status, spec.accuracy, spec.error = "invalid", 0.0, str(e)
    except TrainingFailed as e:
        spec.status, spec.accuracy, spec.error = "failed", 0.0, str(e)
    except Exception as e:  # any other failure drops the candidate, like the reference
        spec.status, spec.accuracy, spec.error = "failed", 0.0, f"{type(e).__name__}: {e}\n{traceback.format_exc(limit=4)}"
    spec.metrics = list(spec.metrics) + [{"trial_time_s": time.time() - t0}]
    from ..utils.events import default_log

    default_log().emit("trial", name=spec.name, status=spec.status, accuracy=spec.accuracy,
                       params=spec.nb_params, seconds=time.time() - t0, device=str(device))
    return spec


# ---------------------------------------------------------------------------
# process pool
# ---------------------------------------------------------------------------
# Error texts of a device runtime failure that leaves the process's HIP context unusable
# (a faulting kernel, a device-side assert, a lost device): every later trial in that process
# would fail the same way, so the worker reports the trial and exits, and the pool replaces it.
_POISON_MARKERS = ("hip error", "hiperror", "cuda error", "device-side assert", "illegal memory access",
                   "memory access fault", "hsa_status", "unspecified launch failure", "device lost")


def device_poisoned(error: str | None) -> bool:
    """True when a trial's error text names a device runtime failure (see ``_POISON_MARKERS``)."""
    e = (error or "").lower()
    return any(m in e for m in _POISON_MARKERS)


def _worker(dev: str, tasks, results, ready):
    os.environ.setdefault("OMP_NUM_THREADS", "4")
    import torch

    device = "cpu"
    if dev != "cpu":
        torch.cuda.set_device(int(dev))
        device = f"cuda:{int(dev)}"
    ready.put(os.getpid())
    while True:
        item = tasks.get()
        if item is None:
            return
        tid, spec_json, cfg = item
        out = run_trial(ModelSpec.from_json(spec_json), TrialConfig(**cfg), device)
        leaving = out.status == "failed" and device_poisoned(out.error)
        results.put((tid, out.to_json(), leaving))
        if leaving:
            # the context is gone for every later trial: flush the result, then leave with a
            # non-zero code (the result says so: the scheduler starts a fresh worker right away)
            results.close()
            results.join_thread()
            os._exit(3)


class TrialScheduler:
    """Run trials on a set of devices: ``workers_per_device`` worker processes per device
    (several small candidates share one MI355X: each worker trains its own trial, the GPU
    interleaves their kernels).  A device may also be listed more than once.

    ``persistent`` (default): the worker processes outlive a :meth:`map` call and serve the next
    one -- an evolution calls ``map`` once per generation, and each fresh worker pays process
    spawn, ``import torch``, HIP initialisation and the first candidate's kernel tables (~2 s of a
    32-candidate generation at 4 workers per GPU).  :meth:`close` (or the context manager, or the
    interpreter's exit: the workers are daemons) ends them."""

    def __init__(self, devices=None, timeout_s: float | None = None, mode: str = "auto", workers_per_device: int = 1,
                 persistent: bool = True):
        if devices is None:
            try:
                import torch

                n = torch.cuda.device_count()
            except Exception:
                n = 0
            devices = [str(i) for i in range(n)] or ["cpu"]
        self.devices = [str(d) for d in devices]
        self.timeout_s = timeout_s
        self.workers_per_device = max(1, int(workers_per_device))
        single = len(self.devices) == 1 and self.workers_per_device == 1
        self.mode = ("inline" if single and timeout_s is None else "process") if mode == "auto" else mode
        self.persistent = bool(persistent)
        self._workers: dict[str, dict] = {}      # the live pool (persistent mode)
        self._retired: list[dict] = []           # replaced workers' queues, kept referenced
        self._next_tid = 0                       # task ids unique across map calls

    def __enter__(self):
        return self

    def __del__(self):
        # (a scheduler dropped without close() -- e.g. the one a search function made for itself
        # -- takes its workers with it)
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown: the daemons end anyway
            pass

    def __exit__(self, *exc):
        self.close()
        return False

    def pids(self) -> list[int]:
        """PIDs of the live worker processes (persistent mode)."""
        return [w["proc"].pid for w in self._workers.values() if w["proc"].is_alive()]

    def close(self):
        """End the worker processes (they finish the task they hold first)."""
        workers, self._workers = self._workers, {}
        for w in workers.values():
            try:
                w["tasks"].put(None)
            except Exception:  # noqa: BLE001 - a broken queue: the process is killed below
                pass
        for w in workers.values():
            w["proc"].join(timeout=30)
            if w["proc"].is_alive():
                w["proc"].kill()
        self._retired.clear()

    def slots(self) -> list[tuple[str, str]]:
        """(worker key, device) of every worker process."""
        return [(f"{d}/{i}/{k}", d) for i, d in enumerate(self.devices) for k in range(self.workers_per_device)]

    def map(self, specs: list[ModelSpec], cfg: TrialConfig) -> list[ModelSpec]:
        if not specs:
            return []
        if self.mode == "inline":
            dev = self.devices[0]
            device = "cpu" if dev == "cpu" else f"cuda:{int(dev)}"
            return [run_trial(s, cfg, device) for s in specs]
        return self._map_processes(specs, cfg)

    def _spawn(self, key: str, workers: dict) -> None:
        ctx = mp.get_context("spawn")
        # every worker gets its OWN result queue, replaced with the worker: killing a
        # process while it writes a shared multiprocessing.Queue can corrupt that queue
        tq = ctx.Queue()
        rq = ctx.Queue()
        ready = ctx.Queue()
        p = ctx.Process(target=_worker, args=(dict(self.slots())[key], tq, rq, ready), daemon=True)
        p.start()
        # keep every queue referenced: a collected queue unlinks its semaphore
        # before the spawned child has unpickled it
        if key in workers:
            self._retired.append(workers[key])
        workers[key] = {"proc": p, "tasks": tq, "results": rq, "ready": ready, "busy": None, "t0": 0.0}

    def start(self) -> "TrialScheduler":
        """Spawn the worker pool now (persistent process mode), so that its start-up -- process
        spawn, ``import torch``, HIP initialisation -- overlaps the caller's own preparation
        (product sampling, model specs) instead of the first generation."""
        if self.mode == "process" and self.persistent:
            for key, _ in self.slots():
                w = self._workers.get(key)
                if w is None or not w["proc"].is_alive():
                    self._spawn(key, self._workers)
        return self

    def _map_processes(self, specs, cfg):
        workers = self._workers if self.persistent else {}
        retired = self._retired

        def start(key):
            self._spawn(key, workers)

        for key, _ in self.slots():
            if key not in workers or not workers[key]["proc"].is_alive():
                start(key)
        base = self._next_tid
        self._next_tid += len(specs)
        pending = [(base + i, s) for i, s in enumerate(specs)]
        out: dict[int, ModelSpec] = {}
        cfgd = cfg.to_dict()
        finished = False
        try:
            while len(out) < len(specs):
                for key in list(workers):
                    w = workers[key]
                    if w["busy"] is None and pending:
                        if not w["proc"].is_alive():       # (a worker that left after reporting a
                            start(key)                       # device failure: a fresh one takes the task)
                            w = workers[key]
                        tid, s = pending.pop(0)
                        w["busy"], w["t0"] = tid, time.time()
                        w["tasks"].put((tid, s.to_json(), cfgd))
                got = False
                for key in list(workers):
                    w = workers[key]
                    try:
                        tid, js, leaving = w["results"].get_nowait()
                    except queue.Empty:
                        continue
                    got = True
                    # only the trial this worker is running, of this call, counts: a result that
                    # arrives after the watchdog already failed (and restarted) it is dropped
                    if w["busy"] == tid and base <= tid < base + len(specs) and tid not in out:
                        out[tid] = ModelSpec.from_json(js)
                        w["busy"] = None
                    if leaving:                          # (its device context is gone: replace it)
                        w["proc"].join(timeout=30)
                        if w["proc"].is_alive():
                            w["proc"].kill()
                            w["proc"].join(timeout=10)
                        w["busy"] = None
                        start(key)
                if not got:
                    time.sleep(0.05)
                # watchdog: hung or dead workers fail their trial and are restarted
                for key in list(workers):
                    w = workers[key]
                    tid = w["busy"]
                    if tid is None:
                        continue
                    dead = not w["proc"].is_alive()
                    hung = self.timeout_s is not None and time.time() - w["t0"] > self.timeout_s
                    if dead or hung:
                        if dead:                          # (its result may have landed just before
                            try:                          #  it exited: take it if so)
                                rtid, js, _ = w["results"].get(timeout=0.5)
                                if rtid == tid and tid not in out:
                                    out[tid] = ModelSpec.from_json(js)
                            except queue.Empty:
                                pass
                        if not dead:
                            w["proc"].kill()
                        w["proc"].join(timeout=10)
                        if tid not in out:
                            s = specs[tid - base].clone()
                            s.status, s.accuracy = "failed", 0.0
                            s.error = "trial timed out" if hung else f"worker died (exit {w['proc'].exitcode})"
                            out[tid] = s
                        start(key)
            finished = True
        finally:
            if not finished:
                # abnormal exit (KeyboardInterrupt, a bad result, ...): a worker still busy with a
                # task of this call would later report into the next call -- end it, so the next
                # map() starts a fresh one
                for key in list(workers):
                    w = workers[key]
                    if w["busy"] is not None:
                        w["proc"].kill()
                        w["proc"].join(timeout=10)
                        w["busy"] = None
        if not self.persistent:
            for w in workers.values():
                w["tasks"].put(None)
            for w in workers.values():
                w["proc"].join(timeout=30)
                if w["proc"].is_alive():
                    w["proc"].kill()
            retired.clear()
        return [out[base + i] for i in range(len(specs))]
