"""Task worker: FM expansion -> native PLEDGE sampling -> initial training.

Reference: ``run_fm_generation`` + ``run_featurenet`` (``ui/back/main.py:85-143``),
which fork from the Flask process.  Here the API spawns this module as a
fresh child process (``python -m featurenet_amd.service.worker``): no fork of a
process that may hold a GPU context, and a crashed worker only fails its task.

Status sequence (same strings as the reference): ``init`` -> ``fm_complete``
-> ``sampling_complete`` | ``sampling_failed`` -> ``generation_complete``
(plus ``generation_failed`` when training raises).
"""
from __future__ import annotations

import argparse
import os
import sys
import traceback

from .store import TaskStore


def run_task(store: TaskStore, task_id: str, base_path: str, template: str | None = None, devices=None) -> dict:
    from ..fm.sampler import default_pledge_output, run_pledge
    from ..fm.space import default_template
    from ..search import pledge_evolution as pe
    from ..search.trial import TrialConfig, TrialScheduler

    from .store import safe_name

    task = store.get(task_id)
    root = os.path.realpath(base_path)
    base = os.path.realpath(os.path.join(root, safe_name(task.get("task_name")) or safe_name(task_id)))
    if os.path.commonpath([root, base]) != root or base == root:
        return store.update(task_id, "generation_failed", error="task directory escapes the products root")
    nb = (int(task.get("max_nb_blocks", 5)), int(task.get("max_nb_cells", 5)), int(task.get("nb_initial_config", 10)))
    # the FM template is a server-side choice (the CLI flag), never a client-supplied path
    if not template:
        template = str(default_template(os.path.join(base, "main_1block_nas.xml")))
    fm = pe.end2end(base, nb, template)
    store.update(task_id, "fm_complete", fm=fm)
    out = default_pledge_output(base, nb[2])
    try:
        rc = run_pledge(fm, nb[2], out, duration=float(task.get("max_sampling_time", 30)))
    except Exception as e:  # sampler failure = reference "sampling_failed"
        rc = 1
        store.update(task_id, error=f"{type(e).__name__}: {e}")
    if rc != 0:
        return store.update(task_id, "sampling_failed", pdt=out)
    store.update(task_id, "sampling_complete", pdt=out)
    dataset = task.get("dataset", "mnist")
    products = os.path.join(base, dataset)
    store.update(task_id, products=products)
    try:
        cfg = TrialConfig(dataset=dataset, epochs=int(task.get("nb_training_iterations", 2)),
                          save_dir=products, fill_defaults=True,
                          synthetic_sizes=tuple(task.get("synthetic_sizes", (6000, 1000))))
        with TrialScheduler(devices=devices) as sched:
            pe.run(base, fm, out, nb_base_products=nb[2], dataset=dataset, training_epochs=cfg.epochs,
                   evolution_epochs=int(task.get("nb_evolution_epochs", 0)), attacks=(), scheduler=sched, trial=cfg,
                   pledge_duration_s=float(task.get("max_sampling_time", 30)), verbose=0)
    except Exception as e:
        return store.update(task_id, "generation_failed", error=f"{type(e).__name__}: {e}\n{traceback.format_exc()}")
    return store.update(task_id, "generation_complete")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="featurenet_amd.service.worker")
    ap.add_argument("task_id")
    ap.add_argument("--db", required=True)
    ap.add_argument("--base", default="products")
    ap.add_argument("--template", default=None, help="1-block FM template (default: the built-in search space)")
    ap.add_argument("--devices", default=None, help="comma list, e.g. 0,1 or cpu")
    a = ap.parse_args(argv)
    devices = a.devices.split(",") if a.devices else None
    t = run_task(TaskStore(a.db), a.task_id, a.base, a.template, devices)
    print(f"task {a.task_id}: {t.get('status') if t else 'missing'}", flush=True)
    return 0 if t and not str(t.get("status", "")).endswith("failed") else 1


if __name__ == "__main__":
    sys.exit(main())
