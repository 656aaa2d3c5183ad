"""Command line: ``python -m featurenet_amd <command> ...``.

========== =================================================================
command    reference equivalent
========== =================================================================
run        ``run.py`` (-n BxCxN -t -b -f -a -i -p -d -m -g -r -s -e -y -l)
pledge     ``pledge_evolution.py`` (-n -d -b -i -o -p -t)
products   ``full.py`` / ``full_mnist.py`` / ``full_cifar.py`` (-i -d -t)
retrain    ``pledge_trainer.py`` (-p -j -i -e -t -b -d)
ga         ``evolution.py`` (-i -o)
resume     ``utils/retrainer.py`` (continue training a checkpoint)
serve      ``ui/back/main.py`` (REST task service, port 9999)
train      ``TensorflowGenerator(...)`` one architecture (template / product /
           featurenet3d) -> checkpoint
classify   load a checkpoint and predict (npy / binvox folder)
extend     ``PledgeEvolution.end2end`` (FM template -> B x C)
sample     ``run_pledge`` (native diverse product sampler)
template   write the built-in 1-block search-space FM
========== =================================================================
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from .config import SearchConfig


def _scheduler(devices: str, timeout: float, workers_per_device: int = 0):
    """Trial scheduler over ``devices``; ``workers_per_device`` 0 = auto: 4 worker processes per GPU
    (the candidates' small kernels from 4 processes keep one MI355X busy: 12.5K -> 19.7K candidates
    per hour against 7.8K for one worker, profiles/r5_nas.md), one trial at a time on the CPU."""
    from .search.trial import TrialScheduler

    devs = [d for d in devices.split(",") if d] if devices else None
    if workers_per_device <= 0:
        probe = TrialScheduler(devices=devs, mode="inline")
        workers_per_device = 1 if probe.devices == ["cpu"] else 4
    return TrialScheduler(devices=devs, timeout_s=timeout or None, workers_per_device=workers_per_device)


def _template(base: str, fm_path: str) -> str:
    if fm_path:
        return fm_path
    from .fm.space import default_template

    return str(default_template(os.path.join(base, "main_1block_nas.xml")))


# ---------------------------------------------------------------------- run
def cmd_run(a) -> int:
    from .fm.sampler import run_pledge
    from .search.evolution import run_evolution
    from .search.mutation import MutationStrategies, SelectionStrategies
    from .search.pledge_evolution import end2end
    from .search.trial import TrialConfig

    cfg = SearchConfig.load(a.config) if a.config else SearchConfig()
    for k in ("nb", "training_epochs", "base_path", "fm_path", "pledge_duration", "products_file", "dataset",
              "mutation_strategy", "selection_strategy", "mutation_rate", "survival_rate", "evolution_epochs",
              "model", "devices", "seed", "workers_per_device"):
        v = getattr(a, k, None)
        if v is not None:
            setattr(cfg, k, v)
    if a.breed is not None:
        cfg.breed = a.breed not in ("0", "false", "False", "")
    nb = cfg.nb_tuple
    # the trial worker pool starts now: its start-up overlaps the product sampling below
    sched = _scheduler(cfg.devices, cfg.trial_timeout_s, cfg.workers_per_device).start()
    ms = MutationStrategies.ALL if cfg.mutation_strategy == "all" else MutationStrategies.CHOICE
    ss = {"pareto": SelectionStrategies.PARETO, "elitist": SelectionStrategies.ELITIST,
          "hybrid": SelectionStrategies.HYBRID}[cfg.selection_strategy]
    products = cfg.products_file
    if len(nb) == 3 and not products:
        blocks, cells, n = nb
        os.makedirs(cfg.base_path, exist_ok=True)
        products = f"{cfg.base_path}/products_{int(cfg.pledge_duration)}s_{blocks}_{cells}_{n}.pdt"
        if not os.path.isfile(products):
            fm = end2end(cfg.base_path, nb, _template(cfg.base_path, cfg.fm_path))
            run_pledge(fm, n, products, duration=cfg.pledge_duration, seed=cfg.seed)
    trial = TrialConfig(dataset=cfg.dataset, epochs=cfg.training_epochs, batch_size=cfg.batch_size,
                        fill_defaults=True, seed=cfg.seed, synthetic_sizes=tuple(cfg.synthetic_sizes))
    res = run_evolution(cfg.base_path, last_pdts_path=products, nb_base_products=nb[-1], dataset=cfg.dataset,
                        training_epochs=cfg.training_epochs, mutation_rate=cfg.mutation_rate,
                        survival_rate=cfg.survival_rate, breed=cfg.breed, evolution_epochs=cfg.evolution_epochs,
                        model=cfg.model, attacks=tuple(cfg.attacks), mutation_strategy=ms, selection_strategy=ss,
                        max_nb_cells=cfg.max_nb_cells, max_nb_blocks=cfg.max_nb_blocks,
                        scheduler=sched, trial=trial, seed=cfg.seed)
    sched.close()
    print(json.dumps({"session": res.session_path, "generations": res.generations, "history": res.history}))
    return 0


def cmd_pledge(a) -> int:
    from .search import pledge_evolution as pe
    from .search.trial import TrialConfig

    nb = tuple(int(v) for v in a.nb.split("x"))
    template = _template(a.base, a.input)
    fm = pe.end2end(a.base, nb, template) if len(nb) == 3 else template
    res = pe.run(a.base, fm, a.output, a.products, nb_base_products=nb[-1], dataset=a.dataset,
                 training_epochs=a.training_epochs, evolution_epochs=a.evolution_epochs,
                 scheduler=_scheduler(a.devices, 0), trial=TrialConfig(fill_defaults=True),
                 pledge_duration_s=a.dtime)
    print(json.dumps({"session": res.session_path, "population": len(res.population)}))
    return 0


def cmd_products(a) -> int:
    from .search.batch import train_product_set
    from .search.trial import TrialConfig

    res = train_product_set(a.input, datasets=a.datasets.split(","), epochs=a.training_epochs,
                            min_index=a.min_index, max_index=a.max_index, output_folder=a.output,
                            scheduler=_scheduler(a.devices, 0), cfg=TrialConfig(fill_defaults=True))
    print(json.dumps({ds: [s.accuracy for s in specs] for ds, specs in res}))
    return 0


def cmd_retrain(a) -> int:
    from .search.batch import train_from_json, train_from_product

    idx = a.index.split("-") if a.index else None
    if a.json:
        out = train_from_json(a.pledge, a.json, idx, a.export, a.training_epochs, a.batch_size, a.dataset,
                              scheduler=_scheduler(a.devices, 0))
        print(json.dumps([v.accuracy for v in out]))
    else:
        v = train_from_product(a.pledge, int(idx[0]) if idx else 0, a.export, a.training_epochs, a.batch_size,
                               a.dataset, scheduler=_scheduler(a.devices, 0))
        print(json.dumps({"accuracy": v.accuracy}))
    return 0


def cmd_ga(a) -> int:
    from .search import legacy_ga

    pop = legacy_ga.run(a.input, a.output, generations=a.generations, scheduler=_scheduler(a.devices, 0))
    print(json.dumps([v.accuracy for v in pop]))
    return 0


def cmd_resume(a) -> int:
    from .search.batch import retrain_checkpoint

    acc, _ = retrain_checkpoint(a.model, a.epochs, a.dataset, not a.no_augment, a.batch_size, a.save or a.model)
    print(json.dumps({"accuracy": acc}))
    return 0


def cmd_serve(a) -> int:
    from .service.server import serve

    serve(a.host, a.port, a.db, a.base, a.devices or None, max_workers=a.max_workers,
          cors_origins=[o for o in a.cors.split(",") if o] or None)
    return 0


def cmd_train(a) -> int:
    from . import api
    from .fm.products import ProductSet

    arch = a.arch
    if a.pdt:
        arch, _ = ProductSet(a.pdt).format_product(a.index)
    res = api.train(arch, data=a.data, epochs=a.epochs, batch_size=a.batch_size, lr=a.lr, save_path=a.save,
                    fill_defaults=True, scheduler=a.lr_schedule, augment=a.augment,
                    robustness=a.robustness.split(",") if a.robustness else None)
    print(json.dumps({"accuracy": res.accuracy, "loss": res.loss, "path": res.path}))
    return 0


def cmd_classify(a) -> int:
    import numpy as np

    from . import api

    if os.path.isdir(a.input):
        from .training.data import binvox_folder

        x, _, _ = binvox_folder(a.input)
        x = np.asarray(x, np.float32)[..., None]
    else:
        x = np.load(a.input, allow_pickle=False)
    calib = None
    if a.fp8_calib is not None:          # (the first N inputs calibrate the fp8 activation scales)
        calib = x[:a.fp8_calib]
    labels, probs = api.classify(a.model, x, packed_size=a.packed_size, fp8_calib=calib)
    print(json.dumps({"labels": labels.tolist(), "confidence": probs.max(-1).round(4).tolist()}))
    return 0


def cmd_extend(a) -> int:
    from .fm.extend import generate_featuretree

    generate_featuretree(_template(os.path.dirname(a.output) or ".", a.input), a.output, a.cells, a.blocks,
                         block_features=a.block_features)
    print(a.output)
    return 0


def cmd_sample(a) -> int:
    from .fm.sampler import run_pledge

    run_pledge(a.fm, a.n, a.output, duration=a.duration, seed=a.seed)
    print(a.output)
    return 0


def cmd_template(a) -> int:
    from .fm.space import default_template

    print(default_template(a.output))
    return 0


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="featurenet_amd", description=__doc__.split("\n")[0])
    sub = p.add_subparsers(dest="cmd", required=True)

    r = sub.add_parser("run", help="feature-model NAS (reference run.py)")
    r.add_argument("--config", help="YAML/JSON SearchConfig")
    r.add_argument("-n", "--nb", help="BLOCKSxCELLSxPRODUCTS (10x5x100) or PRODUCTS")
    r.add_argument("-t", "--training_epoch", dest="training_epochs", type=int)
    r.add_argument("-b", "--bpath", dest="base_path")
    r.add_argument("-f", "--fpath", dest="fm_path")
    r.add_argument("-a", "--ppath", dest="ppath", help="ignored: sampling is native (no PLEDGE.jar)")
    r.add_argument("-i", "--dtime", dest="pledge_duration", type=float)
    r.add_argument("-p", "--pfile", dest="products_file")
    r.add_argument("-d", "--dataset")
    r.add_argument("-m", "--mutation_strategy", choices=["all", "random"])
    r.add_argument("-g", "--selection_strategy", choices=["pareto", "elitist", "hybrid"])
    r.add_argument("-r", "--mutation_rate", type=float)
    r.add_argument("-s", "--survival_rate", type=float)
    r.add_argument("-e", "--evolution_epoch", dest="evolution_epochs", type=int)
    r.add_argument("-y", "--breed")
    r.add_argument("-l", "--model")
    r.add_argument("--devices")
    r.add_argument("--workers-per-device", dest="workers_per_device", type=int,
                   help="trial worker processes per GPU (0 / unset = auto: 4 per GPU)")
    r.add_argument("--seed", type=int)
    r.set_defaults(fn=cmd_run)

    q = sub.add_parser("pledge", help="diversity-driven evolution (reference pledge_evolution.py)")
    q.add_argument("-n", "--nb", default="5x5x100")
    q.add_argument("-d", "--dataset", default="mnist")
    q.add_argument("-b", "--base", default="./products")
    q.add_argument("-i", "--input", default="", help="1-block FM template (default: built-in)")
    q.add_argument("-o", "--output", default="")
    q.add_argument("-p", "--products", default="", help="resume from a {N}products[_e{n}].json")
    q.add_argument("-t", "--training_epochs", type=int, default=2)
    q.add_argument("-e", "--evolution_epochs", type=int, default=50)
    q.add_argument("--dtime", type=float, default=30.0)
    q.add_argument("--devices", default="")
    q.set_defaults(fn=cmd_pledge)

    b = sub.add_parser("products", help="train every product of a .pdt (reference full.py)")
    b.add_argument("-i", "--input", required=True, help="product file (with or without .pdt)")
    b.add_argument("-d", "--datasets", default="cifar")
    b.add_argument("-t", "--training_epochs", type=int, default=12)
    b.add_argument("--min-index", type=int, default=0)
    b.add_argument("--max-index", type=int, default=0)
    b.add_argument("-o", "--output", default="./products/")
    b.add_argument("--devices", default="")
    b.set_defaults(fn=cmd_products)

    t = sub.add_parser("retrain", help="retrain products by index / vector list (reference pledge_trainer.py)")
    t.add_argument("-p", "--pledge", required=True)
    t.add_argument("-j", "--json", default="")
    t.add_argument("-i", "--index", default="")
    t.add_argument("-e", "--export", default="")
    t.add_argument("-t", "--training_epochs", type=int, default=300)
    t.add_argument("-b", "--batch_size", type=int, default=64)
    t.add_argument("-d", "--dataset", default="cifar")
    t.add_argument("--devices", default="")
    t.set_defaults(fn=cmd_retrain)

    g = sub.add_parser("ga", help="bit-vector GA (reference evolution.py)")
    g.add_argument("-i", "--input", required=True)
    g.add_argument("-o", "--output", required=True)
    g.add_argument("--generations", type=int, default=10)
    g.add_argument("--devices", default="")
    g.set_defaults(fn=cmd_ga)

    c = sub.add_parser("resume", help="continue training a checkpoint (reference utils/retrainer.py)")
    c.add_argument("model")
    c.add_argument("--epochs", type=int, default=100)
    c.add_argument("--dataset", default="cifar")
    c.add_argument("--batch-size", type=int, default=64)
    c.add_argument("--no-augment", action="store_true")
    c.add_argument("--save", default="")
    c.set_defaults(fn=cmd_resume)

    s = sub.add_parser("serve", help="REST task service (reference ui/back)")
    s.add_argument("--host", default="127.0.0.1", help="bind address (no authentication: keep it local)")
    s.add_argument("--port", type=int, default=9999)
    s.add_argument("--db", default="samples.db")
    s.add_argument("--base", default="products")
    s.add_argument("--devices", default="")
    s.add_argument("--max-workers", type=int, default=2, help="concurrently running task workers")
    s.add_argument("--cors", default="", help="comma list of origins allowed cross-origin (default none)")
    s.set_defaults(fn=cmd_serve)

    tr = sub.add_parser("train", help="train one architecture and save a checkpoint")
    tr.add_argument("arch", nargs="?", default="featurenet3d", help="featurenet3d | lenet5 | keras | ...")
    tr.add_argument("--pdt", default="", help="train product --index of this .pdt instead")
    tr.add_argument("--index", type=int, default=0)
    tr.add_argument("--data", default="voxel")
    tr.add_argument("--epochs", type=int, default=12)
    tr.add_argument("--batch-size", type=int, default=128)
    tr.add_argument("--lr", type=float, default=1e-3)
    tr.add_argument("--lr-schedule", action="store_true", help="reference plateau/step/early-stop callbacks")
    tr.add_argument("--augment", action="store_true")
    tr.add_argument("--robustness", default="", help="comma list: clever,pgd,cw,fgsm")
    tr.add_argument("--save", default="model.fnk")
    tr.set_defaults(fn=cmd_train)

    cl = sub.add_parser("classify", help="predict with a checkpoint")
    cl.add_argument("model")
    cl.add_argument("input", help=".npy array or a folder of .binvox files")
    cl.add_argument("--packed-size", type=int, default=None)
    cl.add_argument("--fp8-calib", type=int, default=None, metavar="N",
                    help="FeatureNet-3D on the GPU: run in fp8, activation scales calibrated on the first N inputs "
                         "(block / per-tensor scales or bf16, as the calibration check decides)")
    cl.set_defaults(fn=cmd_classify)

    e = sub.add_parser("extend", help="expand the 1-block template to B x C")
    e.add_argument("--input", default="")
    e.add_argument("--output", required=True)
    e.add_argument("--blocks", type=int, default=5)
    e.add_argument("--cells", type=int, default=5)
    e.add_argument("--block-features", action="store_true")
    e.set_defaults(fn=cmd_extend)

    sm = sub.add_parser("sample", help="sample diverse valid products (native PLEDGE)")
    sm.add_argument("fm")
    sm.add_argument("-n", type=int, default=100)
    sm.add_argument("-o", "--output", required=True)
    sm.add_argument("--duration", type=float, default=30.0)
    sm.add_argument("--seed", type=int, default=0)
    sm.set_defaults(fn=cmd_sample)

    tp = sub.add_parser("template", help="write the built-in search-space FM")
    tp.add_argument("output")
    tp.set_defaults(fn=cmd_template)
    return p


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
