"""NAS engine on CPU: trial faults, FullEvolution, PLEDGE evolution, legacy GA."""
import json
import os

import pytest

from featurenet_amd.ir.parse import parse_feature_model
from featurenet_amd.search.trial import TrialConfig, TrialScheduler, run_trial

REF = "/root/reference"
need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference fixtures not present")


def _cfg(**kw):
    base = dict(dataset="mnist", epochs=1, batch_size=64, synthetic_sizes=(256, 64), clever_samples=2,
                robustness_set_size=8)
    base.update(kw)
    return TrialConfig(**base)


def _spec(name):
    s = parse_feature_model("lenet5", name=name)
    return s


def test_run_trial_trains_and_reports(tmp_path):
    out = run_trial(_spec("ok"), _cfg(save_dir=str(tmp_path)), "cpu")
    assert out.status == "trained"
    assert 0.0 <= out.accuracy <= 1.0
    assert out.nb_params > 0 and out.nb_flops > 0
    assert (tmp_path / "ok.fnk").exists()


@pytest.mark.parametrize("fault,status", [("build", "invalid"), ("oom", "failed")])
def test_run_trial_inline_faults(fault, status):
    out = run_trial(_spec("x"), _cfg(inject={"x": fault}), "cpu")
    assert out.status == status
    assert out.accuracy == 0.0
    assert out.error


def test_scheduler_survives_hang_and_crash():
    """A hung and a crashed trial fail only themselves; the search continues."""
    specs = [_spec("a"), _spec("hang"), _spec("crash"), _spec("b")]
    # (45 s: a spawned worker importing torch on a loaded CI box can take most of 20 s)
    with TrialScheduler(devices=["cpu", "cpu"], timeout_s=45, mode="process") as sched:
        res = sched.map(specs, _cfg(inject={"hang": "hang", "crash": "crash"}))
    by = {r.name: r for r in res}
    assert by["a"].status == "trained" and by["b"].status == "trained"
    assert by["hang"].status == "failed" and "timed out" in by["hang"].error
    assert by["crash"].status == "failed" and "died" in by["crash"].error
    assert [r.name for r in res] == ["a", "hang", "crash", "b"]


def test_scheduler_runs_several_workers_per_device():
    """workers_per_device = 2 on one device: two worker processes, every trial trained once,
    results in submission order."""
    with TrialScheduler(devices=["cpu"], timeout_s=60, mode="process", workers_per_device=2) as sched:
        assert len(sched.slots()) == 2 and len({k for k, _ in sched.slots()}) == 2
        specs = [_spec(n) for n in ("a", "b", "c")]
        res = sched.map(specs, _cfg())
        assert [r.name for r in res] == ["a", "b", "c"]
        assert all(r.status == "trained" for r in res)


def test_scheduler_start_spawns_the_pool_before_map():
    """start() spawns the persistent pool up front; the first map then uses those processes."""
    with TrialScheduler(devices=["cpu", "cpu"], timeout_s=60, mode="process") as sched:
        pids = sorted(sched.start().pids())
        assert len(pids) == 2
        res = sched.map([_spec("a"), _spec("b")], _cfg())
        assert all(r.status == "trained" for r in res) and sorted(sched.pids()) == pids


def test_scheduler_workers_persist_across_maps():
    """Two map calls (two generations) run on the same worker processes; after close() none is
    left.  A crash in the second map replaces only that worker."""
    with TrialScheduler(devices=["cpu", "cpu"], timeout_s=60, mode="process") as sched:
        r1 = sched.map([_spec("a"), _spec("b")], _cfg())
        pids = sorted(sched.pids())
        assert len(pids) == 2 and all(r.status == "trained" for r in r1)
        r2 = sched.map([_spec("c"), _spec("crash"), _spec("d")], _cfg(inject={"crash": "crash"}))
        assert [r.name for r in r2] == ["c", "crash", "d"]
        assert r2[0].status == "trained" and r2[2].status == "trained" and r2[1].status == "failed"
        assert len(set(sched.pids()) & set(pids)) >= 1         # (the crashed one was replaced)
        procs = [w["proc"] for w in sched._workers.values()]
    assert not sched.pids() and all(not p.is_alive() for p in procs)


def test_scheduler_replaces_worker_after_device_error():
    """A trial that fails with a HIP runtime error (a poisoned context) is reported as failed and
    its worker exits; the next trials run on a fresh worker instead of failing one after another."""
    from featurenet_amd.search.trial import device_poisoned

    assert device_poisoned("RuntimeError: HIP error: an illegal memory access was encountered")
    assert not device_poisoned("TrainingFailed: loss is nan")
    with TrialScheduler(devices=["cpu"], timeout_s=60, mode="process") as sched:
        pid0 = sched.start().pids()
        res = sched.map([_spec("dev"), _spec("b"), _spec("c")], _cfg(inject={"dev": "device"}))
        assert [r.name for r in res] == ["dev", "b", "c"]
        assert res[0].status == "failed" and "HIP error" in res[0].error
        assert res[1].status == "trained" and res[2].status == "trained"
        assert sched.pids() and set(sched.pids()).isdisjoint(pid0)


def test_scheduler_abnormal_exit_leaves_no_stale_task(monkeypatch):
    """map() leaving by an exception ends the workers still busy with its tasks, so the next map()
    neither accepts their late results nor waits on a slot with no task behind it."""
    import featurenet_amd.search.trial as tr

    with TrialScheduler(devices=["cpu"], timeout_s=60, mode="process") as sched:
        real = tr.ModelSpec.from_json
        calls = {"n": 0}

        def boom(js):
            calls["n"] += 1
            raise KeyboardInterrupt("injected")

        monkeypatch.setattr(tr.ModelSpec, "from_json", staticmethod(boom))
        with pytest.raises(KeyboardInterrupt):
            sched.map([_spec("a"), _spec("b")], _cfg())
        monkeypatch.setattr(tr.ModelSpec, "from_json", staticmethod(real))
        assert all(w["busy"] is None for w in sched._workers.values())
        res = sched.map([_spec("c"), _spec("d")], _cfg())
        assert [r.name for r in res] == ["c", "d"] and all(r.status == "trained" for r in res)


def test_full_evolution_two_generations(tmp_path):
    from featurenet_amd.search.evolution import load_snapshot, run_evolution

    r = run_evolution(str(tmp_path), nb_base_products=4, dataset="mnist", training_epochs=1, evolution_epochs=2,
                      attacks=(), trial=_cfg(), scheduler=TrialScheduler(["cpu"], mode="inline"),
                      survival_rate=0.5, seed=1, verbose=0)
    assert r.generations == 2
    sp = r.session_path
    assert os.path.isfile(os.path.join(sp, "e1.json")) and os.path.isfile(os.path.join(sp, "e2.json"))
    snap = load_snapshot(os.path.join(sp, "4products_e2.json"))
    assert len(snap) == len(r.population)
    # resume continues the generation count
    r2 = run_evolution(str(tmp_path), nb_base_products=4, dataset="mnist", training_epochs=1, evolution_epochs=1,
                       attacks=(), trial=_cfg(), scheduler=TrialScheduler(["cpu"], mode="inline"),
                       survival_rate=0.5, resume_from=os.path.join(sp, "4products_e2.json"), verbose=0)
    assert r2.history[0]["generation"] == 3


@need_ref
def test_pledge_evolution_one_generation(tmp_path):
    from featurenet_amd import _native
    from featurenet_amd.search import pledge_evolution as pe

    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    fm = pe.end2end(str(tmp_path), (1, 1, 4), f"{REF}/main_1block_nas.xml")
    r = pe.run(str(tmp_path), fm, nb_base_products=4, dataset="mnist", training_epochs=1, evolution_epochs=1,
               attacks=(), trial=_cfg(fill_defaults=True), scheduler=TrialScheduler(["cpu"], mode="inline"),
               pledge_duration_s=0.2, verbose=0)
    assert os.path.isfile(tmp_path / "mnist" / "4products.json")
    ranked = json.loads((tmp_path / "mnist" / "4products_e0.json").read_text())
    assert len(ranked) >= 1
    accs = [v[0] for v in ranked]
    assert accs == sorted(accs, reverse=True)
    assert r.population


@need_ref
def test_pledge_children_exclude_constrained_labels(tmp_path):
    """generate_children injects ``~Architecture or ~<label>`` per constrained label
    (reference ``pledge_evolution.py:70-99``): the child FM carries every clause and
    no sampled child selects a constrained feature."""
    import random

    from featurenet_amd import _native
    from featurenet_amd.fm.products import ProductSet
    from featurenet_amd.fm.sampler import run_pledge
    from featurenet_amd.search import pledge_evolution as pe

    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    fm = pe.end2end(str(tmp_path), (1, 1, 8), f"{REF}/main_1block_nas.xml")
    base = tmp_path / "base.pdt"
    run_pledge(fm, 8, base, duration=0.3, seed=1)
    ps = ProductSet(base)
    enabled = [set(ps.enabled_labels(p)) for p in ps.products]
    # non-core leaf labels (absent from some sampled product): excluding them stays satisfiable
    richest = max(enabled, key=len)
    labels = sorted(l for l in richest - set.intersection(*enabled) if len(l) > 3)[:2]
    assert labels, "sampled products are all identical"
    pdt = pe.generate_children(str(tmp_path / "child"), labels, fm, 6, 1.0, random.Random(0), duration_s=0.3)
    xml = (tmp_path / "child.xml").read_text()
    for l in labels:
        assert f"~Architecture  or  ~{l}" in xml
    kids = ProductSet(pdt)
    assert kids.nbProducts >= 1
    for p in kids.products:
        assert not set(kids.enabled_labels(p)) & set(labels)


@need_ref
def test_legacy_ga_runs(tmp_path):
    from featurenet_amd import _native
    from featurenet_amd.fm.sampler import run_pledge
    from featurenet_amd.search import legacy_ga

    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    pdt = tmp_path / "p.pdt"
    run_pledge(f"{REF}/nas_1_1_10.xml", 4, pdt, duration=0.2)
    pop = legacy_ga.run(str(pdt), str(tmp_path / "ga.jsonl"), generations=1, scheduler=TrialScheduler(["cpu"], mode="inline"),
                        cfg=_cfg(fill_defaults=True))
    assert len(pop) == 4
    lines = (tmp_path / "ga.jsonl").read_text().splitlines()
    assert len(lines) == 1
