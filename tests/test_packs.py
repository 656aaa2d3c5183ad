"""The pack-scope bookkeeping of ops/packs.py on the CPU (the GPU side -- the one-launch packing
itself -- is tests/test_pack_multi_gpu.py): a pack is recorded only for model parameters, found by
(pointer, shape, layout, kind) in the generation that made it, invisible outside it, and a dropped
generation disappears from the weak map."""
import gc
import importlib

import torch

packs = importlib.import_module("featurenet_amd.ops.packs")


def _gen(params):
    plan = {}
    g = packs._PackGen(plan, {p.data_ptr(): p for p in params})
    with packs._LOCK:
        packs._NEXT[0] += 1
        gid = packs._NEXT[0]
        packs.GENS[gid] = g
    return gid, g, plan


def test_record_only_parameters_and_lookup_by_generation():
    w = torch.nn.Parameter(torch.randn(4, 3, 3, 3, 2))
    gid, g, plan = _gen([w])
    tmp = torch.randn(4, 3, 3, 3, 2)                 # a per-step temporary: never recorded
    with packs.gen_as(gid):
        packs.record(w.detach(), ("desc",), 0)
        packs.record(tmp, ("desc",), 0)
        packs.record(w.detach().reshape(4, -1), ("desc",), 0)   # (same storage, other shape)
    assert list(plan) == [packs.key(w, ("desc",), 0)]
    g.cache[packs.key(w, ("desc",), 0)] = ("packed", w._version)
    with packs.gen_as(gid):
        assert packs.lookup(w.detach(), ("desc",), 0) == "packed"
        assert packs.lookup(w.detach(), ("other",), 0) is None
        assert packs.lookup(w.detach(), ("desc",), 1) is None
    assert packs.lookup(w, ("desc",), 0) is None      # outside the generation
    assert packs.TLS.gen is None


def test_in_place_change_invalidates_the_pack():
    """A parameter changed in place between the scope's packing and a lookup (an EMA swap, a
    load_state_dict copy, a clamp) misses, so the layer packs its current values."""
    w = torch.nn.Parameter(torch.randn(4, 3))
    gid, g, _ = _gen([w])
    g.cache[packs.key(w, ("d",), 0)] = ("packed", w._version)
    with packs.gen_as(gid):
        assert packs.lookup(w.detach(), ("d",), 0) == "packed"
        with torch.no_grad():
            w.clamp_(-0.5, 0.5)
        assert packs.lookup(w.detach(), ("d",), 0) is None


def test_dropped_generation_leaves_the_weak_map():
    w = torch.nn.Parameter(torch.randn(2, 2))
    gid, g, _ = _gen([w])
    assert gid in packs.GENS
    del g
    gc.collect()
    assert gid not in packs.GENS
    with packs.gen_as(gid):
        assert packs.lookup(w, ("d",), 0) is None


def test_scope_is_a_noop_on_the_cpu():
    m = torch.nn.Linear(3, 2)
    with packs.pack_scope(m):
        assert packs.TLS.gen is None
    assert "_pack_gen" not in m.__dict__
