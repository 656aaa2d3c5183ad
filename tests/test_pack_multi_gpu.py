"""One-launch weight packing (``ops/conv.py`` pack_scope, ``pack_w_multi_kernel`` in
conv_igemm.hip): the many-layer launch gives the same bits as the single-layer packs for every
layout, the halo packing zero-fills channels a channel-padded conv's weight does not have, and a
NAS candidate trained inside the scope (packs from the up-front launch) matches the same steps
with every pack made by its own layer."""
import contextlib
import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402
cv = importlib.import_module("featurenet_amd.ops.conv")  # noqa: E402  (ops.conv is also the conv function)
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402


def _cases():
    # (spec, weight shape, kind): igemm forward / dgrad / packed-W, halo forward / dgrad, with
    # fewer weight rows / channels than the spec where the NAS paths make them
    s1 = ConvSpec.make((4, 16, 16, 16, 24), 40, (3, 3, 3), 1, "same")
    s2 = ConvSpec.make((4, 1, 32, 32, 6), 12, (1, 5, 5), 1, "same")
    s3 = ConvSpec.make((2, 1, 16, 16, 16), 120, (1, 5, 5), 1, "valid")
    s4 = ConvSpec.make((2, 1, 16, 16, 16), 32, (1, 5, 5), 1, "valid")
    return [(s1, (40, 3, 3, 3, 24), 0), (s1, (36, 3, 3, 3, 24), 1), (s2, (12, 1, 5, 5, 6), 2),
            (s3, (120, 1, 5, 5, 12), 3), (s4, (32, 1, 5, 5, 16), 4), (s4, (28, 1, 5, 5, 12), 4)]


def test_pack_w_multi_matches_single_packs():
    assert _native.kernels_available()
    torch.manual_seed(0)
    ws, singles = [], []
    for spec, shape, kind in _cases():
        w = torch.randn(*shape, device="cuda")
        ws.append(w)
        singles.append(cv._native_pack(w, spec, kind)[0] if kind <= 2 else cv.halo_pack(w, spec, kind == 4))
    rows, outs, ext = [], [], []
    for w, (spec, _, kind) in zip(ws, _cases()):
        row, out, _ = cv._pack_job(w, spec, kind)
        rows.append(row)
        outs.append(out)
        ext.append((w.numel(), out.numel()))
    _native.kernels().pack_w_multi([v for r in rows for v in r], _native.stream(ws[0]), [v for e in ext for v in e])
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(outs, singles)):
        assert a.shape == b.shape and torch.equal(a, b), i


@pytest.mark.parametrize("dgrad", [False, True])
def test_halo_pack_zero_fills_missing_channels(dgrad):
    torch.manual_seed(1)
    spec = ConvSpec.make((2, 1, 16, 16, 16), 32, (1, 5, 5), 1, "valid")
    w = torch.randn(28 if dgrad else 32, 1, 5, 5, 12 if not dgrad else 16, device="cuda")
    got = cv.halo_pack(w, spec, dgrad)
    want = cv.halo_pack(cv.pad_to_spec(w, spec), spec, dgrad)
    assert torch.equal(got, want)


def _candidate_steps(monkeypatch, scoped: bool, steps: int = 3):
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.ops import softmax_xent

    if not scoped:
        monkeypatch.setattr(cv, "pack_scope", lambda m: contextlib.nullcontext())
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    model = compile_model(parse_feature_model("lenet5", name="pk"), (32, 32, 3), 10).to(dev)
    x = torch.rand(64, 32, 32, 3, device=dev)
    y = torch.randint(0, 10, (64,), device=dev)
    out = []
    for _ in range(steps):
        model.zero_grad(set_to_none=True)
        loss = softmax_xent(model(x), y)
        loss.backward()
        with torch.no_grad():                    # (weights move between steps, as in training)
            for p in model.parameters():
                p.add_(p.grad, alpha=-1e-2)
        torch.cuda.synchronize()
        out.append((loss.detach().clone(), {n: p.detach().clone() for n, p in model.named_parameters()}))
    monkeypatch.undo()
    return model, out


def test_candidate_scope_matches_per_layer_packs(monkeypatch):
    hits = []
    orig = cv._pack_lookup

    def counting(w, spec, kind):
        r = orig(w, spec, kind)
        if r is not None:
            hits.append(kind)
        return r

    model, a = _candidate_steps(monkeypatch, scoped=False)
    monkeypatch.setattr(cv, "_pack_lookup", counting)
    model2, b = _candidate_steps(monkeypatch, scoped=True)
    assert model2.__dict__.get("_pack_plan"), "no pack recorded"
    assert len(hits) >= 2 * len(model2.__dict__["_pack_plan"]) - 2, hits   # steps 2 and 3 from the cache
    for i, ((la, pa), (lb, pb)) in enumerate(zip(a, b)):
        assert torch.equal(la, lb), (i, la.item(), lb.item())
        for n in pa:
            assert torch.equal(pa[n], pb[n]), (i, n)


def test_scope_cache_dropped_with_next_forward():
    """A generation's packs are gone when the model's next scope opens (no pack outlives the
    weights it was made from)."""
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model

    dev = torch.device("cuda", 0)
    model = compile_model(parse_feature_model("lenet5", name="pk2"), (32, 32, 3), 10).to(dev)
    x = torch.rand(8, 32, 32, 3, device=dev)
    model(x)
    g1 = model.__dict__["_pack_gen"]
    model(x)
    g2 = model.__dict__["_pack_gen"]
    assert g2 != g1 and g1 not in cv._PK_GENS and g2 in cv._PK_GENS
    assert cv._PK_TLS.gen is None


def test_pack_w_multi_tile_streams_match():
    """Kind 5 (the conv_tile B stream, forward and dgrad) from the many-layer launch == the
    single-layer tile packing."""
    ct = importlib.import_module("featurenet_amd.ops.conv_tile")
    torch.manual_seed(4)
    rows, outs, ext, singles, ws = [], [], [], [], []
    for shp, K, k in (((8, 29, 29, 29, 32), 32, 5), ((8, 22, 22, 22, 64), 64, 3)):
        spec = ConvSpec.make(shp, K, (k, k, k), 1, "valid")
        w = torch.randn(K, k, k, k, shp[-1], device="cuda")
        ws.append(w)                                     # (the job rows hold raw pointers: keep w alive)
        for p, dg in ((ct.fwd_plan(spec), False), (ct.dgrad_plan(spec), True)):
            assert p is not None
            singles.append(ct.pack_weights(w, K, spec.taps, spec.C, p, dg))
            row, out, _ = ct._pack_job(w, (K, spec.taps, spec.C, p, dg), 5)
            rows.append(row)
            outs.append(out)
            ext.append((w.numel(), out.numel()))
    _native.kernels().pack_w_multi([v for r in rows for v in r], _native.stream(outs[0]), [v for e in ext for v in e])
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(outs, singles)):
        assert a.shape == b.shape and torch.equal(a, b), i


def test_featurenet3d_scope_matches_per_layer_packs(monkeypatch):
    """FeatureNet-3D training steps in a pack scope (tile-kernel convs: forward + dgrad streams
    recorded, then made by the scope's one launch) == the same steps with every layer packing its
    own weights."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import softmax_xent

    packs = importlib.import_module("featurenet_amd.ops.packs")
    res, hits = [], []
    orig = packs.lookup

    def counting(w, desc, kind):
        r = orig(w, desc, kind)
        if r is not None:
            hits.append(kind)
        return r

    for scoped in (False, True):
        if scoped:
            monkeypatch.setattr(packs, "lookup", counting)
        torch.manual_seed(5)
        m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda()
        x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
        y = torch.randint(0, 24, (8,), device="cuda")
        run = []
        for _ in range(3):
            m.zero_grad(set_to_none=True)
            # (the model does not open a scope itself -- measured neutral there -- so the test does)
            with (packs.pack_scope(m) if scoped else contextlib.nullcontext()):
                loss = softmax_xent(m(x), y)
            loss.backward()
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(p.grad, alpha=-1e-3)
            torch.cuda.synchronize()
            run.append((loss.detach().clone(), {n: p.detach().clone() for n, p in m.named_parameters()}))
        monkeypatch.undo()
        if scoped:
            kinds = [k[3] for k in m.__dict__.get("_pack_plan", {})]
            assert kinds.count(5) >= 6, kinds           # conv2-4: forward + dgrad streams
            assert hits.count(5) >= 2 * 6, hits         # steps 2 and 3 took them from the scope
        res.append(run)
    for i, ((la, pa), (lb, pb)) in enumerate(zip(*res)):
        assert torch.equal(la, lb), (i, la.item(), lb.item())
        for n in pa:
            assert torch.equal(pa[n], pb[n]), (i, n)
