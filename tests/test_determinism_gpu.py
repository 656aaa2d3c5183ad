"""Bitwise run-to-run repeatability of the native training step on the GPU.

The reference's only behavioural check is repeated runs compared against each other
(``/root/reference/full_lenet5.py:48-54``, ``plots/plotter.py:128-169``), and SURVEY 7.5 asks
for fixed-seed DP=8 vs DP=1 equivalence: both need a step that gives the same bits every time.
Every cross-workgroup reduction of the native kernels is therefore a fixed-order sum over a
fixed work assignment (static tile schedules wherever a partial sum is kept per workgroup,
per-workgroup partial slabs added by ``fn_part_reduce`` instead of float atomics).  These tests
run each step several times -- after other GPU work has run in the process, with a differently
shaped step in between -- and require identical losses and parameter gradients, bit for bit.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from featurenet_amd import _native  # noqa: E402


def _grads(model):
    return {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}


def _assert_same(runs):
    (l0, g0) = runs[0]
    for i, (l, g) in enumerate(runs[1:], 1):
        assert torch.equal(l, l0), f"run {i}: loss {l.item()!r} vs {l0.item()!r}"
        assert g.keys() == g0.keys()
        bad = [n for n in g0 if not torch.equal(g[n], g0[n])]
        assert not bad, f"run {i}: gradients differ bitwise in {bad}"


def _perturb(dev):
    """A differently shaped forward + backward in between (other plans, other scratch sizes, the
    schedule counters and the caching allocator in another state)."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import softmax_xent

    m = FeatureNet3D(FeatureNet3DConfig(input_size=32, num_classes=5, kernels=(5, 3, 3, 3))).to(dev)
    x = (torch.rand(3, 32, 32, 32, 1, device=dev) < 0.5).to(torch.bfloat16)
    softmax_xent(m(x), torch.randint(0, 5, (3,), device=dev)).backward()
    torch.cuda.synchronize()


def test_featurenet3d_step_bitwise_repeatable():
    """FeatureNet-3D at the headline shapes (64^3, batch 8): forward (conv_tile with BN statistics),
    backward (masked dgrad statistics, conv_wtile weight gradients, BN identity, FC): three runs,
    identical bits."""
    assert _native.kernels_available()
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import softmax_xent

    dev = torch.device("cuda", 0)
    torch.manual_seed(11)
    model = FeatureNet3D().to(dev)
    x = (torch.rand(8, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (8,), device=dev)
    runs = []
    for i in range(3):
        if i:
            _perturb(dev)
        model.zero_grad(set_to_none=True)
        loss = softmax_xent(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), _grads(model)))
    _assert_same(runs)


def test_featurenet3d_step_batch128_bitwise_repeatable():
    """The benchmark's batch (128): more tiles per workgroup than the static schedules' first
    round, so every workgroup keeps partials over several tiles."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import softmax_xent

    dev = torch.device("cuda", 0)
    torch.manual_seed(12)
    model = FeatureNet3D().to(dev)
    x = (torch.rand(128, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (128,), device=dev)
    runs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        loss = softmax_xent(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), _grads(model)))
    _assert_same(runs)


@pytest.mark.parametrize("subpixel", ["1", "0"])
def test_seg_step_bitwise_repeatable(monkeypatch, subpixel):
    """FeatureNet3DSeg training loss + backward (sub-pixel decoder with the fused head / loss, or
    the upsample + BN-in-pointwise head): three runs, identical bits."""
    from featurenet_amd.models.featurenet3d import FeatureNet3DSeg

    monkeypatch.setenv("FN_SUBPIXEL", subpixel)
    dev = torch.device("cuda", 0)
    torch.manual_seed(13)
    model = FeatureNet3DSeg(input_size=32).to(dev).train()
    x = (torch.rand(2, 32, 32, 32, 1, device=dev) < 0.3).to(torch.bfloat16)
    lab = torch.randint(0, 25, (2, 32, 32, 32), device=dev)
    runs = []
    for i in range(3):
        if i:
            _perturb(dev)
        model.zero_grad(set_to_none=True)
        loss = model.loss(x, lab)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), _grads(model)))
    _assert_same(runs)


def test_nas_candidate_step_bitwise_repeatable():
    """A reference-style 2-D candidate (lenet5 template, CIFAR shapes): the gather-path kernels
    (igemm weight gradients with their bias gradients, pooling, dense): identical bits."""
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.ops import softmax_xent

    dev = torch.device("cuda", 0)
    torch.manual_seed(14)
    model = compile_model(parse_feature_model("lenet5", name="det"), (32, 32, 3), 10).to(dev)
    x = torch.rand(64, 32, 32, 3, device=dev)
    y = torch.randint(0, 10, (64,), device=dev)
    runs = []
    for _ in range(3):
        model.zero_grad(set_to_none=True)
        loss = softmax_xent(model(x), y)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((loss.detach().clone(), _grads(model)))
    _assert_same(runs)


def test_wgrad_kernels_bitwise_repeatable_and_correct():
    """Each weight-gradient kernel that used float atomics through round 4 -- the halo wgrad, the
    gather (igemm) wgrad with its bias gradient, the pointwise wgrad, the depthwise wgrad -- twice
    on the same inputs: identical bits, and equal to an fp32 reference."""
    import importlib

    from featurenet_amd.ops.spec import ConvSpec

    cv = importlib.import_module("featurenet_amd.ops.conv")
    dev = torch.device("cuda", 0)
    torch.manual_seed(15)

    def rel(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

    # halo wgrad (3-D, stride 1, Cout <= 64)
    x = torch.randn(2, 12, 12, 12, 16, device=dev).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 32, 3, 1, "same")
    plan = cv.halo_wgrad_plan(spec)
    assert plan is not None
    dy = torch.randn(spec.out_shape5, device=dev).to(torch.bfloat16)
    a = cv.halo_conv_wgrad(dy, x, spec, plan).clone()
    b = cv.halo_conv_wgrad(dy, x, spec, plan).clone()
    assert torch.equal(a, b)
    xr = x.float().permute(0, 4, 1, 2, 3).requires_grad_(True)
    wr = torch.zeros(32, 16, 3, 3, 3, device=dev, requires_grad=True)
    yr = torch.nn.functional.conv3d(xr, wr, padding=1)
    (yr * dy.float().permute(0, 4, 1, 2, 3)).sum().backward()
    assert rel(a, wr.grad.permute(0, 2, 3, 4, 1)) < 1e-2

    # gather wgrad (2-D, C = 3, Cout = 6 -> channel-padded dy, bias gradient from the same tiles)
    x2 = torch.randn(32, 1, 28, 28, 3, device=dev).to(torch.bfloat16)
    spec2 = ConvSpec.make(x2.shape, 6, (1, 5, 5), 1, "same")
    dy2 = torch.randn(spec2.out_shape5, device=dev).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        bp = torch.nn.Parameter(torch.zeros(6, device=dev))
        r = cv.igemm_wgrad_cropped(dy2, x2, spec2, 3, with_db=True, bias_param=bp)
        assert r is not None
        dw, db = r
        outs.append((dw.clone(), (db if db is not None else bp.grad).clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    xr = x2.float()[:, 0].permute(0, 3, 1, 2).requires_grad_(True)
    wr = torch.zeros(6, 3, 5, 5, device=dev, requires_grad=True)
    br = torch.zeros(6, device=dev, requires_grad=True)
    yr = torch.nn.functional.conv2d(xr, wr, br, padding=2)
    (yr * dy2.float()[:, 0].permute(0, 3, 1, 2)).sum().backward()
    assert rel(outs[0][0].reshape(6, 5, 5, 3), wr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert rel(outs[0][1], br.grad) < 1e-2

    # pointwise wgrad
    x3 = torch.randn(4096, 32, device=dev).to(torch.bfloat16)
    d3 = torch.randn(4096, 24, device=dev).to(torch.bfloat16)
    p1, p2 = cv.pw_wgrad(d3, x3).clone(), cv.pw_wgrad(d3, x3).clone()
    assert torch.equal(p1, p2)
    assert rel(p1, d3.float().t() @ x3.float()) < 1e-3

    # depthwise wgrad
    x4 = torch.randn(8, 1, 20, 20, 16, device=dev).to(torch.bfloat16)
    spec4 = ConvSpec.make(x4.shape, 16, (1, 3, 3), 1, "same")
    w4 = torch.nn.Parameter(torch.randn(16, 1, 3, 3, 1, device=dev) * 0.1)
    res = []
    for _ in range(2):
        w4.grad = None
        xx = x4.clone().requires_grad_(True)
        y4 = cv.depthwise_conv(xx, w4, None, spec4)
        y4.float().sum().backward()
        res.append(w4.grad.detach().clone())
    assert torch.equal(res[0], res[1])
    xr = x4.float()[:, 0].permute(0, 3, 1, 2)
    wr = w4.detach().float().reshape(16, 1, 3, 3).clone().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, padding=1, groups=16).sum().backward()
    assert rel(res[0].reshape(16, 3, 3), wr.grad.reshape(16, 3, 3)) < 1e-2


def test_tile_statistics_do_not_depend_on_the_grid():
    """The chunked dynamic schedule of conv_tile's BN-statistics launches (fixed chunks of tiles,
    one partial row per chunk, rows added in a fixed order): the same step on a grid of 37 or 100
    workgroups instead of one per CU -- other workgroups running other chunks, in another order,
    as when RCCL kernels hold CUs during data-parallel backward -- gives the same bits."""
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import softmax_xent

    K = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(16)
    model = FeatureNet3D().to(dev)
    x = (torch.rand(16, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (16,), device=dev)
    runs = []
    K.conv_tile_set_schedule(1)                 # the chunked schedule (data parallelism's)
    try:
        for cap in (0, 37, 100):
            K.conv_tile_grid_cap(cap)
            model.zero_grad(set_to_none=True)
            loss = softmax_xent(model(x), y)
            loss.backward()
            torch.cuda.synchronize()
            runs.append((loss.detach().clone(), _grads(model)))
    finally:
        K.conv_tile_grid_cap(0)
        K.conv_tile_set_schedule(-1)
    _assert_same(runs)


@pytest.mark.parametrize("sched", [0, 1])
def test_both_tile_schedules_match_the_reference_statistics(sched):
    """The static (1 GPU) and the chunked (data-parallel) schedules of conv_tile's BN-statistics
    launches: forward BN statistics and the masked-dgrad column sums against fp32 sums of the
    stored outputs (the two schedules add the same values in different orders)."""
    from featurenet_amd.ops import conv_tile as ct
    from featurenet_amd.ops.spec import ConvSpec

    K = _native.kernels()
    dev = torch.device("cuda", 0)
    torch.manual_seed(18)
    x = torch.randn(8, 25, 25, 25, 32, device=dev).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, 64, 4, 1, "valid")
    w = (torch.randn(64, 4, 4, 4, 32, device=dev) * 0.05).float()
    K.conv_tile_set_schedule(sched)
    try:
        p = ct.fwd_plan(spec)
        y, stats = ct.conv_fwd(x, w, None, spec, 0, True, p)
        torch.cuda.synchronize()
    finally:
        K.conv_tile_set_schedule(-1)
    yf = y.float().reshape(-1, 64)
    s1, s2 = stats[:, 0].double().sum(0), stats[:, 1].double().sum(0)
    assert torch.allclose(s1, yf.double().sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(s2, (yf.double() ** 2).sum(0), rtol=1e-4, atol=1e-2)


def test_weight_ring_gives_the_register_path_bits():
    """conv_tile's LDS weight ring (the loader DMAs each k-step's weight fragments once per
    workgroup; per-k-step counters hand the slots over) runs the same MFMAs in the same order as
    the register path (every compute wave streaming the fragments itself): the FeatureNet-3D step
    with the ring on and off gives the same bits -- and the ring, when switched on, is on for most
    layers.  (It is opt-in -- FN_TILE_WLDS=1 -- being slower than the register path,
    profiles/r6_bn_prologue.md.)"""
    from featurenet_amd.models.featurenet3d import FeatureNet3D
    from featurenet_amd.ops import conv_tile as ct
    from featurenet_amd.ops import softmax_xent

    K = _native.kernels()
    dev = torch.device("cuda", 0)
    # which layers take the ring (the plan must leave room for >= 4 slots)
    sp = ct.plan(16, (22, 22, 22), (4, 4, 4), 32, 64)
    geom = ct.geometry(sp, (16, 25, 25, 25, 32), (22, 22, 22), (4, 4, 4), (0, 0, 0))
    K.conv_tile_set_wlds(1)
    try:
        assert K.conv_tile_wring(geom, 64, sp.MT, sp.NT, 0) >= 4
    finally:
        K.conv_tile_set_wlds(-1)
    torch.manual_seed(17)
    model = FeatureNet3D().to(dev)
    x = (torch.rand(16, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
    y = torch.randint(0, 24, (16,), device=dev)
    runs = []
    try:
        for mode in (1, 0, 1):
            K.conv_tile_set_wlds(mode)
            model.zero_grad(set_to_none=True)
            loss = softmax_xent(model(x), y)
            loss.backward()
            torch.cuda.synchronize()
            runs.append((loss.detach().clone(), _grads(model)))
    finally:
        K.conv_tile_set_wlds(-1)
    _assert_same(runs)
