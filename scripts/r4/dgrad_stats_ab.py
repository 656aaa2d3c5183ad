"""A/B: the conv_tile dgrad of conv2-4 (batch 128) with and without the column-statistics
epilogue (the forward's BN-statistics path, RSACC) -- the cost of summing the stored dx
values per workgroup in the dgrad epilogue."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

LAYERS = [("conv2", 29, 32, 32, 5), ("conv3", 25, 32, 64, 4), ("conv4", 22, 64, 64, 3)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, S, C, K, k in LAYERS:
    x = torch.randn(128, S, S, S, C, device="cuda").to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, "valid")
    w = torch.randn(K, k, k, k, C, device="cuda") * 0.05
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    p = ct.dgrad_plan(spec)
    kd = (k, k, k)
    geom = ct.geometry(p, (spec.N, spec.OD, spec.OH, spec.OW, spec.K), (spec.D, spec.H, spec.W), kd,
                       (k - 1, k - 1, k - 1))
    wpk = ct.pack_weights(w, spec.K, spec.taps, spec.C, p, dgrad=True)
    dx = torch.empty(128, S, S, S, C, dtype=torch.bfloat16, device="cuda")
    slab = torch.empty(ct.workers(p, geom, C), 2, C, dtype=torch.float32, device="cuda")
    t0 = timeit(lambda: ct.run(dy, wpk, None, dx, None, p, geom, kd, C, 0))
    t1 = timeit(lambda: ct.run(dy, wpk, None, dx, slab, p, geom, kd, C, 0))
    mask = torch.randint(0, 256, (dx.numel() // 8,), dtype=torch.uint8, device="cuda")
    t2 = timeit(lambda: ct.run(dy, wpk, None, dx, slab, p, geom, kd, C, 0, bny=mask))
    t3 = timeit(lambda: ct.run(dy, wpk, None, dx, slab, p, geom, kd, C, 0x200, bny=mask))   # DMA, no mask epilogue
    t0 = timeit(lambda: ct.run(dy, wpk, None, dx, None, p, geom, kd, C, 0))      # (again: clock ramp)
    ref = dx.float().reshape(-1, C).sum(0)
    err = (slab[:, 0].sum(0) - ref).abs().max().item() / ref.abs().max().item()
    print(json.dumps({"layer": name, "dgrad_us": round(t0, 1), "dgrad_stats_us": round(t1, 1),
                      "dgrad_mask_us": round(t2, 1), "dgrad_maskdma_only_us": round(t3, 1),
                      "stats_rel_err": err}), flush=True)
