#!/usr/bin/env python3
"""Measured errors of the model-level GPU comparisons (two bf16 pipelines of the same math):
the sub-pixel decoder against the upsample path, the fused head + loss against the unfused
head + softmax_xent, the BN-identity backward against colstats -- relative L2 of every parameter
gradient, the worst per comparison.  Used to set the tests' bounds from measurements."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def grads(m):
    return {k: p.grad.detach().float().clone() for k, p in m.named_parameters() if p.grad is not None}


def main():
    from featurenet_amd.models.featurenet3d import FeatureNet3DSeg

    torch.manual_seed(4)
    N, S = 2, 24
    m = FeatureNet3DSeg(input_size=S, num_classes=25).cuda().train()
    x = (torch.rand(N, S, S, S, 1, device="cuda") < 0.3).to(torch.bfloat16)
    res = []
    for flag in ("1", "0"):
        os.environ["FN_SUBPIXEL"] = flag
        m.zero_grad(set_to_none=True)
        torch.manual_seed(5)
        out = m(x)
        g = torch.randn_like(out.float())
        (out.float() * g).sum().backward()
        res.append((out.float(), grads(m)))
    os.environ.pop("FN_SUBPIXEL", None)
    e = {k: rel(res[0][1][k], res[1][1][k]) for k in res[1][1]}
    print(f"subpixel vs upsample: out {rel(res[0][0], res[1][0]):.2e}; grads max {max(e.values()):.2e} "
          f"({max(e, key=e.get)})")
    print("  " + ", ".join(f"{k} {v:.1e}" for k, v in sorted(e.items(), key=lambda kv: -kv[1])))
    lab = torch.randint(0, 25, (N, S, S, S), device="cuda")
    for mode in ("1", "2"):
        r = []
        for flag in (mode, "0"):
            os.environ["FN_SEG_XENT"] = flag
            m.zero_grad(set_to_none=True)
            loss, hits = m.loss(x, lab, 0.0, with_correct=True)
            (loss * 3.0).backward()
            r.append((float(loss), grads(m)))
        os.environ.pop("FN_SEG_XENT", None)
        e = {k: rel(r[0][1][k], r[1][1][k]) for k in r[1][1]}
        print(f"fused head mode {mode} vs unfused: loss {abs(r[0][0] - r[1][0]) / abs(r[1][0]):.2e}; grads max "
              f"{max(e.values()):.2e} ({max(e, key=e.get)})")


if __name__ == "__main__":
    main()


def against_fp32():
    """Both GPU decoder paths against the same model run in fp32 on the CPU (the reference ops):
    which one carries the difference?"""
    import copy

    from featurenet_amd.models.featurenet3d import FeatureNet3DSeg

    torch.manual_seed(4)
    N, S = 2, 24
    m = FeatureNet3DSeg(input_size=S, num_classes=25).cuda().train()
    mc = copy.deepcopy(m).cpu().float().train()
    occ = torch.rand(N, S, S, S, 1) < 0.3
    torch.manual_seed(5)
    g = torch.randn(N, S, S, S, 25)
    mc.zero_grad(set_to_none=True)
    outc = mc(occ.float())
    (outc.float() * g).sum().backward()
    ref = grads(mc)
    for flag in ("1", "0"):
        os.environ["FN_SUBPIXEL"] = flag
        m.zero_grad(set_to_none=True)
        out = m(occ.to(torch.bfloat16).cuda())
        (out.float() * g.cuda()).sum().backward()
        gg = grads(m)
        e = {k: rel(gg[k].cpu(), ref[k]) for k in ref}
        print(f"FN_SUBPIXEL={flag} vs fp32 CPU: out {rel(out.float().cpu(), outc.float()):.2e}; grads max "
              f"{max(e.values()):.2e} ({max(e, key=e.get)}); " + ", ".join(f"{k} {v:.1e}" for k, v in
                                                                          sorted(e.items(), key=lambda kv: -kv[1])[:6]))
    os.environ.pop("FN_SUBPIXEL", None)


if __name__ == "__main__" and os.environ.get("FP32", "1") == "1":
    against_fp32()


def classifier_against_fp32(pool: int = 2):
    """FeatureNet-3D (64^3, batch 4) on the GPU kernels vs the same model in fp32 on the CPU, with
    the training loss (softmax cross-entropy on labels) rather than a random output gradient
    (``pool`` 1: the same network without its max-pool -- how much of the difference is the pool's
    arg-max)."""
    import copy

    from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
    from featurenet_amd.ops import softmax_xent

    torch.manual_seed(6)
    m = FeatureNet3D(FeatureNet3DConfig(pool=pool)).cuda().train()
    mc = copy.deepcopy(m).cpu().float().train()
    occ = torch.rand(4, 64, 64, 64, 1) < 0.3
    y = torch.randint(0, 24, (4,))
    mc.zero_grad(set_to_none=True)
    lc = softmax_xent(mc(occ.float()), y)
    lc.backward()
    ref = grads(mc)
    m.zero_grad(set_to_none=True)
    zs = {}
    hooks = [c.register_forward_hook(lambda mod, inp, out, i=i, tag="g": zs.__setitem__((tag, i), out.detach()))
             for i, c in enumerate(m.convs[:3])]
    lg = softmax_xent(m(occ.to(torch.uint8).cuda()), y.cuda())
    for h in hooks:
        h.remove()
    lg.backward()
    gg = grads(m)
    hooks = [c.register_forward_hook(lambda mod, inp, out, i=i: zs.__setitem__(("c", i), out.detach()))
             for i, c in enumerate(mc.convs[:3])]
    with torch.no_grad():
        mc(occ.float())
    for h in hooks:
        h.remove()
    for i in range(3):
        a, b = zs[("g", i)].float().cpu() > 0, zs[("c", i)] > 0
        print(f"relu mask of conv{i + 1}'s output: {100.0 * (a != b).float().mean().item():.2f} % of the elements differ")
    e = {k: rel(gg[k].cpu(), ref[k]) for k in ref}
    print(f"FeatureNet-3D (pool {pool}) vs fp32 CPU: loss {float(lg):.5f} vs {float(lc):.5f}; grads max {max(e.values()):.2e} "
          f"({max(e, key=e.get)}); " + ", ".join(f"{k} {v:.1e}" for k, v in sorted(e.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__" and os.environ.get("FP32CLS", "1") == "1":
    classifier_against_fp32()
    classifier_against_fp32(pool=1)
