"""Focused checks of the statistics-identity pieces on one conv (conv2/conv4 shapes): the masked
dgrad (g, sum g) against dz * mask from the plain dgrad, the conv's weight gradient before /
after a masked dgrad, and bn_wdot against torch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd import _native  # noqa: E402
import importlib  # noqa: E402
cv = importlib.import_module("featurenet_amd.ops.conv")
from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

torch.manual_seed(0)
for (N, S, C, K, k) in [(8, 22, 64, 64, 3), (8, 29, 32, 32, 5), (4, 25, 32, 64, 4)]:
    x = torch.relu(torch.randn(N, S, S, S, C, device="cuda")).to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, k, 1, "valid")
    w = torch.randn(K, k, k, k, C, device="cuda") * 0.05
    dy = torch.randn(spec.out_shape5, device="cuda").to(torch.bfloat16)
    bits = (x.reshape(-1, 8) > 0).to(torch.uint8)
    mask = (bits * (2 ** torch.arange(8, device="cuda", dtype=torch.uint8))).sum(-1).to(torch.uint8).contiguous()
    p = ct.dgrad_plan(spec)
    dz = ct.conv_dgrad(dy, w, spec, p)
    dw0 = cv.native_conv_wgrad(dy, x, spec).clone()
    torch.cuda.synchronize()
    g, ident = ct.conv_dgrad(dy, w, spec, p, bn=(x, None, 1, mask))
    dw1 = cv.native_conv_wgrad(dy, x, spec).clone()
    torch.cuda.synchronize()
    ref = dz.float() * (x.float() > 0)
    print(f"N{N} S{S} C{C} K{K} k{k} plan {p}")
    print("  g vs dz*mask max abs", (g.float() - ref).abs().max().item(), "ref max", ref.abs().max().item())
    sg = ident[1][:, 0].sum(0)
    print("  sum g rel err", ((sg - ref.reshape(-1, C).sum(0)).abs().max() / ref.reshape(-1, C).sum(0).abs().max()).item())
    print("  dW before/after masked dgrad max abs diff", (dw0 - dw1).abs().max().item(), "max", dw0.abs().max().item())
    part = cv.bn_wdot(w, dw0, spec)
    S_k = part.sum(0)
    S_t = (w.to(torch.bfloat16).float() * dw0).reshape(-1, C).sum(0)
    S_z = (dz.float() * x.float()).reshape(-1, C).sum(0)
    print("  wdot vs torch rel", ((S_k - S_t).abs().max() / S_t.abs().max()).item(),
          " identity (sum dz z) rel", ((S_k - S_z).abs().max() / S_z.abs().max()).item())
    # repeat the plain wgrad to see its run-to-run spread
    dw2 = cv.native_conv_wgrad(dy, x, spec).clone()
    print("  dW run-to-run max abs diff", (dw0 - dw2).abs().max().item())
