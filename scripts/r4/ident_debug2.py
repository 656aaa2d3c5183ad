"""FeatureNet-3D (batch 8, 64^3) parameter gradients: identity path off / off / on, per-parameter
relative differences (run-to-run noise vs the identity path)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.models.featurenet3d import FeatureNet3D  # noqa: E402


def grads(model, x, on):
    os.environ["FN_BN_IDENTITY"] = "1" if on else "0"
    model.zero_grad(set_to_none=True)
    out = model(x)
    loss = (out.float() * torch.linspace(-1, 1, out.shape[-1], device=x.device)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}


torch.manual_seed(2)
m = FeatureNet3D().cuda()
x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
a = grads(m, x, False)
b = grads(m, x, False)
c = grads(m, x, True)
d = grads(m, x, True)
for n in a:
    r = lambda u, v: ((u - v).abs().max() / u.abs().max().clamp_min(1e-6)).item()  # noqa: E731
    print(f"{n:28s} off/off {r(a[n], b[n]):.2e}  off/on {r(a[n], c[n]):.2e}  on/on {r(c[n], d[n]):.2e}")
