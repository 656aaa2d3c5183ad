"""Diagnostics for the int8 instance of the fp8 tile kernel: structured inputs whose exact
outputs are known (constant operands, channel halves, single taps), printed side by side."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.ops import conv_tile as ct  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

N, S, C, K = 2, 12, 32, 32
spec = ConvSpec.make((N, S, S, S, C), K, (4, 4, 1), 1, "valid")
p = ct.plan(N, (spec.OD, spec.OH, spec.OW), (4, 4, 1), C, K, f8=True)
print("plan", p)
dev = "cuda"
one = torch.ones(K, device=dev)
zero = torch.zeros(K, device=dev)


def run(xi, wi, i8=True):
    wpk = ct.pack_weights_f8(wi.view(torch.uint8).reshape(K, 16, C), p)
    y = ct.conv_fwd_f8(xi.view(torch.uint8), wpk, one, zero, spec, p, False, None, i8=i8)
    torch.cuda.synchronize()
    acc = torch.nn.functional.conv3d(xi.double().permute(0, 4, 1, 2, 3), wi.double().permute(0, 4, 1, 2, 3))
    return y.double(), acc.permute(0, 2, 3, 4, 1)


def report(name, y, ref):
    d = (y - ref).abs()
    print(f"{name:28s} y[0,0,0,0,:4]={y[0, 0, 0, 0, :4].tolist()} ref={ref[0, 0, 0, 0, :4].tolist()} "
          f"maxerr={d.max().item():.3g} frac_bad={(d > 1e-2 * ref.abs().clamp_min(1)).float().mean().item():.3f} "
          f"y_mean={y.mean().item():.3g} ref_mean={ref.mean().item():.3g}")


xo = torch.ones(N, S, S, S, C, dtype=torch.int8, device=dev)
wo = torch.ones(K, 4, 4, 1, C, dtype=torch.int8, device=dev)
report("ones", *run(xo, wo))
w = wo.clone(); w[..., 16:] = 0
report("w ch<16", *run(xo, w))
w = wo.clone(); w[..., :16] = 0
report("w ch>=16", *run(xo, w))
for t in range(4):
    w = torch.zeros_like(wo); w[:, t, 0, 0, :] = 1
    report(f"w tap kd={t}", *run(xo, w))
w = torch.zeros_like(wo); w[:, 0, 0, 0, 0] = 1
x = torch.arange(N * S * S * S, device=dev).reshape(N, S, S, S, 1).remainder(100).to(torch.int8).expand(N, S, S, S, C).contiguous()
report("w single, x ramp", *run(x, w))
w = torch.zeros_like(wo); w[:, 0, 0, 0, 20] = 1
report("w single ch20, x ramp", *run(x, w))
wk = torch.zeros_like(wo)
for k in range(K):
    wk[k, 0, 0, 0, 0] = k - 16
report("w per-col, x ones", *run(xo, wk))
torch.manual_seed(7)
xr = torch.randint(-20, 21, (N, S, S, S, C), device=dev, dtype=torch.int8)
wr = torch.randint(-127, 128, (K, 4, 4, 1, C), device=dev, dtype=torch.int8)
report("random", *run(xr, wr))
wr2 = torch.randint(-10, 11, (K, 4, 4, 1, C), device=dev, dtype=torch.int8)
report("random small w", *run(xr, wr2))
# the same small-integer data through the e4m3 kernel (exact in e4m3 for |v| <= 16)
xs = torch.randint(-4, 5, (N, S, S, S, C), device=dev).float()
ws = torch.randint(-4, 5, (K, 4, 4, 1, C), device=dev).float()
x8, w8 = xs.to(torch.float8_e4m3fn).view(torch.int8), ws.to(torch.float8_e4m3fn).view(torch.int8)
yf, _ = run(x8, w8, i8=False)
ref = torch.nn.functional.conv3d(xs.double().permute(0, 4, 1, 2, 3), ws.double().permute(0, 4, 1, 2, 3)).permute(0, 2, 3, 4, 1)
report("e4m3 small ints", yf, ref)
yi, refi = run(xs.to(torch.int8), ws.to(torch.int8))
report("int8 small ints", yi, refi)
