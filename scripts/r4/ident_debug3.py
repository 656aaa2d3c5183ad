"""After a forked-BN model ran (identity on / off), are FeatureNet-3D's conv4 weight gradients
still deterministic run to run?  argv[1]: '1' = the fork model runs with the identity path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from featurenet_amd.models.featurenet3d import FeatureNet3D  # noqa: E402
from featurenet_amd.models.layers import Conv  # noqa: E402

fork_ident = sys.argv[1] if len(sys.argv) > 1 else "1"
fork_tile = sys.argv[2] if len(sys.argv) > 2 else "2"


class Fork(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = Conv(32, 32, 3, 1, "valid", bn=True, act="relu", init="he")
        self.b = Conv(32, 32, 3, 1, "same", bn=False, act=None, init="he")

    def forward(self, x):
        z = self.a(x)
        return self.b(z) + z


def grads(model, x):
    model.zero_grad(set_to_none=True)
    out = model(x)
    loss = (out.float() * torch.linspace(-1, 1, out.shape[-1], device=x.device)).sum()
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}


os.environ["FN_BN_IDENTITY"] = fork_ident
os.environ["FN_CONV_TILE"] = fork_tile
torch.manual_seed(3)
f = Fork().cuda()
xf = torch.randn(2, 18, 18, 18, 32, device="cuda").to(torch.bfloat16)
grads(f, xf)
os.environ["FN_BN_IDENTITY"] = "0"
os.environ.pop("FN_CONV_TILE")
torch.manual_seed(2)
m = FeatureNet3D().cuda()
x = (torch.rand(8, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
gs = [grads(m, x) for _ in range(4)]
for n in ["convs.3.weight", "convs.2.weight", "fc1.weight"]:
    print(f"fork_ident={fork_ident} tile={fork_tile} {n}", [f"{((gs[0][n] - g[n]).abs().max() / gs[0][n].abs().max()).item():.2e}" for g in gs[1:]])
