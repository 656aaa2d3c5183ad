"""Python call sites of the torch ops in one FeatureNet-3D training step (GPU, eager)."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig  # noqa: E402
from featurenet_amd.ops import FlatAdam, softmax_xent  # noqa: E402
from featurenet_amd.training.flat import FlatParams  # noqa: E402

dev = torch.device("cuda")
model = FeatureNet3D(FeatureNet3DConfig()).to(dev)
flat = FlatParams(model)
opt = FlatAdam(flat.data, flat.grad, lr=1e-3)
x = (torch.rand(128, 64, 64, 64, 1, device=dev) < 0.3).to(torch.bfloat16)
y = torch.randint(0, 24, (128,), device=dev)


def step():
    flat.zero_grad()
    loss = softmax_xent(model(x), y)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
agg = collections.Counter()
skip = {"empty", "empty_strided", "view", "_unsafe_view", "reshape", "detach", "as_strided", "t", "permute",
        "alias", "select", "slice", "expand", "unsqueeze", "squeeze", "transpose", "_reshape_alias", "lift_fresh"}


class Probe(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in skip and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "featurenet_amd" in fr.filename or "step_glue_probe" in fr.filename:
                    site = f"{fr.filename.split('/')[-1]}:{fr.lineno} {fr.line}"
                    break
            agg[(name, site)] += 1
        return func(*args, **(kwargs or {}))


with Probe():
    step()
torch.cuda.synchronize()
for k, v in agg.most_common(40):
    print(f"{v:4d}  {k[0]:24s} {k[1][:140]}")
