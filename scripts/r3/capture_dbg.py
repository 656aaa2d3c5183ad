"""Capture one seg training step in a hipGraph and print where capture breaks (debug aid)."""
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from featurenet_amd.models.featurenet3d import FeatureNet3DSeg  # noqa: E402
from featurenet_amd.ops import softmax_xent  # noqa: E402

m = FeatureNet3DSeg(input_size=32, num_classes=25).cuda().train()
x = (torch.rand(4, 32, 32, 32, 1, device="cuda") < 0.3).to(torch.bfloat16)
lab = torch.randint(0, 25, (4, 32, 32, 32), device="cuda")


def step():
    out = m(x)
    loss = softmax_xent(out.reshape(-1, 25), lab.reshape(-1))
    loss.backward()
    return loss


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g):
        step()
    print("capture ok")
except Exception:
    traceback.print_exc()
    sys.exit(1)
