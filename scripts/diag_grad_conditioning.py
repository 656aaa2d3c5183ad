#!/usr/bin/env python3
"""How sensitive FeatureNet-3D's gradient is to bf16-sized perturbations, in pure fp32 on the CPU:
the same model with its weights rounded to bf16 (0.4 % relative) and every operation in fp32 --
relative L2 change of each parameter gradient (profiles/r5_bf16_vs_fp32.md)."""
import copy, torch, time
import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from featurenet_amd.models.featurenet3d import FeatureNet3D
from featurenet_amd.ops import softmax_xent
torch.set_num_threads(8)
torch.manual_seed(6)
m = FeatureNet3D().train()
occ = torch.rand(4, 64, 64, 64, 1) < 0.3
y = torch.randint(0, 24, (4,))
def run(model):
    model.zero_grad(set_to_none=True)
    l = softmax_xent(model(occ.float()), y); l.backward()
    return float(l), {k: p.grad.detach().clone() for k, p in model.named_parameters()}
t=time.time()
l0, g0 = run(m)
m2 = copy.deepcopy(m)
with torch.no_grad():
    for p in m2.parameters():
        p.copy_(p.bfloat16().float())      # weights rounded to bf16 (0.4 % relative), all math fp32
l1, g1 = run(m2)
rel = lambda a, b: ((a - b).norm() / b.norm()).item()
print("loss", l0, l1, "time", time.time()-t)
print(", ".join(f"{k} {rel(g1[k], g0[k]):.1e}" for k in g0))
