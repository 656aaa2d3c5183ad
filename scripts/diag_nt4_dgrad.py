import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from featurenet_amd.ops import subpixel as sp
torch.manual_seed(9)
N, S, C, K = 2, 12, 64, 32
w = torch.randn(K, 3, 3, 3, C, device="cuda") * 0.05
dsh = torch.randn(N, S + 1, S + 1, S + 1, 8 * K, device="cuda").to(torch.bfloat16)
res = {}
for flag in ("0", "1"):
    os.environ["FN_SUBPIXEL_NT4"] = flag
    p = sp._dgrad_plan((N, S, S, S, C), K)
    res[flag] = sp.upconv_dgrad(dsh, w, (N, S, S, S, C)).float()
    print(flag, p)
torch.cuda.synchronize()
a, b = res["0"], res["1"]
d = (a - b).abs()
print("max abs diff", d.max().item(), "frac differing", (d > 0).float().mean().item(), "rel", ((a-b).norm()/a.norm()).item())
idx = (d > 0).nonzero()[:5]
print(idx.tolist())
for i in idx.tolist():
    print(a[tuple(i)].item(), b[tuple(i)].item())
ref = sp.ref_dgrad(dsh.float(), w) if hasattr(sp, "ref_dgrad") else None
if ref is not None:
    print("rel vs ref nt2", ((a-ref).norm()/ref.norm()).item(), "nt4", ((b-ref).norm()/ref.norm()).item())
