import sys, torch
sys.path.insert(0, '/root/repo')
from featurenet_amd.ops import conv_tile as ct
from featurenet_amd.ops import reference as ref
from featurenet_amd.ops.spec import ConvSpec
for (N,S,C,K,k) in [(24,22,64,64,3),(24,22,32,64,3),(24,22,64,32,3),(2,22,64,64,3),(8,22,64,64,3)]:
    torch.manual_seed(0)
    x = torch.randn(N,S,S,S,C,device='cuda').to(torch.bfloat16)
    spec = ConvSpec.make(x.shape, K, (k,k,k), 1, 'valid')
    w = (torch.randn(K,k,k,k,C,device='cuda')*0.05).to(torch.bfloat16).float()
    p = ct.fwd_plan(spec)
    y,_ = ct.conv_fwd(x, w, None, spec, 0, False, p)
    yr = ref.conv(x.float(), w, None, spec)
    err = ((y.float()-yr).norm()/yr.norm()).item()
    bad = ((y.float()-yr).abs() > 0.05*yr.abs().max()).float()
    nb = bad.sum().item()
    where = bad.nonzero()[:3].tolist() if nb else []
    print(N,S,C,K,k,'CS',p.CS,'err',round(err,4),'nbad',nb, where, flush=True)
