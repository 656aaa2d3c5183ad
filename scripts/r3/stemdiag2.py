import os, sys, numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import featurenet_amd as fn
from featurenet_amd.training.data import voxel_dataset, unpack_voxels
from featurenet_amd.inference import fp8 as F8
from featurenet_amd import ops
from featurenet_amd.ops.spec import ConvSpec
torch.cuda.set_device(0)
ds = voxel_dataset(200 * 24, 10 * 24, size=64, num_classes=24, seed=0)
res = fn.train("featurenet3d", data=ds, epochs=3, batch_size=128, lr=1e-3, seed=0, verbose=0, callbacks=[])
model = res.model.eval()
dev = next(model.parameters()).device
def batch(xs, i, n):
    xb = torch.as_tensor(np.asarray(xs[i:i + n])).to(dev)
    return unpack_voxels(xb, 64).to(torch.bfloat16)
cx = batch(ds.x_train, 0, 256)
print("calib", tuple(cx.shape), cx.dtype, cx.is_contiguous(), float(cx.float().min()), float(cx.float().max()))
q8 = F8.quantize_model(model, cx)
qs = F8.quantize_model(model, cx, fp8_stem=False)
xb = batch(ds.x_test, 0, 128)
x = xb.unsqueeze(-1) if xb.dim() == 4 else xb
c1 = model.convs[0]
with torch.no_grad():
    spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
    yb = ops.conv(x.contiguous(), q8.c1_w, q8.c1_b, spec, "relu").float()
    ts = F8.stem_tap_plan(c1, tuple(x.shape))
    print("tap plan", ts is not None, "in_scale", q8.in_scale, "act0", q8.act_scales[0])
    xt = F8.stem_tap_input(x, ts, q8.in_scale)
    yq, shp = q8.stem(xt, (ts.N, ts.D, ts.H, ts.W, ts.C))
    yd = yq.view(torch.float8_e4m3fn).float() * q8.act_scales[0]
    print("stem rel err", ((yd - yb).norm() / yb.norm()).item(), yb.abs().max().item(), yd.abs().max().item())
    print("w stats", q8.c1_w.abs().max().item(), q8.c1_b.abs().max().item(), "scale", q8.stem.scale.min().item(), q8.stem.scale.max().item())
    a, b, r = q8(xb).float(), qs(xb).float(), model(xb).float()
    print("logit rel", ((a - r).norm() / r.norm()).item(), ((b - r).norm() / r.norm()).item())
    print("agree", (a.argmax(-1) == r.argmax(-1)).float().mean().item(), (b.argmax(-1) == r.argmax(-1)).float().mean().item())
