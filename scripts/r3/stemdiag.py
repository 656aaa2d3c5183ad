import torch, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from featurenet_amd.inference import fp8 as F8
from featurenet_amd.models.featurenet3d import FeatureNet3D, FeatureNet3DConfig
from featurenet_amd import ops
from featurenet_amd.ops.spec import ConvSpec
torch.manual_seed(0)
m = FeatureNet3D(FeatureNet3DConfig(input_size=64, num_classes=24)).cuda().eval()
for c in m.convs:
    if c.bn:
        with torch.no_grad():
            c.running_var.uniform_(0.01, 0.5); c.running_mean.normal_(0, 0.5); c.gamma.uniform_(0.5, 2); c.beta.normal_(0, 0.3)
for B in (8, 128):
    x = (torch.rand(B, 64, 64, 64, 1, device="cuda") < 0.3).to(torch.bfloat16)
    q8 = F8.quantize_model(m, x[:8], fp8_stem=True)
    c1 = m.convs[0]
    with torch.no_grad():
        spec = ConvSpec.make(tuple(x.shape), c1.cout, c1.kernel, c1.stride, c1.padding)
        yb = ops.conv(x, q8.c1_w, q8.c1_b, spec, "relu").float()
        ts = F8.stem_tap_plan(c1, tuple(x.shape))
        xt = F8.stem_tap_input(x, ts, q8.in_scale)
        yq, shp = q8.stem(xt, (ts.N, ts.D, ts.H, ts.W, ts.C))
        yd = yq.view(torch.float8_e4m3fn).float() * q8.act_scales[0]
        print(B, "stem out shapes", tuple(yb.shape), tuple(yd.shape), "rel err", ((yd - yb).norm() / yb.norm()).item(),
              "max", yb.abs().max().item(), yd.abs().max().item(), "tile plan", q8.stem.tile_plan(ts))
        bad = ((yd - yb).abs() > 0.2 * yb.abs().max())
        if bad.any():
            idx = bad.nonzero()[:5]; print("bad idx", idx.tolist())
