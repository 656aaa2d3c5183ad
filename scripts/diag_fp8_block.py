#!/usr/bin/env python3
"""Block-scaled fp8 conv diagnostics: does the scaled MFMA apply the halo's E8M0 scales, and to
which lanes?  Uniform scale bytes (127 = x1, 128 = x2) against the per-tensor kernel, then
per-position scales against the fp32 emulation.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from featurenet_amd.inference.fp8 import Fp8Conv, dequantize_fp8_block, quantize_fp8_block  # noqa: E402
from featurenet_amd.models.layers import Conv  # noqa: E402
from featurenet_amd.ops import reference as ref  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402


def rel(a, b):
    return round(((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item(), 5)


torch.manual_seed(0)
for cin, cout, k, dims in ((32, 32, 5, (2, 17, 16, 15)), (64, 64, 3, (2, 12, 13, 14))):
    conv = Conv(cin, cout, (k, k, k), 1, "valid", bias=False).cuda()
    x = torch.rand(*dims, cin, device="cuda") * 2 - 1
    spec = ConvSpec.make(x.shape, cout, (k, k, k))
    xq8 = x.to(torch.float8_e4m3fn).view(torch.uint8)
    lt = Fp8Conv(conv, 1.0, None, relu=False)
    yt, _ = lt(xq8, tuple(x.shape))                                   # per-tensor kernel, scale 1
    lb = Fp8Conv(conv, 1.0, None, relu=False)
    out = {"case": f"{cin}->{cout} k{k}"}
    for byte in (127, 128, 126):
        xs = torch.full(dims, byte * 0x01010101 - (1 << 32 if byte >= 128 else 0), dtype=torch.int32, device="cuda")
        yb, _ = lb((xq8, xs), tuple(x.shape))
        out[f"uniform_{byte}_vs_pertensor_x{2.0 ** (byte - 127)}"] = rel(yb, yt * 2.0 ** (byte - 127))
        out[f"uniform_{byte}_ratio"] = round((yb.float().norm() / yt.float().norm()).item(), 4)
    xq, xs = quantize_fp8_block((x * torch.exp2(torch.randint(-6, 7, (*dims, 1), device="cuda").float())).to(torch.bfloat16))
    yb, _ = lb((xq, xs), tuple(x.shape))
    yr = ref.conv(dequantize_fp8_block(xq, xs), lb.w_dequant, lb.bias, spec)
    out["per_position_vs_emulation"] = rel(yb, yr)
    # one position's block scale raised by 2^4: which outputs move?
    xs2 = xs.clone()
    xs2[0, 5, 5, 5] += 4
    yb2, _ = lb((xq, xs2), tuple(x.shape))
    d = (yb2.float() - yb.float()).abs().amax(-1)
    nz = d.nonzero()
    out["moved_outputs"] = int(nz.shape[0])
    out["moved_span"] = [nz.min(0).values.tolist(), nz.max(0).values.tolist()] if nz.numel() else None
    print(json.dumps(out), flush=True)
