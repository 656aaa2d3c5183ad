#!/usr/bin/env python3
"""Where the many-layer pack launch (kind 5, tile streams) and the single tile packing differ:
first mismatching elements decoded into (slice, k-step, fragment, lane, j)."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from featurenet_amd import _native  # noqa: E402
from featurenet_amd.ops.spec import ConvSpec  # noqa: E402

ct = importlib.import_module("featurenet_amd.ops.conv_tile")
torch.manual_seed(4)
spec = ConvSpec.make((8, 29, 29, 29, 32), 32, (5, 5, 5), 1, "valid")
w = torch.randn(32, 5, 5, 5, 32, device="cuda")
for p, dg in ((ct.fwd_plan(spec), False), (ct.dgrad_plan(spec), True)):
    a = ct.pack_weights(w, 32, spec.taps, spec.C, p, dg)
    row, out, _ = ct._pack_job(w, (32, spec.taps, spec.C, p, dg), 5)
    print("plan", p.CS, p.nks, p.nct, "row", row[2:])
    _native.kernels().pack_w_multi(row, _native.stream(out), [w.numel(), out.numel()])
    torch.cuda.synchronize()
    b = out
    bad = (a.view(torch.int16) != b.view(torch.int16)).nonzero().flatten()
    print("mismatches", bad.numel(), "of", a.numel())
    for i in bad[:12].tolist():
        u, j = divmod(i, 8)
        lane = u % 64
        r = u // 64
        ctf = r % p.nct
        r //= p.nct
        ks = r % p.nks
        sl = r // p.nks
        print(f"  i={i} slice={sl} ks={ks} ct={ctf} lane={lane} j={j} single={a[i].item()} multi={b[i].item()}")
