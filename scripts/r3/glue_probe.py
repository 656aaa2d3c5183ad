#!/usr/bin/env python3
"""Which Python lines launch the torch glue kernels of a NAS candidate's training step.

Trains a few LeNet-5 mutants (CIFAR-shaped synthetic data, eager steps) under
torch.profiler and groups the aten copy / fill / cast / reduction ops by the innermost
featurenet_amd frame that issued them (count and device time)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import traceback  # noqa: E402

from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from featurenet_amd.ir.parse import parse_feature_model  # noqa: E402
from featurenet_amd.search.mutation import MutationConfig, Mutator  # noqa: E402
from featurenet_amd.search.trial import TrialConfig, run_trial  # noqa: E402


def main():
    mut = Mutator(MutationConfig(seed=0))
    base = parse_feature_model("lenet5", name="lenet5")
    specs = [base] + [mut.generate_mutant(base, 0.1) for _ in range(3)]
    cfg = TrialConfig(dataset="cifar", epochs=1, batch_size=64, synthetic_sizes=(640, 128), graph=False,
                      clever_samples=None)
    run_trial(specs[0], cfg, device="cuda")      # warm up (kernel tables, plans)
    glue = ("copy_", "fill_", "zero_", "sum", "mul", "add", "div", "index", "gather", "cat", "mean", "_to_copy",
            "clone", "zeros", "empty_strided", "constant_pad_nd", "masked_fill", "where", "sub")
    agg = collections.Counter()

    class Probe(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.overloadpacket.__name__
            if name in glue and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
                site = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if "featurenet_amd" in fr.filename:
                        site = f"{fr.filename.split('featurenet_amd/')[-1]}:{fr.lineno} {fr.line}"
                        break
                agg[(name, site)] += 1
            return func(*args, **(kwargs or {}))

    with Probe():
        for s in specs:
            run_trial(s, cfg, device="cuda")
    torch.cuda.synchronize()
    print(f"glue ops (dispatch-level, incl. ones that launch no kernel) over {len(specs)} candidates")
    for k, v in agg.most_common(60):
        print(f"{v:6d}  {k[0]:16s} {k[1][:150]}")

if __name__ == "__main__":
    main()
