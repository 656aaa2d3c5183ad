"""One rank of the killed-rank fault test (tests/test_ddp.py::test_killed_rank_fails_fast).

Rank ``FN_KILL_RANK`` dies abruptly (``os._exit``) after the initial
broadcast; every surviving rank must leave its training loop with a
:class:`DistributedFailure` (exit code 3) well inside the process-group
timeout instead of hanging.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main() -> int:
    from featurenet_amd.ir.compile import compile_model
    from featurenet_amd.ir.parse import parse_feature_model
    from featurenet_amd.parallel.ddp import DistributedFailure, init_from_env
    from featurenet_amd.training.trainer import Trainer

    rank, world, _ = init_from_env("gloo")
    torch.manual_seed(0)
    model = compile_model(parse_feature_model("lenet5", name="l"), (28, 28, 1), 10)
    tr = Trainer(model, lr=1e-3, device="cpu", bucket_mb=0.05)
    if rank == int(os.environ.get("FN_KILL_RANK", "1")):
        os._exit(17)                                  # a crashed node: no clean shutdown
    x = torch.rand(8, 28, 28, 1)
    y = torch.randint(0, 10, (8,))
    try:
        for _ in range(200):
            tr.train_step(x, y)
    except DistributedFailure as e:
        print(f"rank {rank}: DistributedFailure: {e}", flush=True)
        return 3
    print(f"rank {rank}: finished without noticing the dead peer", flush=True)
    return 0


if __name__ == "__main__":
    code = main()
    sys.stdout.flush()
    # leave without tearing down the broken process group: its gloo threads can abort the
    # interpreter's shutdown (seen under load: the exit code then hid the clean failure)
    os._exit(code)
