"""Data parallelism: one process per GPU, RCCL all-reduce over xGMI.

Replaces the reference's in-graph ``keras.utils.multi_gpu_model``
(``model/keras_model.py:137-146``), which sliced the batch inside ONE process
and merged outputs on the CPU (and silently fell back to one GPU on any
error, ``:144-146``).  Here every rank holds a full replica; the gradient of
the flat buffer (:class:`~featurenet_amd.training.flat.FlatParams`) is cut
into contiguous buckets in backward-production order and each bucket's
``all_reduce`` is issued the moment its last gradient has been accumulated
(``register_post_accumulate_grad_hook``).  ProcessGroupNCCL (= RCCL on ROCm)
runs collectives on its own HIP stream, ordered after the compute stream at
issue time, so the reduction of bucket *i* overlaps the backward kernels of
the layers that feed bucket *i+1*.  The 1/world averaging is folded into the
optimizer's gradient scale -- no extra pass over the gradients.

Bucket sizing for MI355X: an 8-GPU node is a fully connected xGMI mesh
(7 links x ~153 GB/s per GPU); a ring step is bound by one link, so small
buckets are latency-bound (tens of us per collective) while one huge bucket
serialises behind the last layer's backward.  Default cap 32 MiB.  A bucket
is closed BEFORE a tensor that would push it past the cap, and any tensor of
at least half the cap gets a bucket of its own: FeatureNet-3D's 64000x128 FC1
weight gradient (32.8 MB, produced by the very first backward GEMM) is
therefore reduced alone while the whole conv stack is still in backward.
The tail -- the gradients backward produces last -- is cut from the end into
buckets of 0.25, 0.5, 1, ... MiB: conv4+conv3, conv2 and the stem reduce
separately, conv2's while the stem's weight gradient still runs, so only the
stem's tiny bucket is exposed.  HBM is never the constraint (288 GB per GPU).

Failure handling: the process group is created with an
explicit timeout (``FN_PG_TIMEOUT`` seconds, default 300) and, on RCCL, with
the async-error watchdog on, so a dead or hung peer aborts every surviving
rank with a non-zero exit instead of hanging the job; a collective that
raises is re-raised as :class:`DistributedFailure` naming the rank and
bucket.
"""
from __future__ import annotations

import os
import time
from datetime import timedelta

import torch
import torch.distributed as dist

from ..training.flat import FlatParams


class DistributedFailure(RuntimeError):
    """A collective failed or timed out (peer died, network/RCCL error)."""


def pg_timeout_s() -> float:
    return float(os.environ.get("FN_PG_TIMEOUT", "300"))


def init_from_env(backend: str | None = None, force: bool = False,
                  timeout_s: float | None = None) -> tuple[int, int, int]:
    """Initialise torch.distributed from torchrun env vars; returns (rank, world, local_rank).

    ``force`` creates the process group even at world size 1 (a single-rank
    RCCL communicator: exercises the bucketed collective path on a 1-GPU box).
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        timeout = timedelta(seconds=timeout_s if timeout_s is not None else pg_timeout_s())
        if backend == "nccl":
            # watchdog: a timed-out or failed collective tears the process down
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=timeout,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world, timeout=timeout)
    return rank, world, local


def plan_buckets(sizes: list[int], cap: int, tail_cap: int | None = None) -> list[list[int]]:
    """Group consecutive tensors (element counts ``sizes``) into buckets of at most ``cap`` elements.

    A tensor of at least ``cap // 2`` elements is a bucket of its own; otherwise
    the open bucket is closed before a tensor that would push it past ``cap``.
    ``tail_cap``: the LAST buckets (the gradients backward produces last, whose
    all-reduce nothing can hide) are cut from the end with caps ``tail_cap``,
    ``2 tail_cap``, ``4 tail_cap`` ... up to ``cap``, so the exposed final collective
    is small and each earlier one overlaps the remaining backward.
    Returns lists of tensor indices, in order.
    """
    if tail_cap and tail_cap < cap and sizes:
        tail: list[list[int]] = []
        c, i = tail_cap, len(sizes) - 1
        while i >= 0 and c < cap:
            if sizes[i] >= cap // 2:                 # a large tensor is a bucket of its own; the
                tail.insert(0, [i])                  # tail walk goes on past it at the same cap
                i -= 1
                continue
            cur, size = [], 0
            while i >= 0 and sizes[i] < cap // 2 and (not cur or size + sizes[i] <= c):
                cur.insert(0, i)
                size += sizes[i]
                i -= 1
            tail.insert(0, cur)
            c *= 2
        head = plan_buckets(sizes[:i + 1], cap) if i >= 0 else []
        return head + tail
    out: list[list[int]] = []
    cur: list[int] = []
    size = 0
    for i, n in enumerate(sizes):
        if n >= cap // 2:
            if cur:
                out.append(cur)
            out.append([i])
            cur, size = [], 0
            continue
        if cur and size + n > cap:
            out.append(cur)
            cur, size = [], 0
        cur.append(i)
        size += n
    if cur:
        out.append(cur)
    return out


def use_chunked_tile_schedule(device) -> bool:
    """Data parallelism: the conv kernels' BN-statistics launches take the chunked schedule
    (``conv_tile.hip``: fixed chunks of tiles from XCD queues, one partial row per chunk -- the same
    bits whatever workgroup ran what), which degrades gracefully while the RCCL rings of the
    bucketed all-reduce hold CUs during backward; one GPU keeps the static schedule, the faster
    one when a kernel has the GPU to itself (``profiles/r6_dp_interference.md``).  ``FN_TILE_SCHED``
    set in the environment wins."""
    if os.environ.get("FN_TILE_SCHED") or getattr(device, "type", "cpu") != "cuda":
        return False
    try:
        from .. import _native

        _native.kernels().conv_tile_set_schedule(1)
        return True
    except Exception:  # noqa: BLE001 - no kernel library (CPU): nothing to select
        return False


class GradBucketer:
    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = 32.0, overlap: bool = True,
                 force: bool = False, tail_mb: float | None = 0.25):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # active: collectives are issued (world > 1, or a forced single-rank communicator)
        self.active = dist.is_initialized() and (self.world > 1 or force)
        self.overlap = overlap
        self.paused = False               # tests: run a backward without issuing collectives
        self.cap = max(1, int(bucket_mb * 1024 * 1024 / 4))
        self.buckets: list[tuple[int, int]] = []
        self.members: list[list] = []
        self.param_bucket: dict[int, int] = {}
        # flat slices are contiguous in flat order: a bucket spans first offset .. last end
        tail = max(1, int(tail_mb * 1024 * 1024 / 4)) if tail_mb else None
        for idx in plan_buckets([n for _, _, n in flat.slices], self.cap, tail):
            ps = [flat.slices[i] for i in idx]
            s = ps[0][1]
            e = ps[-1][1] + ps[-1][2]
            if idx[-1] + 1 < len(flat.slices):
                e = flat.slices[idx[-1] + 1][1]          # include the alignment pad up to the next slice
            else:
                e = flat.numel
            self.buckets.append((s, e))
            self.members.append([p for p, _, _ in ps])
            for p, _, _ in ps:
                self.param_bucket[id(p)] = len(self.buckets) - 1
        self.pending = [len(m) for m in self.members]
        self.launched = [False] * len(self.buckets)
        self.works: list = []
        self.hooks = []
        self.n_collectives = 0
        if self.active and self.world > 1:
            use_chunked_tile_schedule(flat.data.device)
        if self.active and overlap:
            for p, _, _ in flat.slices:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    @property
    def n_buckets(self) -> int:
        return len(self.buckets)

    def bucket_bytes(self) -> list[int]:
        return [(e - s) * 4 for s, e in self.buckets]

    def _launch(self, b: int) -> None:
        s, e = self.buckets[b]
        self.launched[b] = True
        try:
            self.works.append((b, dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True)))
        except Exception as ex:                      # noqa: BLE001 - re-raised with context
            raise DistributedFailure(f"rank {self.rank}: all_reduce of bucket {b} failed to launch: {ex}") from ex
        self.n_collectives += 1

    def _on_grad(self, p) -> None:
        if self.paused:
            return
        b = self.param_bucket.get(id(p))
        if b is None or self.launched[b]:
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            # launch in bucket order so every rank issues collectives identically
            for i in range(len(self.buckets)):
                if self.launched[i]:
                    continue
                if self.pending[i] > 0:
                    break
                self._launch(i)

    def finish(self) -> float:
        """Complete all reductions; returns the gradient scale (1/world) for the optimizer."""
        if not self.active or self.paused:
            return 1.0
        for i in range(len(self.buckets)):
            if not self.launched[i]:
                self._launch(i)
        try:
            for b, w in self.works:
                w.wait()
        except Exception as ex:                      # noqa: BLE001
            raise DistributedFailure(f"rank {self.rank}: all_reduce of bucket {b} failed: {ex}") from ex
        finally:
            self.works.clear()
            self.pending = [len(m) for m in self.members]
            self.launched = [False] * len(self.buckets)
        return 1.0 / self.world

    def reset(self) -> None:
        """Forget a partially issued step (after a skipped/aborted backward)."""
        self.works.clear()
        self.pending = [len(m) for m in self.members]
        self.launched = [False] * len(self.buckets)

    def broadcast_from(self, src: int = 0) -> None:
        """Make every replica start from rank ``src``'s parameters and buffers."""
        if not self.active or self.world == 1:
            return
        dist.broadcast(self.flat.data, src, group=self.group)
        for b in self.flat.module.buffers():
            dist.broadcast(b, src, group=self.group)

    def time_allreduce(self, iters: int = 5) -> float:
        """Median wall ms of one all-reduce of the whole flat gradient (bucketed as in training)."""
        if not self.active:
            return 0.0
        cuda = self.flat.grad.is_cuda
        ts = []
        for _ in range(iters + 1):
            if cuda:
                torch.cuda.synchronize()
            dist.barrier(group=self.group)
            t0 = time.perf_counter()
            works = [dist.all_reduce(self.flat.grad[s:e], group=self.group, async_op=True) for s, e in self.buckets]
            for w in works:
                w.wait()
            if cuda:
                torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts = sorted(ts[1:])
        return ts[len(ts) // 2]
