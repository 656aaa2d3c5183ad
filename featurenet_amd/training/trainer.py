"""Trainer: the fit / evaluate / predict loop over native ops.

Reference parity: ``TensorflowGenerator.build/train`` (``tensorflow_generator.py:221-277``:
compile with Adam(1e-3) + categorical cross-entropy, fit, evaluate test
accuracy) and ``helpers.train_model`` (``helpers.py:69-175``: optional
augmentation, callbacks, reload of the best checkpoint, OOM -> dropped
candidate).

Engine design (MI355X):
* all trainable parameters live in one fp32 buffer (:class:`FlatParams`),
  updated by ONE fused Adam/SGD kernel per step;
* activations are bf16, channels-last, produced by the hand-written kernels;
* with ``torch.distributed`` initialised (one process per GPU), gradients are
  reduced in buckets over RCCL while backward is still running
  (:class:`~featurenet_amd.parallel.ddp.GradBucketer`), each rank trains on its
  shard of every epoch and metrics are all-reduced;
* the per-step loss / correct counters stay on the device; the host reads them
  once per epoch, so the step loop never synchronises.
"""
from __future__ import annotations

import math
import time
from pathlib import Path
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .. import _native
from ..ops import FlatAdam, FlatSGD, softmax_xent
from ..ops.loss import backward as loss_backward
from ..parallel.ddp import DistributedFailure, GradBucketer
from ..utils.events import default_log
from .callbacks import Callback
from .checkpoint import capture_rng, read_checkpoint, read_rng, restore_rng, save_checkpoint
from .data import DeviceLoader
from .flat import FlatParams


def bn_modules(model: torch.nn.Module) -> list[tuple[torch.nn.Module, str]]:
    """(module, momentum attribute) of every layer that keeps BN running statistics."""
    out = []
    for m in model.modules():
        if isinstance(getattr(m, "running_mean", None), torch.Tensor):
            attr = "bn_momentum" if hasattr(m, "bn_momentum") else "momentum" if hasattr(m, "momentum") else None
            if attr is not None:
                out.append((m, attr))
    return out


def _has_dropout(model: torch.nn.Module) -> bool:
    """Active dropout draws a fresh mask every step (host-side seed), so it cannot replay from a graph."""
    prog = getattr(model, "prog", None)
    if prog is not None and any(kind == "dropout" and arg and float(arg) > 0 for kind, arg, _ in prog):
        return True
    return any(float(getattr(m, "dropout", 0) or 0) > 0 for m in model.modules())


class TrainingFailed(RuntimeError):
    pass


@dataclass
class History:
    history: dict = field(default_factory=dict)
    epoch: list = field(default_factory=list)

    def log(self, epoch: int, logs: dict) -> None:
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)



class _EpochMetrics:
    """Device-side running sums of an epoch's loss and correct predictions: one in-place add
    each per step (the per-step reductions and casts were 5-7 tiny launches next to a NAS
    candidate's ~50-kernel step), reduced once by :meth:`totals`."""

    def __init__(self, device):
        self.loss = torch.zeros((), dtype=torch.float64, device=device)
        self.correct = None                      # int64 per-position counts (first batch's size)
        self.extra = torch.zeros((), dtype=torch.int64, device=device)

    def add(self, loss: torch.Tensor, corr: torch.Tensor, n: int) -> None:
        self.loss.add_(loss.detach(), alpha=n)   # float64 += float32 * n in one kernel
        c = corr.reshape(-1)
        if self.correct is None and c.numel() <= 65536:
            self.correct = torch.zeros(c.numel(), dtype=torch.int64, device=c.device)
        if self.correct is not None and c.numel() <= self.correct.numel():
            self.correct[:c.numel()].add_(c)
        else:                                    # (per-voxel counts, or a batch larger than the first)
            self.extra.add_(c.sum())

    def totals(self):
        corr = self.extra if self.correct is None else self.correct.sum() + self.extra
        return self.loss, corr

def _gather_rank_rng(rng: tuple[dict, dict], world: int) -> tuple[dict, dict]:
    """Every rank's :func:`capture_rng` snapshot, gathered for rank 0's checkpoint: rank 0's own
    under the plain ``rng.*`` keys (single-process readers) and rank r's under ``rng.rank<r>.*``;
    the header records the world size and each rank's json part."""
    tensors, meta = rng
    local = ({k: v.detach().cpu() for k, v in tensors.items()}, meta)
    allr: list = [None] * world
    dist.all_gather_object(allr, local)
    out = dict(local[0])
    for r, (t, _) in enumerate(allr):
        for k, v in t.items():
            out["rng.rank%d.%s" % (r, k[len("rng."):])] = v
    return out, {**meta, "world": world, "ranks": [m for _, m in allr]}


class Trainer:
    def __init__(self, model: torch.nn.Module, optimizer: str = "adam", lr: float = 1e-3, device=None,
                 keras_eps: bool = True, weight_decay: float = 0.0, momentum: float = 0.9,
                 label_smoothing: float = 0.0, bucket_mb: float = 32.0, meta: dict | None = None,
                 graph: bool = False, precise_bn: int = 32):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.flat = FlatParams(self.model)
        if optimizer == "adam":
            self.opt = FlatAdam(self.flat.data, self.flat.grad, lr=lr, keras_eps=keras_eps, weight_decay=weight_decay)
        elif optimizer == "sgd":
            self.opt = FlatSGD(self.flat.data, self.flat.grad, lr=lr, momentum=momentum, weight_decay=weight_decay)
        else:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        self.optimizer_name = optimizer
        self.label_smoothing = label_smoothing
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.bucketer = GradBucketer(self.flat, bucket_mb=bucket_mb)
        self.bucketer.broadcast_from(0)
        self.stop_training = False
        # PreciseBN: before validation / at the end of training, BN running statistics
        # are re-estimated as the plain average over this many training batches at the
        # current weights (EMA running stats lag far behind the batch statistics while
        # Adam moves the weights quickly; the eval-mode accuracy then collapses).
        # 0 keeps the reference's EMA statistics (Keras BatchNormalization semantics).
        self.precise_bn = int(precise_bn) if bn_modules(self.model) else 0
        self._bn_fresh = False
        self.meta = dict(meta or {})
        self.history = History()
        # hipGraph capture of the whole training step (forward + backward + the bucketed
        # RCCL all-reduces issued from the gradient hooks + Adam): the same step bench.py
        # times.  NAS candidates on 28x28 / 32x32 inputs are launch-bound, one replay
        # replaces ~100 kernel launches.  Adam, no dropout; one process or RCCL ranks (a
        # rank whose capture fails makes every rank fall back to eager steps together).
        dist_ok = self.world == 1 or (dist.is_initialized() and dist.get_backend() == "nccl")
        self.graph_mode = bool(graph) and self.device.type == "cuda" and dist_ok and \
            optimizer == "adam" and not _has_dropout(self.model)
        self.graph_fallback = False
        self._graph = None
        self._gkey = None
        self._gwarm = 0
        # resume state: epochs completed, and the fit loader's generator at the last epoch end
        self.epochs_done = 0
        self._loader = None
        self._resume_loader_state = None

    # ------------------------------------------------------------------ lr
    def get_lr(self) -> float:
        return self.opt.lr

    def set_lr(self, lr: float) -> None:
        self.opt.lr = float(lr)
        if getattr(self.opt, "_dev", None) is not None:
            # the device-state Adam (graph mode, and the eager steps after a capture fallback)
            # reads lr from its device copy (keeps the 1/world gradient scale)
            self.opt.sync_device_state()

    # ------------------------------------------------------------------ steps
    def _prep(self, xb: torch.Tensor) -> torch.Tensor:
        if self.device.type == "cuda" and xb.dtype != torch.bfloat16:
            xb = xb.to(torch.bfloat16)
        if self.device.type == "cpu" and xb.dtype not in (torch.float32, torch.float64):
            xb = xb.float()
        return xb

    def _loss(self, xb: torch.Tensor, yb: torch.Tensor):
        """(mean loss, top-1 hits): the model's own fused loss when it has one (e.g.
        FeatureNet3DSeg.loss, the cross-entropy inside the head's kernel), else softmax_xent
        of its logits."""
        lossf = getattr(self.model, "loss", None)
        if callable(lossf):
            return lossf(self._prep(xb), yb, self.label_smoothing, with_correct=True)
        return softmax_xent(self.model(self._prep(xb)), yb, self.label_smoothing, with_correct=True)

    def _eager_step(self, xb: torch.Tensor, yb: torch.Tensor):
        self.flat.zero_grad()
        loss, correct = self._loss(xb, yb)
        loss_backward(loss)
        try:
            scale = self.bucketer.finish()
        except DistributedFailure as e:              # fail fast: log and let the process exit non-zero
            default_log().emit("dp_failure", rank=self.rank, world=self.world, error=str(e))
            raise
        self.opt.step(grad_scale=scale)
        return loss.detach(), correct

    def train_step(self, xb: torch.Tensor, yb: torch.Tensor):
        if not self.graph_mode:
            return self._eager_step(xb, yb)
        key = (tuple(xb.shape), xb.dtype, tuple(yb.shape))
        if self._graph is not None:
            if key != self._gkey:                      # e.g. the last partial batch of an epoch
                return self._eager_step(xb, yb)
            _native.copy_in(self._sx, xb, self._sy, yb)   # (one launch for both)
            self._graph.replay()
            self.opt.t += 1
            return self._gloss, self._gcorr
        scale = 1.0 / self.world if self.bucketer.active else 1.0
        self.opt.enable_device_state(grad_scale=scale)
        if self._gwarm < 3:                            # warm caches / kernel tables before capture
            self._gwarm += 1
            return self._eager_step(xb, yb)
        if self.world > 1:                             # identical kernels on every rank
            from ..ops import tuning

            tuning.sync_from_rank0()
        self._sx, self._sy = xb.clone(), yb.clone()
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.device)
        ok = True
        try:
            with torch.cuda.graph(g):
                self.flat.zero_grad()
                loss, correct = self._loss(self._sx, self._sy)
                loss_backward(loss)
                self.bucketer.finish()
                self.opt.step_device()
                self._gloss, self._gcorr = loss.detach(), correct
        except Exception as ex:  # noqa: BLE001 - every rank falls back together (below)
            default_log().emit("graph_capture_failed", rank=self.rank, error=str(ex))
            self.bucketer.reset()
            ok = False
        if self.world > 1:
            f = torch.tensor([1.0 if ok else 0.0], device=self.device)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item() > 0.5)
        if not ok:
            self.graph_mode, self.graph_fallback = False, True
            return self._eager_step(xb, yb)
        self._graph, self._gkey = g, key
        self._graph.replay()                           # capture records only; run this batch now
        self.opt.t += 1
        return self._gloss, self._gcorr

    def _reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            if self.device.type != "cuda" and dist.get_backend() == "nccl":
                t = t.to("cuda")
            dist.all_reduce(t)
        return t

    # ------------------------------------------------------------------ fit
    def fit(self, x, y, epochs: int = 1, batch_size: int = 128, validation_data=None, callbacks=None,
            augment: bool = False, packed_size: int | None = None, verbose: int = 1, shuffle: bool = True,
            seed: int = 0, initial_epoch: int = 0) -> History:
        """Train epochs ``initial_epoch`` .. ``epochs - 1`` (Keras semantics).  After
        :meth:`resume` from a checkpoint written at an epoch end, ``initial_epoch`` = the
        checkpoint's epoch count continues the run bit-for-bit (same shuffle order -- a function
        of (seed, epoch) -- augment draws and dropout masks: this rank's generators come from the
        checkpoint).  Under data parallelism every rank trains on its strided slice of one
        global per-epoch permutation (:class:`DeviceLoader`)."""
        callbacks: list[Callback] = list(callbacks or [])
        loader = DeviceLoader(x, y, batch_size, self.device, shuffle=shuffle, augment=augment,
                              packed_size=packed_size, rank=self.rank, world=self.world, seed=seed, even=True)
        if self._resume_loader_state is not None:
            loader.gen.set_state(self._resume_loader_state.to(torch.uint8))
            self._resume_loader_state = None
        self._loader = loader
        val_loader = None
        if validation_data is not None:   # uploaded once, not once per epoch
            val_loader = DeviceLoader(*validation_data, batch_size, self.device, shuffle=False,
                                      packed_size=packed_size, rank=self.rank, world=self.world, even=False)
        self.stop_training = False
        for cb in callbacks:
            cb.on_train_begin(self)
        t_start = time.time()
        try:
            for epoch in range(initial_epoch, epochs):
                for cb in callbacks:
                    cb.on_epoch_begin(self, epoch)
                self.model.train()
                t0 = time.time()
                acc = _EpochMetrics(self.device)
                seen = 0
                loader.set_epoch(epoch)
                for bi, (xb, yb) in enumerate(loader):
                    loss, corr = self.train_step(xb, yb)
                    acc.add(loss, corr, yb.numel())           # numel: per-voxel labels (segmentation)
                    seen += yb.numel()
                    if callbacks:
                        for cb in callbacks:
                            cb.on_batch_end(self, bi, {})
                loss_sum, correct = acc.totals()
                stats = self._reduce(torch.stack([loss_sum, correct.double(),
                                                  torch.tensor(float(seen), dtype=torch.float64, device=self.device)]))
                logs = {"loss": float(stats[0] / max(stats[2], 1)), "acc": float(stats[1] / max(stats[2], 1)),
                        "lr": self.get_lr(), "time": time.time() - t0,
                        "samples_per_s": float(stats[2]) / max(time.time() - t0, 1e-9)}
                self._bn_fresh = False
                if self.precise_bn and (validation_data is not None or epoch == epochs - 1):
                    self.recalibrate_bn(x, y, self.precise_bn, batch_size, packed_size, seed + epoch,
                                        loader=loader.derived(seed=seed + epoch + 7919))
                if val_loader is not None:
                    vl, va = self.evaluate(None, None, loader=val_loader)
                    logs["val_loss"], logs["val_acc"] = vl, va
                if not math.isfinite(logs["loss"]):
                    raise TrainingFailed("non-finite training loss")
                self.history.log(epoch, logs)
                self.epochs_done = epoch + 1
                default_log().emit("epoch", epoch=epoch, world=self.world, **logs)
                if verbose and self.rank == 0:
                    msg = " ".join(f"{k}={v:.4g}" for k, v in logs.items())
                    print(f"epoch {epoch + 1}/{epochs} {msg}", flush=True)
                for cb in callbacks:
                    cb.on_epoch_end(self, epoch, logs)
                if self.stop_training:
                    break
            if self.precise_bn and not self._bn_fresh:    # stopped early without validation
                self.recalibrate_bn(x, y, self.precise_bn, batch_size, packed_size, seed,
                                    loader=loader.derived(seed=seed + 7919))
        except torch.cuda.OutOfMemoryError as e:   # reference: ResourceExhaustedError -> candidate dropped
            raise TrainingFailed(f"out of device memory: {e}") from e
        finally:
            for cb in callbacks:
                cb.on_train_end(self)
        self.meta["train_time_s"] = time.time() - t_start
        return self.history

    @torch.no_grad()
    def recalibrate_bn(self, x, y, batches: int = 32, batch_size: int = 128, packed_size: int | None = None,
                       seed: int = 0, loader: DeviceLoader | None = None) -> int:
        """PreciseBN: set every BN layer's running mean / var to the average of the batch
        statistics over ``batches`` shuffled training batches (train-mode forward, no
        gradients, momentum 1/(k+1)); replicas average their estimates.  Returns the
        number of batches used.  ``loader`` (e.g. ``DeviceLoader.derived`` of the fit
        loader) reuses device-resident data instead of uploading ``x``/``y`` again."""
        mods = bn_modules(self.model)
        if not mods or batches <= 0:
            return 0
        saved = [getattr(m, a) for m, a in mods]
        was_training = self.model.training
        self.model.train()
        if loader is None:
            loader = DeviceLoader(x, y, batch_size, self.device, shuffle=True, packed_size=packed_size,
                                  rank=self.rank, world=self.world, seed=seed + 7919)
        k = 0
        try:
            for xb, _ in loader:
                if k >= batches:
                    break
                for m, a in mods:
                    setattr(m, a, 1.0 / (k + 1))
                self.model(self._prep(xb))
                k += 1
        finally:
            for (m, a), v in zip(mods, saved):
                setattr(m, a, v)
            self.model.train(was_training)
        if self.world > 1 and k:
            for m, _ in mods:
                for buf in (m.running_mean, m.running_var):
                    t = self._reduce(buf.detach().clone())
                    buf.copy_(t / self.world)
        self._bn_fresh = True
        return k

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, x, y, batch_size: int = 256, packed_size: int | None = None,
                 loader: DeviceLoader | None = None) -> tuple[float, float]:
        self.model.eval()
        if loader is None:
            loader = DeviceLoader(x, y, batch_size, self.device, shuffle=False, packed_size=packed_size,
                                  rank=self.rank, world=self.world, even=False)
        acc = _EpochMetrics(self.device)
        seen = 0
        for xb, yb in loader:
            logits = self.model(self._prep(xb))
            loss, corr = softmax_xent(logits, yb, with_correct=True)
            acc.add(loss, corr, yb.numel())
            seen += yb.numel()
        loss_sum, correct = acc.totals()
        stats = self._reduce(torch.stack([loss_sum, correct.double(),
                                          torch.tensor(float(seen), dtype=torch.float64, device=self.device)]))
        self.model.train()
        n = max(float(stats[2]), 1.0)
        return float(stats[0]) / n, float(stats[1]) / n

    @torch.no_grad()
    def predict(self, x, batch_size: int = 256, packed_size: int | None = None) -> np.ndarray:
        self.model.eval()
        y_dummy = np.zeros(len(x), dtype=np.int64)
        loader = DeviceLoader(x, y_dummy, batch_size, self.device, shuffle=False, packed_size=packed_size)
        out = []
        for xb, _ in loader:
            out.append(torch.softmax(self.model(self._prep(xb)).float(), -1).cpu())
        self.model.train()
        return torch.cat(out).numpy() if out else np.zeros((0,))

    # ------------------------------------------------------------------ io
    def save(self, path, include_optimizer: bool = True, include_rng: bool = True):
        """Weights (+ optimizer moments and step count) (+ every random generator's state and
        the epoch counter: a :meth:`resume` continues the run bit-for-bit)."""
        meta = dict(self.meta)
        meta["history"] = self.history.history
        meta["optimizer_name"] = self.optimizer_name
        meta["train_state"] = {"epochs_done": self.epochs_done, "step": int(getattr(self.opt, "t", 0)),
                               "history_epochs": list(self.history.epoch)}
        rng = None
        if include_rng:
            gens = {"loader": self._loader.gen} if self._loader is not None else {}
            rng = capture_rng(gens)
            if self.world > 1:
                rng = _gather_rank_rng(rng, self.world)   # (a collective: every rank calls save)
        if self.world <= 1:
            return save_checkpoint(path, self.model, meta, self.opt if include_optimizer else None, rng=rng)
        # one writer (rank 0 holds every rank's generator state), then the outcome goes to every
        # rank: a failed write raises everywhere, and no rank returns before the file is complete
        # (ranks read it back through a shared filesystem -- resume() / api.load on other nodes
        # need the path on storage they all see)
        err, out = None, Path(path)
        if self.rank == 0:
            try:
                out = save_checkpoint(path, self.model, meta, self.opt if include_optimizer else None, rng=rng)
            except Exception as e:  # noqa: BLE001 - re-raised on every rank below
                err = f"{type(e).__name__}: {e}"
        flag = [err]
        dist.broadcast_object_list(flag, src=0)
        if flag[0] is not None:
            raise RuntimeError(f"checkpoint write failed on rank 0: {flag[0]}")
        return out

    def resume(self, path) -> int:
        """Load weights, optimizer state, history and random-generator states written by
        :meth:`save`; returns the number of completed epochs (pass it to ``fit`` as
        ``initial_epoch``)."""
        meta, state, opt_state = read_checkpoint(path)
        self.model.load_state_dict(state)
        self.flat.check_bound()
        if opt_state:
            ometa = meta.get("optimizer") or {}
            self.opt.load_state_dict({**ometa, **{k: v.to(self.device) for k, v in opt_state.items()}})
        ts = meta.get("train_state") or {}
        self.epochs_done = int(ts.get("epochs_done", 0))
        self.history = History()
        hist = meta.get("history") or {}
        self.history.history = {k: list(v) for k, v in hist.items()}
        self.history.epoch = list(ts.get("history_epochs", []))
        tensors, rmeta = read_rng(path)
        saved_world = int(rmeta.get("world", 1)) if rmeta else 1
        if saved_world > 1:
            if saved_world == self.world:                # this rank's own generators
                pre = f"rank{self.rank}."
                tensors = {k[len(pre):]: v for k, v in tensors.items() if k.startswith(pre)}
                rmeta = rmeta["ranks"][self.rank]
            else:                                        # another world size: the shuffle order still
                default_log().emit("resume_rng_skipped", saved_world=saved_world, world=self.world)
                tensors, rmeta = {}, {}                  # follows (seed, epoch); augment draws do not
        elif self.world > 1 and tensors:                 # a single-process checkpoint: not per rank
            default_log().emit("resume_rng_skipped", saved_world=1, world=self.world)
            tensors, rmeta = {}, {}
        if tensors or rmeta:
            restore_rng(tensors, rmeta)
            self._resume_loader_state = tensors.get("gen.loader")
        self._graph = None                             # replays captured the old buffers' contents
        return self.epochs_done
