"""Training callbacks.

Reference parity (``helpers.py:12-97``, ``sgdr.py:5-85``): ReduceLROnPlateau
(factor sqrt(0.1), patience 5, min 5e-7), the step LR schedule (x0.1 after
80, x1e-2 after 120, x1e-3 after 160, x5e-4 after 180 epochs), EarlyStopping
on val_acc (min_delta 0.01, patience 20), ModelCheckpoint keeping the best
val_loss weights (restored at the end of fit, like the reference's
reload-and-delete of the temp .h5), TimedStopping and SGDR (cosine annealing
with warm restarts).  Callbacks talk to a :class:`~featurenet_amd.training.trainer.Trainer`.
"""
from __future__ import annotations

import copy
import math
import time


class Callback:
    def on_train_begin(self, trainer): ...
    def on_train_end(self, trainer): ...
    def on_epoch_begin(self, trainer, epoch: int): ...
    def on_epoch_end(self, trainer, epoch: int, logs: dict): ...
    def on_batch_end(self, trainer, batch: int, logs: dict): ...


def reference_lr_schedule(epoch: int, base_lr: float = 1e-3) -> float:
    lr = base_lr
    if epoch > 180:
        lr *= 0.5e-3
    elif epoch > 160:
        lr *= 1e-3
    elif epoch > 120:
        lr *= 1e-2
    elif epoch > 80:
        lr *= 1e-1
    return lr


class LearningRateScheduler(Callback):
    def __init__(self, schedule=reference_lr_schedule):
        self.schedule = schedule

    def on_epoch_begin(self, trainer, epoch):
        trainer.set_lr(self.schedule(epoch))


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor: str = "val_loss", factor: float = math.sqrt(0.1), patience: int = 5,
                 min_lr: float = 0.5e-6, cooldown: int = 0, min_delta: float = 1e-4, mode: str = "auto"):
        self.monitor, self.factor, self.patience, self.min_lr = monitor, factor, patience, min_lr
        self.cooldown, self.min_delta = cooldown, min_delta
        self.mode = ("max" if "acc" in monitor else "min") if mode == "auto" else mode
        self.best = None
        self.wait = 0
        self.cool = 0

    def _better(self, v):
        if self.best is None:
            return True
        return v > self.best + self.min_delta if self.mode == "max" else v < self.best - self.min_delta

    def on_epoch_end(self, trainer, epoch, logs):
        v = logs.get(self.monitor)
        if v is None:
            return
        if self.cool > 0:
            self.cool -= 1
            self.wait = 0
        if self._better(v):
            self.best, self.wait = v, 0
        elif self.cool <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                new = max(trainer.get_lr() * self.factor, self.min_lr)
                trainer.set_lr(new)
                self.cool, self.wait = self.cooldown, 0


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "val_acc", mode: str = "max", min_delta: float = 0.01, patience: int = 20):
        self.monitor, self.mode, self.min_delta, self.patience = monitor, mode, min_delta, patience
        self.best = None
        self.wait = 0
        self.stopped_epoch = None

    def on_epoch_end(self, trainer, epoch, logs):
        v = logs.get(self.monitor)
        if v is None:
            return
        improved = self.best is None or (v - self.best > self.min_delta if self.mode == "max"
                                         else self.best - v > self.min_delta)
        if improved:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                trainer.stop_training = True
                self.stopped_epoch = epoch


class ModelCheckpoint(Callback):
    """Keep the best weights in memory (optionally also on disk) and restore them at train end."""

    def __init__(self, path: str | None = None, monitor: str = "val_loss", mode: str = "min",
                 save_best_only: bool = True, restore_best: bool = True):
        self.path, self.monitor, self.mode = path, monitor, mode
        self.save_best_only, self.restore_best = save_best_only, restore_best
        self.best = None
        self.best_state = None

    def on_epoch_end(self, trainer, epoch, logs):
        v = logs.get(self.monitor)
        if v is None:
            return
        better = self.best is None or (v < self.best if self.mode == "min" else v > self.best)
        if better or not self.save_best_only:
            self.best = v if better else self.best
            self.best_state = {k: t.detach().clone() for k, t in trainer.model.state_dict().items()}
            if self.path:
                trainer.save(self.path)

    def on_train_end(self, trainer):
        if self.restore_best and self.best_state is not None:
            trainer.model.load_state_dict(self.best_state)


class TimedStopping(Callback):
    def __init__(self, epoch_seconds: float | None = None, total_seconds: float | None = None):
        self.epoch_seconds, self.total_seconds = epoch_seconds, total_seconds
        self.t0 = self.te = 0.0

    def on_train_begin(self, trainer):
        self.t0 = time.time()

    def on_epoch_begin(self, trainer, epoch):
        self.te = time.time()

    def on_epoch_end(self, trainer, epoch, logs):
        now = time.time()
        if self.total_seconds and now - self.t0 > self.total_seconds:
            trainer.stop_training = True
        if self.epoch_seconds and now - self.te > self.epoch_seconds:
            trainer.stop_training = True


class SGDRScheduler(Callback):
    """Cosine annealing with warm restarts, per batch (reference ``sgdr.py``)."""

    def __init__(self, min_lr: float, max_lr: float, steps_per_epoch: int, lr_decay: float = 1.0,
                 cycle_length: int = 10, mult_factor: float = 2.0):
        self.min_lr, self.max_lr, self.lr_decay = min_lr, max_lr, lr_decay
        self.steps_per_epoch, self.cycle_length, self.mult_factor = steps_per_epoch, cycle_length, mult_factor
        self.batch_since_restart = 0
        self.next_restart = cycle_length
        self.best_weights = None
        self.history: dict = {}

    def clr(self) -> float:
        frac = self.batch_since_restart / (self.steps_per_epoch * self.cycle_length)
        return self.min_lr + 0.5 * (self.max_lr - self.min_lr) * (1 + math.cos(frac * math.pi))

    def on_train_begin(self, trainer):
        trainer.set_lr(self.max_lr)

    def on_batch_end(self, trainer, batch, logs):
        self.history.setdefault("lr", []).append(trainer.get_lr())
        self.batch_since_restart += 1
        trainer.set_lr(self.clr())

    def on_epoch_end(self, trainer, epoch, logs):
        if epoch + 1 == self.next_restart:
            self.batch_since_restart = 0
            self.cycle_length = math.ceil(self.cycle_length * self.mult_factor)
            self.next_restart += self.cycle_length
            self.max_lr *= self.lr_decay
            self.best_weights = copy.deepcopy(trainer.model.state_dict())

    def on_train_end(self, trainer):
        if self.best_weights is not None:
            trainer.model.load_state_dict(self.best_weights)


def reference_callbacks(scheduler: bool = False) -> list[Callback]:
    """The callback set ``helpers.train_model`` builds (``helpers.py:72-97``)."""
    cbs: list[Callback] = []
    if scheduler:
        cbs += [ReduceLROnPlateau(), LearningRateScheduler(), EarlyStopping()]
    cbs.append(ModelCheckpoint(monitor="val_loss", mode="min", save_best_only=True))
    return cbs
