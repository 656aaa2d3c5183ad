"""Datasets and device-resident loaders.

Reference parity: ``TensorflowGenerator.init_dataset`` (``tensorflow_generator.py:280-353``:
MNIST / CIFAR-10 / CIFAR-100 via ``keras.datasets``, reshape to NHWC, /255,
cached per name, first 500 test samples as the robustness set) and the
ImageDataGenerator augmentation of ``helpers.py:112-167`` (width/height
shift 0.1 with nearest fill, horizontal flip).

There is no network here, so image datasets are read from local files when
present (``$FEATURENET_DATA`` or ``~/.keras/datasets``: ``mnist.npz``,
``cifar-10-batches-bin/``, ``cifar-100-binary/`` -- formats that need no
unpickling) and otherwise replaced by a synthetic stand-in of identical
shape and class count (``Dataset.synthetic`` is then True and every report
says so).  The voxel workload uses the native procedural generator
(``csrc/runtime/voxel.cpp``) or a folder of ``.binvox`` files.

Everything is kept on the GPU (a full CIFAR epoch is ~150 MB; HBM is
288 GB), shuffling is a device permutation and augmentation runs as batched
index gathers -- the training loop never waits on host I/O.  Voxel grids
stay bit-packed on the device and are expanded per batch by the
``unpack_bits`` HIP kernel.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import torch

from .. import _native

DATASET_CLASSES = {"mnist": 10, "cifar": 10, "cifar10": 10, "cifar100": 100, "voxel": 24, "featurenet24": 24}
DATASET_SHAPES = {"mnist": (28, 28, 1), "cifar": (32, 32, 3), "cifar10": (32, 32, 3), "cifar100": (32, 32, 3)}


@dataclass
class Dataset:
    name: str
    x_train: np.ndarray | torch.Tensor
    y_train: np.ndarray | torch.Tensor
    x_test: np.ndarray | torch.Tensor
    y_test: np.ndarray | torch.Tensor
    num_classes: int
    input_shape: tuple
    synthetic: bool = False
    packed: bool = False            # voxel grids stored bit-packed (uint8 [N, S^3/8])
    meta: dict = field(default_factory=dict)

    def robustness_set(self, size: int = 500):
        """The first ``size`` test samples (reference ``tensorflow_generator.py:350-351``)."""
        return self.x_test[:size], self.y_test[:size]


_CACHE: dict = {}


def _data_roots() -> list[Path]:
    roots = []
    if os.environ.get("FEATURENET_DATA"):
        roots.append(Path(os.environ["FEATURENET_DATA"]))
    roots.append(Path.home() / ".keras" / "datasets")
    return roots


def _find(name: str) -> Path | None:
    for r in _data_roots():
        p = r / name
        if p.exists():
            return p
    return None


def _load_mnist() -> tuple | None:
    p = _find("mnist.npz")
    if p is None:
        return None
    with np.load(p, allow_pickle=False) as d:
        return d["x_train"], d["y_train"], d["x_test"], d["y_test"]


def _read_cifar_bin(files: list[Path], label_bytes: int, label_index: int):
    xs, ys = [], []
    rec = label_bytes + 3072
    for f in files:
        raw = np.fromfile(f, dtype=np.uint8).reshape(-1, rec)
        ys.append(raw[:, label_index].astype(np.int64))
        xs.append(raw[:, label_bytes:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return np.concatenate(xs), np.concatenate(ys)


def _load_cifar10() -> tuple | None:
    d = _find("cifar-10-batches-bin")
    if d is None:
        return None
    xtr, ytr = _read_cifar_bin([d / f"data_batch_{i}.bin" for i in range(1, 6)], 1, 0)
    xte, yte = _read_cifar_bin([d / "test_batch.bin"], 1, 0)
    return xtr, ytr, xte, yte


def _load_cifar100() -> tuple | None:
    d = _find("cifar-100-binary")
    if d is None:
        return None
    xtr, ytr = _read_cifar_bin([d / "train.bin"], 2, 1)
    xte, yte = _read_cifar_bin([d / "test.bin"], 2, 1)
    return xtr, ytr, xte, yte


def _synthetic_images(shape, n_classes, n_train, n_test, seed):
    """Learnable stand-in: class-dependent blob position + noise (same shapes as the real set)."""
    g = np.random.default_rng(seed)
    H, W, C = shape

    def make(n):
        y = g.integers(0, n_classes, n)
        x = g.normal(0.2, 0.1, (n, H, W, C)).astype(np.float32)
        cy = (y * 7 % max(H - 6, 1)) + 3
        cx = (y * 13 % max(W - 6, 1)) + 3
        yy, xx = np.mgrid[0:H, 0:W]
        for i in range(n):
            x[i, (yy - cy[i]) ** 2 + (xx - cx[i]) ** 2 < 9, :] += 0.7
        return np.clip(x, 0, 1), y.astype(np.int64)

    xtr, ytr = make(n_train)
    xte, yte = make(n_test)
    return xtr, ytr, xte, yte


def load_dataset(name: str, synthetic_sizes=(6000, 1000), seed: int = 0, allow_synthetic: bool = True) -> Dataset:
    """``mnist`` / ``cifar`` (= ``cifar10``) / ``cifar100`` / ``voxel``; cached per name."""
    key = (name, synthetic_sizes, seed)
    if key in _CACHE:
        return _CACHE[key]
    name_l = name.lower()
    if name_l in ("voxel", "featurenet24"):
        ds = voxel_dataset(*synthetic_sizes, size=64, seed=seed)
    else:
        loader = {"mnist": _load_mnist, "cifar": _load_cifar10, "cifar10": _load_cifar10,
                  "cifar100": _load_cifar100}.get(name_l)
        if loader is None:
            raise ValueError(f"unknown dataset {name!r}")
        shape = DATASET_SHAPES[name_l]
        ncls = DATASET_CLASSES[name_l]
        raw = loader()
        synthetic = raw is None
        if synthetic:
            if not allow_synthetic:
                raise FileNotFoundError(f"dataset {name} not found under {[str(r) for r in _data_roots()]}")
            xtr, ytr, xte, yte = _synthetic_images(shape, ncls, synthetic_sizes[0], synthetic_sizes[1], seed)
        else:
            xtr, ytr, xte, yte = raw
            xtr = xtr.reshape((-1,) + shape).astype(np.float32) / 255.0
            xte = xte.reshape((-1,) + shape).astype(np.float32) / 255.0
        ds = Dataset(name_l, xtr, np.asarray(ytr, np.int64).reshape(-1), xte, np.asarray(yte, np.int64).reshape(-1),
                     ncls, shape, synthetic=synthetic)
    _CACHE[key] = ds
    return ds


def voxel_dataset(n_train: int, n_test: int, size: int = 64, num_classes: int = 24, seed: int = 0) -> Dataset:
    """Procedural machining-feature voxel dataset (bit-packed), see ``csrc/runtime/voxel.cpp``."""
    rt = _native.runtime()
    xtr, ytr = rt.generate_voxels(n_train, size, seed, num_classes)
    xte, yte = rt.generate_voxels(n_test, size, seed + 1_000_003, num_classes)
    return Dataset("voxel", xtr, ytr, xte, yte, num_classes, (size, size, size, 1), synthetic=True, packed=True,
                   meta={"generator": "featurenet_amd._rt.generate_voxels", "seed": seed})


def binvox_folder(root: str | Path, size: int | None = None) -> tuple[np.ndarray, np.ndarray, list[str]]:
    """Load ``root/<class>/*.binvox`` -> (bit-packed grids, labels, class names)."""
    rt = _native.runtime()
    root = Path(root)
    classes = sorted(d.name for d in root.iterdir() if d.is_dir())
    xs, ys = [], []
    for ci, c in enumerate(classes):
        for f in sorted((root / c).glob("*.binvox")):
            grid, _, _ = rt.read_binvox(str(f))
            if size is not None and grid.shape[0] != size:
                raise ValueError(f"{f}: grid {grid.shape[0]} != {size}")
            xs.append(rt.pack_bits(grid.reshape(-1)))
            ys.append(ci)
    return np.stack(xs), np.asarray(ys, np.int64), classes


# ---------------------------------------------------------------------------
# device-side batching
# ---------------------------------------------------------------------------
def unpack_voxels(bits: torch.Tensor, size: int) -> torch.Tensor:
    """uint8 [B, S^3/8] (device) -> bf16 [B, S, S, S, 1]."""
    B = bits.shape[0]
    out = torch.empty(B, size, size, size, 1, dtype=torch.bfloat16, device=bits.device)
    if bits.is_cuda and _native.use_native(bits):
        _native.kernels().unpack_bits(bits.data_ptr(), out.data_ptr(), bits.numel(), _native.stream(bits))
        return out
    shifts = torch.arange(8, device=bits.device, dtype=torch.uint8)
    dense = ((bits.unsqueeze(-1) >> shifts) & 1).reshape(B, size, size, size, 1)
    return dense.to(out.dtype)


def augment_images(x: torch.Tensor, shift: float = 0.1, hflip: bool = True,
                   generator: torch.Generator | None = None) -> torch.Tensor:
    """Random integer shifts (nearest fill) + horizontal flip on [B, H, W, C] (helpers.py:131-145)."""
    B, H, W, _ = x.shape
    dev = x.device
    dy = torch.randint(-int(shift * H), int(shift * H) + 1, (B, 1), device=dev, generator=generator)
    dx = torch.randint(-int(shift * W), int(shift * W) + 1, (B, 1), device=dev, generator=generator)
    rows = (torch.arange(H, device=dev).unsqueeze(0) - dy).clamp_(0, H - 1)
    cols = (torch.arange(W, device=dev).unsqueeze(0) - dx)
    if hflip:
        flip = torch.rand(B, 1, device=dev, generator=generator) < 0.5
        cols = torch.where(flip, W - 1 - cols, cols)
    cols = cols.clamp_(0, W - 1)
    bidx = torch.arange(B, device=dev)[:, None, None]
    return x[bidx, rows[:, :, None], cols[:, None, :]]


class DeviceLoader:
    """Shuffled mini-batches from device-resident arrays.

    Data parallelism (reference ``model/keras_model.py:137-146``: ``multi_gpu_model``
    slices every batch of a Keras ``fit`` that reshuffles each epoch, so every replica
    sees a random cross-section of the whole set): every rank holds the WHOLE set on
    its device (bit-packed voxels are 32 KB per 64^3 grid; HBM is 288 GB) and, each
    epoch, takes the rank-strided slice ``perm[rank::world]`` of ONE global permutation
    drawn from ``(seed, epoch)`` -- identical on every rank, so the shards partition the
    epoch and change between epochs, whatever order the set is stored in (e.g. the
    class-sorted :func:`binvox_folder`).  Training shards are cut to ``n // world``
    samples (equal step counts on every rank: the per-step gradient all-reduce needs
    them); ``even=False`` (evaluation) keeps every sample exactly once instead.

    ``gen`` (seeded ``seed + rank``) drives the augmentation draws only; the shuffle is
    a pure function of ``(seed, epoch)`` (:meth:`set_epoch`), so a resumed run needs the
    epoch count, not a generator state, to reproduce the order."""

    def __init__(self, x, y, batch_size: int, device, shuffle: bool = True, augment: bool = False,
                 packed_size: int | None = None, rank: int = 0, world: int = 1, drop_last: bool = False,
                 seed: int = 0, dtype=None, even: bool = True):
        self.device = torch.device(device)
        self.packed_size = packed_size
        xt = torch.as_tensor(np.asarray(x)) if not isinstance(x, torch.Tensor) else x
        yt = torch.as_tensor(np.asarray(y)) if not isinstance(y, torch.Tensor) else y
        if dtype is None:
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        if packed_size is None and xt.dtype != torch.uint8:
            xt = xt.to(dtype)
        self.x = xt.to(self.device)
        self.y = yt.long().to(self.device)
        self.batch_size, self.shuffle, self.augment, self.drop_last = batch_size, shuffle, augment, drop_last
        self.dtype = dtype
        self.rank, self.world, self.seed, self.even = int(rank), max(1, int(world)), int(seed), bool(even)
        self.epoch = 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + rank)

    def derived(self, shuffle: bool = True, seed: int = 0, augment: bool = False) -> "DeviceLoader":
        """Another loader over the SAME device-resident tensors (no re-upload of the set):
        own shuffle seed / epoch / augmentation generator, e.g. PreciseBN recalibration
        batches during fit."""
        d = object.__new__(DeviceLoader)
        d.__dict__.update(self.__dict__)
        d.shuffle, d.augment, d.seed, d.epoch = shuffle, augment, int(seed), 0
        d.gen = torch.Generator(device=self.device)
        d.gen.manual_seed(seed + self.rank)
        return d

    def set_epoch(self, epoch: int) -> None:
        """The epoch whose global permutation the next iteration uses."""
        self.epoch = int(epoch)

    def shard_size(self) -> int:
        n = len(self.x)
        if self.world == 1:
            return n
        return n // self.world if self.even else len(range(self.rank, n, self.world))

    def indices(self, epoch: int | None = None) -> torch.Tensor:
        """This rank's sample indices of ``epoch`` (default: the next one), in batch order (CPU)."""
        n = len(self.x)
        e = self.epoch if epoch is None else int(epoch)
        if self.shuffle:
            g = torch.Generator()                # CPU: bit-identical on every rank and device type
            g.manual_seed((self.seed * 1_000_003 + e * 7_919 + 12_345) & 0x7FFF_FFFF_FFFF_FFFF)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if self.world > 1:
            idx = idx[self.rank::self.world]
            if self.even:
                idx = idx[:n // self.world]
        return idx

    def __len__(self) -> int:
        n = self.shard_size()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        idx = self.indices().to(self.device)
        self.epoch += 1
        for i in range(len(self)):
            sel = idx[i * self.batch_size:(i + 1) * self.batch_size]
            xb = self.x[sel]
            if self.packed_size is not None:
                xb = unpack_voxels(xb, self.packed_size)
                if self.device.type != "cuda":
                    xb = xb.float()
            if self.augment and xb.dim() == 4:
                xb = augment_images(xb, generator=self.gen)
            yield xb, self.y[sel]
