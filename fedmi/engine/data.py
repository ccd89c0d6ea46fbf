"""Device-resident datasets, augmentation and client sharding.

Reference data path (src/main.py:36-56): torchvision CIFAR-10, train transform
RandomCrop(32, padding=4) -> RandomHorizontalFlip -> ToTensor -> Normalize, batch
128, and the federated loader is rebuilt every round with shuffle=False
(src/main.py:140) and filtered by ``(batch_idx+1) % world == rank``
(src/main.py:141-145).

fedmi keeps the dataset as uint8 CHW on the client's GPU (CIFAR's own format:
154 MB for 50k images), applies crop/flip/normalize inside the first HIP kernel
with a counter-based RNG (so the epoch can be graph-replayed), and computes the
rank's batch schedule once instead of iterating every batch each round.
The same augmentation is implemented here in PyTorch for the CPU reference
engine and for numerics tests; both use :func:`hash3` bit-for-bit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)
MNIST_MEAN = (0.1307,)
MNIST_STD = (0.3081,)

_M32 = 0xFFFFFFFF


def hash3(a, b, c) -> np.ndarray:
    """Host twin of ``hash3`` in csrc/kernels/common.h (uint32 arithmetic)."""
    a = np.asarray(a, dtype=np.uint64) & _M32
    b = np.asarray(b, dtype=np.uint64) & _M32
    c = np.asarray(c, dtype=np.uint64) & _M32
    h = (a * 0x9E3779B1) & _M32
    h ^= ((b + 0x7F4A7C15) & _M32) * 0x85EBCA77 & _M32
    h ^= ((c + 0x165667B1) & _M32) * 0xC2B2AE3D & _M32
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & _M32
    h ^= h >> 12
    h = (h * 0x297A2D39) & _M32
    h ^= h >> 15
    return h.astype(np.uint64)


def crop_flip_params(seed: int, round_idx: int, gidx: np.ndarray):
    h = hash3(seed, round_idx, gidx)
    i0 = (h % 9).astype(np.int64)
    j0 = ((h >> 8) % 9).astype(np.int64)
    flip = ((h >> 16) & 1).astype(np.int64)
    return i0, j0, flip


def augment_normalize(x_u8: torch.Tensor, gidx: np.ndarray | None, seed: int, round_idx: int,
                      mean=CIFAR_MEAN, std=CIFAR_STD) -> torch.Tensor:
    """uint8 [N,C,H,W] -> float32 normalized, with RandomCrop(pad 4)+HFlip when gidx is given."""
    dev = x_u8.device
    x = x_u8.float() / 255.0
    n, c, hgt, wid = x.shape
    if gidx is not None:
        i0, j0, flip = crop_flip_params(seed, round_idx, gidx)
        pad = torch.nn.functional.pad(x, (4, 4, 4, 4))            # zero pixels, pre-normalize
        ys = torch.arange(hgt, device=dev)[None, :] + torch.as_tensor(i0, device=dev)[:, None]
        xr = torch.arange(wid, device=dev)[None, :]
        fl = torch.as_tensor(flip, device=dev)[:, None].bool()
        xs = torch.where(fl, (wid - 1) - xr, xr) + torch.as_tensor(j0, device=dev)[:, None]
        ni = torch.arange(n, device=dev)[:, None, None, None]
        ci = torch.arange(c, device=dev)[None, :, None, None]
        x = pad[ni, ci, ys[:, None, :, None], xs[:, None, None, :]]
    m = torch.tensor(mean, device=dev, dtype=torch.float32).view(1, -1, 1, 1)
    s = torch.tensor(std, device=dev, dtype=torch.float32).view(1, -1, 1, 1)
    return (x - m) / s


def strided_schedule(n: int, batch: int, rank: int, world: int):
    """Batches owned by ``rank``: batch i iff (i+1) % world == rank (src/main.py:141-145)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    starts, sizes = [], []
    for i in range(math.ceil(n / batch)):
        if (i + 1) % world == rank:
            starts.append(i * batch)
            sizes.append(min(batch, n - i * batch))
    return starts, sizes


def contiguous_schedule(n: int, batch: int):
    starts = list(range(0, n, batch))
    return starts, [min(batch, n - s) for s in starts]


def label_shard_indices(labels: np.ndarray, world: int, shards_per_client: int = 2, seed: int = 0):
    """Non-IID split (McMahan et al.): sort by label, cut into world*spc shards, deal spc per client.

    Each client's indices come back in ascending index order (a fixed shuffle of its labels)."""
    rng = np.random.default_rng(seed)
    order = np.argsort(labels, kind="stable")
    nshards = world * shards_per_client
    shards = np.array_split(order, nshards)
    perm = rng.permutation(nshards)
    out = []
    for r in range(world):
        ids = np.concatenate([shards[j] for j in perm[r * shards_per_client:(r + 1) * shards_per_client]])
        out.append(np.sort(ids))
    return out


@dataclass
class ImageSet:
    x: torch.Tensor          # uint8 [N, C, H, W]
    y: torch.Tensor          # int32 [N]

    def __len__(self):
        return int(self.x.shape[0])

    def to(self, device) -> "ImageSet":
        return ImageSet(self.x.to(device).contiguous(), self.y.to(device).contiguous())

    def subset(self, idx) -> "ImageSet":
        idx_t = torch.as_tensor(np.asarray(idx), dtype=torch.long, device=self.x.device)
        return ImageSet(self.x.index_select(0, idx_t).contiguous(), self.y.index_select(0, idx_t).contiguous())


@dataclass
class FedDataset:
    name: str
    train: ImageSet
    test: ImageSet
    mean: tuple
    std: tuple
    augment: bool

    def to(self, device) -> "FedDataset":
        return FedDataset(self.name, self.train.to(device), self.test.to(device), self.mean, self.std, self.augment)


def _synthetic_images(n: int, shape, n_classes: int, seed: int, device, split: int = 0, contrast: float = 0.12,
                      noise_std: float = 0.3) -> ImageSet:
    """Class-structured synthetic images (learnable), uint8, generated on ``device``.

    The class templates depend only on ``seed`` (shared by train and test);
    labels and noise depend on ``split``.
    """
    gt = torch.Generator(device="cpu").manual_seed(seed)
    g = torch.Generator(device="cpu").manual_seed(seed * 1000003 + split)
    c, h, w = shape
    # low-frequency class templates: random 8x8 patterns upsampled to HxW
    base = torch.rand(n_classes, c, 8, 8, generator=gt)
    templates = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
    labels = torch.randint(0, n_classes, (n,), generator=g, dtype=torch.int64)
    templates = templates.to(device)
    labels_d = labels.to(device)
    out = torch.empty(n, c, h, w, dtype=torch.uint8, device=device)
    chunk = 8192
    gd = torch.Generator(device=device).manual_seed(seed * 1000003 + split + 1)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        noise = torch.randn(e - s, c, h, w, generator=gd, device=device) * noise_std
        # contrast/noise chosen so the reference recipe (SGD lr 0.1, m 0.9, no BN) trains
        # LeNet stably for 24+ epochs (fp32 torch: ~50 % test acc, loss ~1.77); higher
        # contrast makes that recipe diverge to a dead network after ~12 epochs
        img = templates[labels_d[s:e]] * contrast + 0.5 - contrast / 2 + noise
        out[s:e] = (img.clamp_(0, 1) * 255.0).round_().to(torch.uint8)
    return ImageSet(out, labels_d.to(torch.int32))


def synthetic_cifar10(n_train=50000, n_test=10000, seed=0, device="cpu", contrast=0.12, noise_std=0.3) -> FedDataset:
    tr = _synthetic_images(n_train, (3, 32, 32), 10, seed, device, split=0, contrast=contrast, noise_std=noise_std)
    te = _synthetic_images(n_test, (3, 32, 32), 10, seed, device, split=1, contrast=contrast, noise_std=noise_std)
    return FedDataset("synthetic-cifar10", tr, te, CIFAR_MEAN, CIFAR_STD, True)


def synthetic_mnist(n_train=60000, n_test=10000, seed=0, device="cpu") -> FedDataset:
    tr = _synthetic_images(n_train, (1, 28, 28), 10, seed, device, split=0)
    te = _synthetic_images(n_test, (1, 28, 28), 10, seed, device, split=1)
    return FedDataset("synthetic-mnist", tr, te, MNIST_MEAN, MNIST_STD, False)


def _read_cifar_bin(path: Path) -> ImageSet:
    raw = np.fromfile(path, dtype=np.uint8)
    if raw.size % 3073:
        raise ValueError(f"{path}: not a CIFAR-10 binary batch")
    raw = raw.reshape(-1, 3073)
    y = torch.from_numpy(raw[:, 0].astype(np.int32))
    x = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).copy())
    return ImageSet(x, y)


def cifar10_binary(root: str | Path) -> FedDataset:
    """Real CIFAR-10 from the *binary* distribution (data_batch_1..5.bin, test_batch.bin).

    The python-pickle distribution is deliberately unsupported (no unpickling).
    """
    root = Path(root)
    parts = [_read_cifar_bin(root / f"data_batch_{i}.bin") for i in range(1, 6)]
    train = ImageSet(torch.cat([p.x for p in parts]), torch.cat([p.y for p in parts]))
    test = _read_cifar_bin(root / "test_batch.bin")
    return FedDataset("cifar10", train, test, CIFAR_MEAN, CIFAR_STD, True)


def make_dataset(spec: str, device="cpu", n_train: int | None = None, n_test: int | None = None,
                 seed: int = 0) -> FedDataset:
    """``synthetic-cifar10`` | ``synthetic-cifar10-easy`` | ``synthetic-mnist`` | ``cifar10-bin:<dir>``.

    ``-easy``: high-contrast, low-noise templates (deep BN nets learn it in a few epochs; the
    default low-contrast set is tuned so the reference LeNet recipe trains stably)."""
    if spec.startswith("cifar10-bin:"):
        ds = cifar10_binary(spec.split(":", 1)[1])
        if n_train:
            ds.train = ImageSet(ds.train.x[:n_train], ds.train.y[:n_train])
        if n_test:
            ds.test = ImageSet(ds.test.x[:n_test], ds.test.y[:n_test])
        return ds.to(device)
    if spec in ("synthetic-cifar10", "synthetic", "cifar10-synthetic"):
        return synthetic_cifar10(n_train or 50000, n_test or 10000, seed, device)
    if spec == "synthetic-cifar10-easy":
        return synthetic_cifar10(n_train or 50000, n_test or 10000, seed, device, contrast=0.6, noise_std=0.1)
    if spec in ("synthetic-mnist", "mnist-synthetic"):
        return synthetic_mnist(n_train or 60000, n_test or 10000, seed, device)
    raise ValueError(f"unknown dataset spec {spec!r}")
