"""Host data pipeline feeding the train step.

Mirrors the reference's datasets and loader:
  * ``Depth10k(image_dir, image_files; augmentations, grayscale)``  src/dtk.jl:1-49
    one PNG per sample holding the three frames side by side (3*416 x 128), split at
    ``width*j`` (dtk.jl:36), optional ``Gray{Float32}`` conversion (dtk.jl:32-34);
  * ``KittyDataset(image_dir, sequence; target_size, augmentations)``  src/kitty.jl:1-84
    consecutive ``image_0/%06d.png`` triplets, ``calib.txt`` P0 -> K rescaled to the target
    size (kitty.jl:19-44, 83-96), resize to ``target_size`` (kitty.jl:52);
  * ``DChain(datasets)``  src/dchain.jl:1-30 (concatenation by cumulative bins);
  * ``FlipX(p)``  Augmentations.jl as used by scripts/script.jl:38 -- one coin per sample, the
    same flip applied to all three frames (the frames stay geometrically consistent);
  * ``DataLoader(dataset, batch_size)``  DataLoaders.jl as used by scripts/script.jl:90 --
    worker threads decode (PIL releases the GIL while decoding), batches are collated into
    pinned host memory in the library's layout ``x[N][3][C][H][W]`` (Julia ``(W,H,C,3,N)``,
    same bytes) and copied to the GPU on a side stream, one batch ahead of the consumer.
    With ``rank``/``world`` the sample order is sharded by global index (md2hip.dist).

Sample layout returned by ``__getitem__``: float32 numpy ``[3 frames][C][H][W]`` in [0, 1].
Assumptions (third-party semantics, unpinned -- no reference test covers the loaders): Gray
conversion uses the ITU-R BT.601 weights (0.299, 0.587, 0.114) of Colors.jl; ``imresize`` is
restated as PIL bilinear resampling (ImageTransformations' interpolation / antialiasing filter is
not reproduced bit-for-bit).
"""
from __future__ import annotations

import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np

from .dist import shard_range

_GRAY = np.array([0.299, 0.587, 0.114], dtype=np.float32)


def _load_png(path: str) -> np.ndarray:
    """PNG -> float32 [C][H][W] in [0, 1] (N0f8 / N0f16 -> Float32, channelview)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I"):
            a = np.asarray(im, dtype=np.float32) / 65535.0
            return a[None]
        if im.mode not in ("L", "RGB"):
            im = im.convert("RGB")
        a = np.asarray(im, dtype=np.float32) / 255.0
    return a[None] if a.ndim == 2 else np.ascontiguousarray(a.transpose(2, 0, 1))


def _to_gray(chw: np.ndarray) -> np.ndarray:
    if chw.shape[0] == 1:
        return chw
    return np.tensordot(_GRAY, chw, axes=(0, 0))[None].astype(np.float32)


def _resize(chw: np.ndarray, height: int, width: int) -> np.ndarray:
    if chw.shape[1:] == (height, width):
        return chw
    from PIL import Image
    out = np.empty((chw.shape[0], height, width), dtype=np.float32)
    for c in range(chw.shape[0]):
        out[c] = np.asarray(Image.fromarray(chw[c], mode="F").resize((width, height), Image.BILINEAR))
    return out


class FlipX:
    """``FlipX(p)``: mirror every frame of a sample left-right with probability ``p``."""

    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, frames: List[np.ndarray], rng: np.random.Generator) -> List[np.ndarray]:
        if rng.random() < self.p:
            return [np.ascontiguousarray(f[..., ::-1]) for f in frames]
        return frames


def intrinsics(fx: float, fy: float, cx: float, cy: float) -> np.ndarray:
    """``construct_intrinsic`` (src/kitty.jl:92-97)."""
    return np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]])


class _Dataset:
    source_ids = (1, 3)
    target_id = 2
    augmentations = None

    def _augment(self, frames, i: int, seed: int):
        if self.augmentations is None:
            return frames
        return self.augmentations(frames, np.random.default_rng((seed, i)))


class Depth10k(_Dataset):
    """``Depth10k(image_dir, image_files; augmentations=nothing, grayscale=false)`` (src/dtk.jl:15-26)."""

    def __init__(self, image_dir: str, image_files: Sequence[str], *, augmentations=None,
                 grayscale: bool = False):
        focal = 2648.0 / 4.63461538462
        self.resolution = (416, 128)                 # (width, height)
        self.K = intrinsics(focal, focal, 416 / 2.0, 128 / 2.0)
        self.invK = np.linalg.inv(self.K)
        self.dir, self.files = image_dir, list(image_files)
        self.augmentations, self.grayscale = augmentations, grayscale
        self.channels = 1 if grayscale else 3

    def __len__(self):
        return len(self.files)

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        """Sample ``i`` (0-based): float32 [3][C][H][W] (dtk.jl:29-46)."""
        width, height = self.resolution
        img = _load_png(os.path.join(self.dir, self.files[i]))
        if self.grayscale:
            img = _to_gray(img)
        if img.shape[1] != height or img.shape[2] != 3 * width:
            raise ValueError(f"{self.files[i]}: expected {3 * width}x{height} triplet, got "
                             f"{img.shape[2]}x{img.shape[1]}")
        frames = [img[:, :, width * j:width * (j + 1)] for j in range(3)]
        frames = self._augment(frames, i, seed)
        return np.stack(frames, 0)

    __getitem__ = getobs


def _parse_calib_P0(line: str) -> np.ndarray:
    """``parse_matrix`` (src/kitty.jl:86-90) of the ``P0:`` line -> K (3x3)."""
    vals = [float(v) for v in line.split(":", 1)[1].split()]
    return np.array(vals, dtype=np.float64).reshape(3, 4)[:, :3]


class KittyDataset(_Dataset):
    """``KittyDataset(image_dir, sequence; target_size=(height, width), augmentations)``
    (src/kitty.jl:19-44): grayscale ``image_0`` frames, non-overlapping triplets."""

    def __init__(self, image_dir: str, sequence: str, *, target_size, augmentations=None):
        seq_dir = os.path.join(image_dir, "sequences", sequence)
        with open(os.path.join(seq_dir, "calib.txt")) as f:
            K0 = _parse_calib_P0(f.readline())
        self.frames_dir = os.path.join(seq_dir, "image_0")
        files = sorted(os.listdir(self.frames_dir))
        n_frames = len(files)
        orig = _load_png(os.path.join(self.frames_dir, files[0])).shape[1:]   # (height, width)
        height, width = target_size
        fx = float(np.mean(np.array(target_size, dtype=np.float64) / np.array(orig))) * K0[0, 0]
        self.K = intrinsics(fx, fx, width // 2, height // 2)
        self.invK = np.linalg.inv(self.K)
        self.resolution = (width, height)
        self.frame_ids = (1, 2, 3)
        self.total_length = n_frames // len(self.frame_ids)
        self.augmentations = augmentations
        self.channels = 1

    def __len__(self):
        return self.total_length

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        """Sample ``i`` (0-based): frames 3i, 3i+1, 3i+2 (kitty.jl:47-61) -> [3][1][H][W]."""
        width, height = self.resolution
        sid = i * len(self.frame_ids)
        frames = []
        for x in self.frame_ids:
            img = _to_gray(_load_png(os.path.join(self.frames_dir, "%06d.png" % (sid + x - 1))))
            frames.append(_resize(img, height, width))
        frames = self._augment(frames, i, seed)
        return np.stack(frames, 0)

    __getitem__ = getobs


class DChain:
    """``DChain(datasets)`` (src/dchain.jl:1-30)."""

    def __init__(self, datasets: Sequence):
        self.datasets = list(datasets)
        self.bins = np.cumsum([len(d) for d in self.datasets]).tolist()
        self.channels = self.datasets[0].channels
        self.resolution = self.datasets[0].resolution

    def __len__(self):
        return self.bins[-1] if self.bins else 0

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        if not 0 <= i < len(self):
            raise IndexError(i)
        bid = next(b for b, edge in enumerate(self.bins) if i < edge)
        return self.datasets[bid].getobs(i - (self.bins[bid - 1] if bid else 0), seed)

    __getitem__ = getobs


class DataLoader:
    """Batches of ``batch_size`` samples as a tensor ``[N][3][C][H][W]`` on ``device``.

    Epoch order: ``shuffle`` permutes with ``seed + epoch``; the global batch ``batch_size *
    world`` is cut into per-rank shards by global index (md2hip.dist.shard_range), so the union
    over ranks is identical for every GPU count.  Incomplete trailing batches are dropped
    (fixed-shape train step).  ``workers`` decode threads; one batch is prefetched and its
    host->device copy runs on a side stream while the previous batch trains."""

    def __init__(self, dataset, batch_size: int, *, shuffle: bool = True, seed: int = 0,
                 workers: int = 8, device=None, rank: int = 0, world: int = 1, prefetch: int = 2):
        self.ds, self.batch_size, self.shuffle, self.seed = dataset, batch_size, shuffle, seed
        self.workers, self.rank, self.world, self.prefetch = workers, rank, world, prefetch
        self.device = device
        self.epoch = 0

    def __len__(self):
        return len(self.ds) // (self.batch_size * self.world)

    def _order(self, epoch: int) -> np.ndarray:
        n = len(self.ds)
        if not self.shuffle:
            return np.arange(n)
        return np.random.default_rng((self.seed, epoch)).permutation(n)

    def batch_indices(self, epoch: int) -> List[List[int]]:
        order = self._order(epoch)
        gb = self.batch_size * self.world
        lo, hi = shard_range(gb, self.world, self.rank)
        return [order[b * gb + lo:b * gb + hi].tolist() for b in range(len(order) // gb)]

    def __iter__(self):
        import torch
        epoch = self.epoch
        self.epoch += 1
        batches = self.batch_indices(epoch)
        dev = torch.device(self.device) if self.device is not None else None
        on_gpu = dev is not None and dev.type == "cuda"
        stream = torch.cuda.Stream(device=dev) if on_gpu else None
        q: "queue.Queue" = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def produce():
            try:
                with ThreadPoolExecutor(self.workers) as pool:
                    for idx in batches:
                        if stop.is_set():
                            return
                        samples = list(pool.map(lambda i: self.ds.getobs(i, seed=self.seed + epoch), idx))
                        host = torch.from_numpy(np.stack(samples, 0))
                        if on_gpu:
                            host = host.pin_memory()
                            with torch.cuda.stream(stream):
                                x = host.to(dev, non_blocking=True)
                                ev = torch.cuda.Event()
                                ev.record(stream)
                            q.put((x, ev, host))
                        else:
                            q.put((host.to(dev) if dev is not None else host, None, None))
            except BaseException as e:            # surface decode errors in the consumer
                q.put(e)
            finally:
                q.put(None)

        t = threading.Thread(target=produce, daemon=True)
        t.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    break
                if isinstance(item, BaseException):
                    raise item
                x, ev, _host = item
                if ev is not None:
                    torch.cuda.current_stream(dev).wait_event(ev)
                    x.record_stream(torch.cuda.current_stream(dev))
                yield x
        finally:
            stop.set()
            while t.is_alive():
                try:
                    q.get(timeout=0.1)
                except queue.Empty:
                    pass
            t.join()


def find_static(dataset, alpha: float, batch: int = 16, device=None, seed: int = 0) -> List[str]:
    """``find_static(dataset, α)`` (src/dtk.jl:51-69): the files of the samples whose mean
    identity-reprojection loss (``automasking_loss`` of the raw frames against the target) exceeds
    ``alpha`` -- the non-static triplets, in dataset order.  Scores on the GPU in batches
    (``md2_static_scores``); no CPU fallback."""
    import torch
    from .primitives import static_scores
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    src = tuple(dataset.source_ids)
    keep: List[str] = []
    for b0 in range(0, len(dataset), batch):
        idx = list(range(b0, min(len(dataset), b0 + batch)))
        x = torch.from_numpy(np.stack([dataset.getobs(i, seed) for i in idx])).to(dev).contiguous()
        scores = static_scores(x, dataset.target_id, src).cpu().tolist()
        keep.extend(dataset.files[i] for i, s in zip(idx, scores) if s > alpha)
    return keep
