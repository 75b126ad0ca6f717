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
    same bytes) and copied to the GPU on a side stream, one batch ahead of the consumer.  The
    N0f8 datasets (RGB Depth10k, KITTI) cross PCIe as BYTES and become Float32 on the GPU
    (``md2_unorm8_to_float``: Float32(u) / 255f0, bit-identical to the host conversion) -- a
    quarter of the H2D traffic and no float conversion on the host.  With ``rank``/``world``
    the sample order is sharded by global index (md2hip.dist).

Sample layout returned by ``__getitem__``: float32 numpy ``[3 frames][C][H][W]`` in [0, 1];
``getobs_u8`` gives the same sample as the uint8 N0f8 bytes where the dataset's element type is
N0f8 (RGB Depth10k, KITTI; not grayscale Depth10k, whose Gray{Float32} values are not bytes).
Third-party semantics (unpinned -- no reference test or fixture covers the loaders):
  * Gray conversion: the ITU-R BT.601 weights (0.299, 0.587, 0.114) of Colors.jl;
  * ``imresize`` (ImageTransformations.jl, src/kitty.jl:52): restated from its published
    algorithm (``imresize!``): the outer pixel corners of both images are mapped onto each other,
    i.e. output pixel i (1-based) samples the input at ``sf * (i - 1/2) + 1/2`` with
    ``sf = n_in / n_out`` per axis (clamped to [1, n_in] when upsampling), by
    ``BSpline(Linear())`` interpolation (bilinear, NO antialiasing filter), and the result is
    stored back in the input's element type -- N0f8 for the KITTI ``image_0`` PNGs, i.e. rounded
    to the nearest 1/255.  Pinned here by known answers (tests/test_data.py) and cross-checked
    against torch's ``interpolate(align_corners=False, antialias=False)``, the same map.
"""
from __future__ import annotations

import ctypes as C
import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence

import numpy as np

from .dist import shard_range

_GRAY = np.array([0.299, 0.587, 0.114], dtype=np.float32)


def _load_png_raw(path: str) -> np.ndarray:
    """PNG -> its stored integers [C][H][W] (uint8 for N0f8, uint16 for N0f16 images)."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I"):
            return np.asarray(im, dtype=np.uint16)[None]
        if im.mode not in ("L", "RGB"):
            im = im.convert("RGB")
        a = np.asarray(im, dtype=np.uint8)
    return a[None] if a.ndim == 2 else np.ascontiguousarray(a.transpose(2, 0, 1))


def _unorm(a: np.ndarray) -> np.ndarray:
    """N0f8 / N0f16 -> Float32: Float32(u) / 255f0 (or 65535f0), as ``Float32.(channelview)``."""
    return a.astype(np.float32) / np.float32(65535.0 if a.dtype == np.uint16 else 255.0)


def _load_png(path: str) -> np.ndarray:
    """PNG -> float32 [C][H][W] in [0, 1] (N0f8 / N0f16 -> Float32, channelview)."""
    return _unorm(_load_png_raw(path))


def _to_gray(chw: np.ndarray) -> np.ndarray:
    if chw.shape[0] == 1:
        return chw
    return np.tensordot(_GRAY, chw, axes=(0, 0))[None].astype(np.float32)


def _imresize_axis(n_in: int, n_out: int):
    """Per output index: (i0, i1, f) of ``imresize!``'s sample position (module docstring)."""
    sf = n_in / n_out
    p = sf * (np.arange(1, n_out + 1, dtype=np.float64) - 0.5) + 0.5      # 1-based position
    if sf < 1:
        p = np.clip(p, 1.0, float(n_in))
    p -= 1.0                                                              # 0-based
    i0 = np.minimum(np.floor(p).astype(np.int64), n_in - 1)
    f = p - i0
    i1 = np.minimum(i0 + 1, n_in - 1)
    return i0, i1, f


def imresize(chw: np.ndarray, height: int, width: int) -> np.ndarray:
    """``imresize(img, (height, width))`` of ImageTransformations.jl (src/kitty.jl:52) on
    [C][H][W] images: bilinear at the outer-corner-aligned positions, no antialiasing; N0f8
    (uint8) input -> N0f8 output rounded to the nearest 1/255 (the element type is kept), float
    input -> float64 values."""
    if chw.shape[1:] == (height, width):
        return chw
    y0, y1, fy = _imresize_axis(chw.shape[1], height)
    x0, x1, fx = _imresize_axis(chw.shape[2], width)
    v = chw.astype(np.float64) / 255.0 if chw.dtype == np.uint8 else chw.astype(np.float64)
    fx = fx[None, None, :]
    fy = fy[None, :, None]
    top = v[:, y0][:, :, x0] * (1 - fx) + v[:, y0][:, :, x1] * fx
    bot = v[:, y1][:, :, x0] * (1 - fx) + v[:, y1][:, :, x1] * fx
    out = top * (1 - fy) + bot * fy
    if chw.dtype == np.uint8:
        return np.rint(out * 255.0).astype(np.uint8)
    return out


class FlipX:
    """``FlipX(p)``: mirror every frame of a sample left-right with probability ``p``."""

    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, frames: List[np.ndarray], rng: np.random.Generator) -> List[np.ndarray]:
        if rng.random() < self.p:
            return [np.ascontiguousarray(f[..., ::-1]) for f in frames]
        return frames


def _torch_from(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a))


def _addr(a) -> int:
    """Data pointer of a C-contiguous numpy array or CPU torch tensor."""
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    assert a.is_contiguous() and not a.is_cuda
    return a.data_ptr()


def intrinsics(fx: float, fy: float, cx: float, cy: float) -> np.ndarray:
    """``construct_intrinsic`` (src/kitty.jl:92-97)."""
    return np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]])


class _Dataset:
    source_ids = (1, 3)
    target_id = 2
    augmentations = None
    u8 = False                     # getobs_u8 gives the sample's N0f8 bytes

    def _augment(self, frames, i: int, seed: int):
        if self.augmentations is None:
            return frames
        return self.augmentations(frames, np.random.default_rng((seed, i)))

    def _native_flips(self, idx, seed):
        """The FlipX coins of samples ``idx`` (the same draws as _augment), or None when the
        augmentations are not the natively supported ones (nothing or one FlipX)."""
        a = self.augmentations
        if a is None:
            return np.zeros(len(idx), dtype=np.uint8)
        if isinstance(a, FlipX):
            return np.array([np.random.default_rng((seed, i)).random() < a.p for i in idx], dtype=np.uint8)
        return None

    def batch_u8(self, idx, seed: int = 0, threads: int = 8, out=None):
        """Samples ``idx`` as one uint8 [n][3][C][H][W] array, decoded by the library's native
        loader on ``threads`` host threads (md2_load_*_u8); the per-sample Python path when the
        augmentations are not natively supported.  ``out``: a caller buffer (e.g. pinned)."""
        w, h = self.resolution
        if out is None:
            out = np.empty((len(idx), 3, self.channels, h, w), dtype=np.uint8)
        flips = self._native_flips(idx, seed)
        if flips is None:
            for k, i in enumerate(idx):
                s = self.getobs_u8(i, seed)
                out[k] = s if isinstance(out, np.ndarray) else _torch_from(s)
            return out
        self._native_load(idx, flips, out, threads)
        return out

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        return _unorm(self.getobs_u8(i, seed))

    __getitem__ = getobs


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
        self.u8 = not grayscale

    def __len__(self):
        return len(self.files)

    def _frames(self, img, i, seed):
        width, height = self.resolution
        if img.shape[1] != height or img.shape[2] != 3 * width:
            raise ValueError(f"{self.files[i]}: expected {3 * width}x{height} triplet, got "
                             f"{img.shape[2]}x{img.shape[1]}")
        frames = [img[:, :, width * j:width * (j + 1)] for j in range(3)]
        return np.stack(self._augment(frames, i, seed), 0)

    def _native_load(self, idx, flips, out, threads):
        from ._lib import check, lib
        paths = (C.c_char_p * len(idx))(*[os.path.join(self.dir, self.files[i]).encode() for i in idx])
        w, h = self.resolution
        check(lib().md2_load_triplets_u8(paths, len(idx), w, h, flips.ctypes.data_as(C.c_void_p),
                                         C.c_void_p(_addr(out)), threads), "md2_load_triplets_u8")

    def getobs_u8(self, i: int, seed: int = 0) -> np.ndarray:
        """Sample ``i`` (0-based) as its N0f8 bytes: uint8 [3][3][H][W] (RGB only)."""
        if self.grayscale:
            raise TypeError("grayscale Depth10k samples are Gray{Float32}, not N0f8 bytes")
        img = _load_png_raw(os.path.join(self.dir, self.files[i]))
        if img.dtype != np.uint8:
            raise TypeError(f"{self.files[i]}: not an 8-bit image")
        return self._frames(img, i, seed)

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        """Sample ``i`` (0-based): float32 [3][C][H][W] (dtk.jl:29-46)."""
        img = _load_png(os.path.join(self.dir, self.files[i]))
        if self.grayscale:
            img = _to_gray(img)
        return self._frames(img, i, seed)

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
        self.u8 = True

    def __len__(self):
        return self.total_length

    def _native_load(self, idx, flips, out, threads):
        from ._lib import check, lib
        files = [os.path.join(self.frames_dir, "%06d.png" % (i * len(self.frame_ids) + x - 1)).encode()
                 for i in idx for x in self.frame_ids]
        paths = (C.c_char_p * len(files))(*files)
        w, h = self.resolution
        check(lib().md2_load_kitti_u8(paths, len(idx), h, w, flips.ctypes.data_as(C.c_void_p),
                                      C.c_void_p(_addr(out)), threads), "md2_load_kitti_u8")

    def getobs_u8(self, i: int, seed: int = 0) -> np.ndarray:
        """Sample ``i`` (0-based): frames 3i, 3i+1, 3i+2 (kitty.jl:47-61), each ``imresize``d to
        the target size and kept N0f8 -> uint8 [3][1][H][W]."""
        width, height = self.resolution
        sid = i * len(self.frame_ids)
        frames = []
        for x in self.frame_ids:
            img = _load_png_raw(os.path.join(self.frames_dir, "%06d.png" % (sid + x - 1)))
            if img.dtype != np.uint8 or img.shape[0] != 1:
                raise TypeError("KITTI image_0 frames are 8-bit grayscale")
            frames.append(imresize(img, height, width))
        frames = self._augment(frames, i, seed)
        return np.stack(frames, 0)


class DChain:
    """``DChain(datasets)`` (src/dchain.jl:1-30)."""

    def __init__(self, datasets: Sequence):
        self.datasets = list(datasets)
        self.bins = np.cumsum([len(d) for d in self.datasets]).tolist()
        self.channels = self.datasets[0].channels
        self.resolution = self.datasets[0].resolution
        self.u8 = all(getattr(d, "u8", False) for d in self.datasets)

    def __len__(self):
        return self.bins[-1] if self.bins else 0

    def getobs(self, i: int, seed: int = 0) -> np.ndarray:
        if not 0 <= i < len(self):
            raise IndexError(i)
        bid = next(b for b, edge in enumerate(self.bins) if i < edge)
        return self.datasets[bid].getobs(i - (self.bins[bid - 1] if bid else 0), seed)

    def getobs_u8(self, i: int, seed: int = 0) -> np.ndarray:
        if not 0 <= i < len(self):
            raise IndexError(i)
        bid = next(b for b, edge in enumerate(self.bins) if i < edge)
        return self.datasets[bid].getobs_u8(i - (self.bins[bid - 1] if bid else 0), seed)

    def batch_u8(self, idx, seed: int = 0, threads: int = 8, out=None):
        """Per member dataset one native batch call, scattered back into ``idx`` order."""
        w, h = self.resolution
        if out is None:
            out = np.empty((len(idx), 3, self.channels, h, w), dtype=np.uint8)
        groups = {}
        for k, i in enumerate(idx):
            if not 0 <= i < len(self):
                raise IndexError(i)
            bid = next(b for b, edge in enumerate(self.bins) if i < edge)
            groups.setdefault(bid, []).append((k, i - (self.bins[bid - 1] if bid else 0)))
        for bid, items in groups.items():
            sub = self.datasets[bid].batch_u8([li for _, li in items], seed, threads)
            for (k, _), s in zip(items, sub):
                out[k] = s if isinstance(out, np.ndarray) else _torch_from(s)
        return out

    __getitem__ = getobs


class DataLoader:
    """Batches of ``batch_size`` samples as a tensor ``[N][3][C][H][W]`` on ``device``.

    Epoch order: ``shuffle`` permutes with ``seed + epoch``; the global batch ``batch_size *
    world`` is cut into per-rank shards by global index (md2hip.dist.shard_range), so the union
    over ranks is identical for every GPU count.  Incomplete trailing batches are dropped
    (fixed-shape train step).  ``workers`` decode threads; one batch is prefetched and its
    host->device copy runs on a side stream while the previous batch trains.  ``bytes_h2d``
    (default): N0f8 datasets are copied as uint8 and converted on the GPU.  ``native`` (default):
    N0f8 datasets decode through the library's C++ PNG loader (md2_load_*_u8; GIL-free threads,
    ``prefetch`` batches in flight, ``workers`` threads in all) into pinned memory."""

    def __init__(self, dataset, batch_size: int, *, shuffle: bool = True, seed: int = 0,
                 workers: int = 8, device=None, rank: int = 0, world: int = 1, prefetch: int = 2,
                 bytes_h2d: bool = True, native: bool = True):
        self.ds, self.batch_size, self.shuffle, self.seed = dataset, batch_size, shuffle, seed
        self.workers, self.rank, self.world, self.prefetch = workers, rank, world, prefetch
        self.bytes_h2d, self.native = bytes_h2d, native
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

        use_u8 = on_gpu and self.bytes_h2d and getattr(self.ds, "u8", False)
        native = self.native and getattr(self.ds, "u8", False) and hasattr(self.ds, "batch_u8")
        if use_u8:
            from ._lib import check, lib, ptr
            get = lambda i: self.ds.getobs_u8(i, seed=self.seed + epoch)
        else:
            get = lambda i: self.ds.getobs(i, seed=self.seed + epoch)
        w_, h_ = self.ds.resolution
        shape = (self.batch_size, 3, self.ds.channels, h_, w_)
        jobs = max(1, min(self.prefetch, len(batches)))
        per_call = max(1, self.workers // jobs)

        def native_batch(idx):
            # the library's PNG decoder on per_call host threads, straight into (pinned) memory
            buf = torch.empty(shape, dtype=torch.uint8, pin_memory=on_gpu)
            self.ds.batch_u8(idx, seed=self.seed + epoch, threads=per_call, out=buf)
            return buf if use_u8 else torch.from_numpy(_unorm(buf.numpy()))

        def produce():
            try:
                with ThreadPoolExecutor(jobs if native else self.workers) as pool:
                    pending = []
                    it = iter(batches)
                    if native:               # `jobs` batches in flight, each decoded natively
                        for idx in it:
                            pending.append(pool.submit(native_batch, idx))
                            if len(pending) >= jobs:
                                break
                    while pending or not native:
                        if stop.is_set():
                            return
                        if native:
                            host = pending.pop(0).result()
                            nxt = next(it, None)
                            if nxt is not None:
                                pending.append(pool.submit(native_batch, nxt))
                        else:
                            idx = next(it, None)
                            if idx is None:
                                break
                            host = torch.from_numpy(np.stack(list(pool.map(get, idx)), 0))
                        if on_gpu:
                            if not host.is_pinned():
                                host = host.pin_memory()
                            with torch.cuda.stream(stream):
                                x = host.to(dev, non_blocking=True)
                                if use_u8:          # N0f8 bytes -> Float32 on the GPU
                                    xf = torch.empty(x.shape, dtype=torch.float32, device=dev)
                                    check(lib().md2_unorm8_to_float(ptr(x), ptr(xf), x.numel(),
                                                                    C.c_void_p(stream.cuda_stream)),
                                          "md2_unorm8_to_float")
                                    x = xf
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
