"""store — on-disk descriptor store for large galleries.

The reference keeps GLDv2 images in an lmdb of pickled (imgbuf, label)
records (dataset/configdataset.py:264-364) and holds gallery descriptors only
in memory (iris_evaluate.py:378-386: one [N,D] tensor).  At 1.6M x 2048 that
tensor is 13.1 GB, so the build stores descriptors once and streams each
rank's row range straight into HBM:

  <dir>/store.json          {"format": "rr-descriptor-store", "version": 1,
                             "n", "d", "dtype": "float32",
                             "shards": [{"file", "lo", "rows", "xxh64"}],
                             "labels": "labels.i64" | null}
  <dir>/shard-00000.f32     raw little-endian rows [rows, d] (no header:
                            np.memmap-able, page-aligned at offset 0)
  <dir>/labels.i64          optional int64 per row (landmark ids)

Files are row-major and contiguous, so a rank's range [lo, hi) is one or two
sequential reads; `to_device` streams it through two pinned host buffers on
a side stream (disk -> pinned copy overlaps the previous chunk's H2D DMA).
lmdb itself is not importable in this image; the image-side
reader stays with the caller's DataLoader (dataset.py).
"""
import json
import os

import numpy as np
import torch

FORMAT = "rr-descriptor-store"
VERSION = 1


def _xxh64_file(path, block=1 << 24):
    import xxhash
    h = xxhash.xxh64()
    with open(path, "rb") as f:
        while True:
            b = f.read(block)
            if not b:
                break
            h.update(b)
    return h.hexdigest()


class DescriptorStoreWriter:
    """Append fp32 descriptor rows; shards roll over every `shard_rows` rows."""

    def __init__(self, path, d, shard_rows=262144, with_labels=False):
        if d <= 0 or shard_rows <= 0:
            raise ValueError("d and shard_rows must be positive")
        os.makedirs(path, exist_ok=True)
        if os.path.exists(os.path.join(path, "store.json")):
            raise FileExistsError(f"{path} already holds a descriptor store")
        self.path, self.d, self.shard_rows = path, int(d), int(shard_rows)
        self.shards = []
        self.n = 0
        self._f = None
        self._rows_in = 0
        self._labels = open(os.path.join(path, "labels.i64"), "wb") if with_labels else None

    def _roll(self):
        if self._f is not None:
            self._f.close()
        name = f"shard-{len(self.shards):05d}.f32"
        self.shards.append({"file": name, "lo": self.n, "rows": 0})
        self._f = open(os.path.join(self.path, name), "wb")
        self._rows_in = 0

    def append(self, vecs, labels=None):
        if isinstance(vecs, torch.Tensor):
            vecs = vecs.detach().cpu().numpy()
        vecs = np.ascontiguousarray(vecs, dtype="<f4")
        if vecs.ndim != 2 or vecs.shape[1] != self.d:
            raise ValueError(f"expected [rows, {self.d}] descriptors, got {vecs.shape}")
        if (labels is None) != (self._labels is None):
            raise ValueError("labels must be given iff the store was opened with_labels")
        if labels is not None:
            labels = np.ascontiguousarray(labels, dtype="<i8").reshape(-1)
            if labels.shape[0] != vecs.shape[0]:
                raise ValueError("one label per row")
            self._labels.write(labels.tobytes())
        i = 0
        while i < vecs.shape[0]:
            if self._f is None or self._rows_in == self.shard_rows:
                self._roll()
            take = min(self.shard_rows - self._rows_in, vecs.shape[0] - i)
            self._f.write(vecs[i:i + take].tobytes())
            self._rows_in += take
            self.shards[-1]["rows"] += take
            self.n += take
            i += take

    def close(self, checksum=True):
        if self._f is not None:
            self._f.close()
            self._f = None
        if self._labels is not None:
            self._labels.close()
        for s in self.shards:
            s["xxh64"] = _xxh64_file(os.path.join(self.path, s["file"])) if checksum else None
        meta = {"format": FORMAT, "version": VERSION, "n": self.n, "d": self.d, "dtype": "float32",
                "shards": self.shards, "labels": "labels.i64" if self._labels is not None else None}
        tmp = os.path.join(self.path, "store.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(tmp, os.path.join(self.path, "store.json"))
        return DescriptorStore(self.path)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        if exc[0] is None:
            self.close()
        elif self._f is not None:
            self._f.close()


def write_store(path, vecs, shard_rows=262144, labels=None):
    w = DescriptorStoreWriter(path, np.shape(vecs)[1], shard_rows, with_labels=labels is not None)
    w.append(vecs, labels)
    return w.close()


class DescriptorStore:
    def __init__(self, path):
        with open(os.path.join(path, "store.json")) as f:
            meta = json.load(f)
        if meta.get("format") != FORMAT or meta.get("version") != VERSION:
            raise ValueError(f"{path}: not an {FORMAT} v{VERSION}")
        if meta.get("dtype") != "float32":
            raise ValueError(f"{path}: unsupported dtype {meta.get('dtype')}")
        self.path, self.meta = path, meta
        self.n, self.d = int(meta["n"]), int(meta["d"])
        self.shards = meta["shards"]
        lo = 0
        for s in self.shards:
            if s["lo"] != lo:
                raise ValueError(f"{path}: shard {s['file']} starts at {s['lo']}, expected {lo}")
            size = os.path.getsize(os.path.join(path, s["file"]))
            if size != s["rows"] * self.d * 4:
                raise ValueError(f"{path}: {s['file']} has {size} bytes, expected {s['rows'] * self.d * 4}")
            lo += s["rows"]
        if lo != self.n:
            raise ValueError(f"{path}: shards hold {lo} rows, header says {self.n}")
        self._maps = {}

    def _map(self, s):
        m = self._maps.get(s["file"])
        if m is None:
            m = np.memmap(os.path.join(self.path, s["file"]), dtype="<f4", mode="r", shape=(s["rows"], self.d))
            self._maps[s["file"]] = m
        return m

    def verify(self):
        """Recompute every shard's xxh64 against the header."""
        for s in self.shards:
            if s.get("xxh64") and _xxh64_file(os.path.join(self.path, s["file"])) != s["xxh64"]:
                raise ValueError(f"{self.path}: checksum mismatch in {s['file']}")
        return True

    def _pieces(self, lo, hi):
        """(shard, row0, row1) pieces covering global rows [lo, hi)."""
        if not (0 <= lo <= hi <= self.n):
            raise IndexError(f"rows [{lo}, {hi}) outside [0, {self.n})")
        for s in self.shards:
            a, b = max(lo, s["lo"]), min(hi, s["lo"] + s["rows"])
            if a < b:
                yield s, a - s["lo"], b - s["lo"]

    def rows(self, lo, hi):
        """Host copy of rows [lo, hi) as float32 [hi-lo, d]."""
        out = np.empty((hi - lo, self.d), np.float32)
        o = 0
        for s, a, b in self._pieces(lo, hi):
            out[o:o + b - a] = self._map(s)[a:b]
            o += b - a
        return out

    def labels(self, lo=0, hi=None):
        if self.meta.get("labels") is None:
            return None
        hi = self.n if hi is None else hi
        m = np.memmap(os.path.join(self.path, self.meta["labels"]), dtype="<i8", mode="r", shape=(self.n,))
        return np.array(m[lo:hi])

    def to_device(self, lo, hi, device, chunk_rows=65536):
        """Rows [lo, hi) into a new device tensor, streamed in chunks through
        two pinned buffers; the H2D copies run on a side stream and the call
        returns after they are complete on the current stream."""
        device = torch.device(device)
        out = torch.empty((hi - lo, self.d), dtype=torch.float32, device=device)
        if hi == lo:
            return out
        if device.type != "cuda":
            out.copy_(torch.from_numpy(self.rows(lo, hi)))
            return out
        chunk = max(1, min(chunk_rows, hi - lo))
        bufs = [torch.empty((chunk, self.d), dtype=torch.float32).pin_memory() for _ in range(2)]
        done = [None, None]
        side = torch.cuda.Stream(device=device)
        cur = torch.cuda.current_stream(device)
        side.wait_stream(cur)  # `out` was allocated on the current stream
        r, k = lo, 0
        while r < hi:
            e = min(hi, r + chunk)
            b = k & 1
            if done[b] is not None:
                done[b].synchronize()  # the DMA that last read this buffer is over
            bufs[b][: e - r].numpy()[:] = self.rows(r, e)
            with torch.cuda.stream(side):
                out[r - lo:e - lo].copy_(bufs[b][: e - r], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
            done[b] = ev
            r, k = e, k + 1
        cur.wait_stream(side)
        out.record_stream(side)
        for ev in done:
            if ev is not None:
                ev.synchronize()
        return out


def load_gallery_shard(store, rank, world, device, chunk_rows=65536):
    """This rank's contiguous row range (distributed.shard_bounds) in HBM:
    -> (tensor [hi-lo, d], lo)."""
    from .distributed import shard_bounds
    if isinstance(store, str):
        store = DescriptorStore(store)
    lo, hi = shard_bounds(store.n, world, rank)
    return store.to_device(lo, hi, device, chunk_rows), lo
