"""records — batched image-record decode for gallery extraction (SURVEY.md
§8f row 4): the GLDv2 / distractor record stores of dataset/configdataset.py:
264-364, restated for the GPU extractor.

The reference keeps images in an LMDB whose values are pickled records
``((imgbuf,), (label,))`` (read back with ``loads_data`` = ``pickle.loads``,
:359-364; the image bytes at ``unpacked[0][0]``, the label at
``unpacked[1][0]``, :291-300 / :343-350), plus two special keys: ``b'__len__'``
(the record count) and ``b'__keys__'`` (the record keys in order, :271-273 /
:314-316).  ``GLDV2Dataset_lmdb`` yields ``(img, label)`` over an optional
index ``pool``; ``Distractor_lmdb`` yields images, thumbnailed to ``imsize``
(:332-333), over an optional per-rank ``partition`` range.

Here:
  * the key -> bytes store is pluggable (``RecordStore``): an in-memory dict,
    a file-backed store this module writes (one data file + an offset index,
    read with positional reads), or LMDB when the ``lmdb`` package is present
    (it is not in this image);
  * records are decoded with a restricted unpickler: it builds the tuples,
    bytes, ints and strings a record holds and refuses to construct anything
    else (the reference's ``pickle.loads`` would run any callable a record
    names);
  * ``Distractor_lmdb``'s partition is honoured.  The reference resets
    ``self.pool = list(range(self.length))`` right after applying it (:326),
    so every rank reads records [0, hi - lo) instead of [lo, hi) and the
    ``split`` selection is dropped too; that defect is documented, not
    reproduced;
  * ``SizeBuckets`` batches records by their post-thumbnail size (read from
    the image header, no decode) so the GPU extractor runs same-size batches
    instead of the reference's batch 1, and ``extract_records`` returns the
    descriptors in record order.
"""
import io
import os
import pickle
import struct

import numpy as np
import torch
import torch.utils.data as data
from PIL import Image

from .dataset import ToUint8HWC, imthumbnail


# ---- record codec ----------------------------------------------------------

class _RecordUnpickler(pickle.Unpickler):
    """Records hold tuples/lists of bytes, ints and strings (and numpy integer
    labels); the special keys hold an int and a list of bytes."""

    _ALLOWED = {("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"), ("numpy", "dtype")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"record: refusing to construct {module}.{name}")


def loads_record(buf):
    """The reference's loads_data (configdataset.py:359-364) without code execution."""
    if buf is None:
        raise KeyError("record not found")
    return _RecordUnpickler(io.BytesIO(bytes(buf))).load()


def dumps_record(imgbuf, label):
    """The record layout the reference reads: ((imgbuf,), (label,))."""
    return pickle.dumps(((bytes(imgbuf),), (int(label),)), protocol=4)


# ---- stores ----------------------------------------------------------------

class RecordStore:
    """key (bytes) -> value (bytes) or None."""

    def get(self, key):
        raise NotImplementedError

    def close(self):
        pass


class DictRecordStore(RecordStore):
    def __init__(self, mapping=None):
        self.map = dict(mapping or {})

    def put(self, key, value):
        self.map[bytes(key)] = bytes(value)

    def get(self, key):
        return self.map.get(bytes(key))


class FileRecordStore(RecordStore):
    """A read-only key/value file pair: ``<path>.dat`` (values back to back)
    and ``<path>.idx`` (for every entry: key length u32, key, offset u64,
    length u64).  Values are read with positional reads, so worker processes
    can share one store without seeking each other."""

    MAGIC = b"RRREC1\n"

    def __init__(self, path):
        self.path = path
        self.index = {}
        with open(path + ".idx", "rb") as f:
            if f.read(len(self.MAGIC)) != self.MAGIC:
                raise ValueError(f"{path}.idx: not a record index")
            while True:
                head = f.read(4)
                if not head:
                    break
                (kl,) = struct.unpack("<I", head)
                key = f.read(kl)
                off, ln = struct.unpack("<QQ", f.read(16))
                self.index[key] = (off, ln)
        self._fd = None

    def _fdesc(self):
        if self._fd is None:
            self._fd = os.open(self.path + ".dat", os.O_RDONLY)
        return self._fd

    def get(self, key):
        ent = self.index.get(bytes(key))
        if ent is None:
            return None
        return os.pread(self._fdesc(), ent[1], ent[0])

    def close(self):
        if self._fd is not None:
            os.close(self._fd)
            self._fd = None

    def __getstate__(self):  # DataLoader workers reopen the data file
        st = dict(self.__dict__)
        st["_fd"] = None
        return st

    @classmethod
    def write(cls, path, items):
        """items: iterable of (key bytes, value bytes)."""
        with open(path + ".dat", "wb") as fd, open(path + ".idx", "wb") as fi:
            fi.write(cls.MAGIC)
            off = 0
            for k, v in items:
                k, v = bytes(k), bytes(v)
                fd.write(v)
                fi.write(struct.pack("<I", len(k)) + k + struct.pack("<QQ", off, len(v)))
                off += len(v)
        return cls(path)


class LmdbRecordStore(RecordStore):
    """The reference's own store (lmdb.open(db_path, readonly=True, lock=False,
    readahead=False, meminit=False), configdataset.py:268/311).  Needs the
    ``lmdb`` package, which this image does not have."""

    def __init__(self, db_path):
        try:
            import lmdb
        except ImportError as e:
            raise ImportError("LmdbRecordStore needs the `lmdb` package; FileRecordStore / DictRecordStore hold "
                              "the same records") from e
        self.env = lmdb.open(db_path, subdir=os.path.isdir(db_path), readonly=True, lock=False, readahead=False,
                             meminit=False)

    def get(self, key):
        with self.env.begin(write=False) as txn:
            v = txn.get(bytes(key))
        return None if v is None else bytes(v)


def build_records(images, labels=None, keys=None):
    """(key, value) pairs of a store in the reference layout: one record per
    image (encoded bytes, e.g. JPEG) plus b'__len__' and b'__keys__'."""
    n = len(images)
    labels = list(range(n)) if labels is None else list(labels)
    keys = [f"{i:08d}".encode() for i in range(n)] if keys is None else [bytes(k) for k in keys]
    items = [(k, dumps_record(img, lab)) for k, img, lab in zip(keys, images, labels)]
    items.append((b"__len__", pickle.dumps(n, protocol=4)))
    items.append((b"__keys__", pickle.dumps(keys, protocol=4)))
    return items


def partition_for_rank(n, world, rank):
    """Contiguous [lo, hi) share of n records for one rank (first n % world get one more)."""
    base, extra = divmod(int(n), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


# ---- datasets ----------------------------------------------------------------

def _decode(imgbuf):
    return Image.open(io.BytesIO(imgbuf)).convert("RGB")


class GLDV2Records(data.Dataset):
    """GLDV2Dataset_lmdb (configdataset.py:264-305): (img, label) over ``pool``."""

    def __init__(self, store, transforms=None, pool=None):
        super().__init__()
        self.store = store
        self.transforms = transforms
        self.length = loads_record(store.get(b"__len__"))
        self.keys = loads_record(store.get(b"__keys__"))
        self.pool = list(range(self.length)) if pool is None else list(pool)
        self.length = len(self.pool)

    def read(self, index):
        rec = loads_record(self.store.get(self.keys[self.pool[index]]))
        return _decode(rec[0][0]), rec[1][0]

    def __getitem__(self, index):
        img, label = self.read(index)
        if self.transforms is not None:
            img = self.transforms(img)
        return img, label

    def __len__(self):
        return self.length


class DistractorRecords(data.Dataset):
    """Distractor_lmdb (configdataset.py:307-357): thumbnailed images over a
    per-rank ``partition`` = (lo, hi) of the record order (honoured; see the
    module docstring for the reference's :326 reset).  Items are uint8
    [H, W, 3] (ToUint8HWC) unless other ``transforms`` are given."""

    def __init__(self, store, transforms=None, imsize=None, partition=None):
        super().__init__()
        self.store = store
        self.transforms = ToUint8HWC() if transforms is None else transforms
        self.imsize = imsize
        n = loads_record(store.get(b"__len__"))
        self.keys = loads_record(store.get(b"__keys__"))
        lo, hi = (0, n) if partition is None else (int(partition[0]), int(partition[1]))
        if not 0 <= lo <= hi <= n:
            raise ValueError(f"partition {partition} outside [0, {n}]")
        self.pool = list(range(lo, hi))
        self.length = len(self.pool)

    def imgbuf(self, index):
        return loads_record(self.store.get(self.keys[self.pool[index]]))[0][0]

    def thumb_size(self, index):
        """(H, W) after thumbnail(imsize), from the image header alone."""
        w, h = Image.open(io.BytesIO(self.imgbuf(index))).size
        if self.imsize is not None and max(w, h) > self.imsize:
            # PIL's thumbnail keeps the aspect ratio, rounding the short side
            # (Image.thumbnail's preserve_aspect_ratio)
            img = Image.new("L", (w, h))
            img.thumbnail((self.imsize, self.imsize))
            w, h = img.size
        return h, w

    def __getitem__(self, index):
        img = _decode(self.imgbuf(index))
        if self.imsize is not None:
            img = imthumbnail(img, self.imsize)
        return self.transforms(img)

    def __len__(self):
        return self.length


class SizeBuckets(data.Sampler):
    """Batches of dataset indices whose images share one post-thumbnail size
    (at most ``batch_size`` each), so the GPU extractor runs real batches."""

    def __init__(self, dataset, batch_size):
        self.batches = []
        by_size = {}
        for i in range(len(dataset)):
            by_size.setdefault(dataset.thumb_size(i), []).append(i)
        for _, idx in sorted(by_size.items()):
            for b0 in range(0, len(idx), batch_size):
                self.batches.append(idx[b0:b0 + batch_size])

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


def _stack_u8(items):
    return torch.stack(items, 0)


@torch.no_grad()
def extract_records(net, dataset, batch_size=32, device=torch.device("cuda"), num_workers=0, ms=(1,)):
    """Descriptors of every record of ``dataset`` (a DistractorRecords) in
    record order: same-size batches through extract.extract_vectors."""
    from .extract import extract_vectors
    sampler = SizeBuckets(dataset, batch_size)
    loader = data.DataLoader(dataset, batch_sampler=sampler, num_workers=num_workers, collate_fn=_stack_u8)
    vecs = extract_vectors(net, loader, ms=ms, device=device, print_freq=0)
    order = np.concatenate([np.asarray(b, dtype=np.int64) for b in sampler.batches]) if sampler.batches else \
        np.zeros(0, np.int64)
    out = torch.empty_like(vecs)
    out[torch.from_numpy(order)] = vecs
    return out
