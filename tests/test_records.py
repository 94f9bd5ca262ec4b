"""Image-record stores (research_image_retrieval_amd/records.py), restating
the GLDv2 / distractor LMDB readers of dataset/configdataset.py:264-364 on CPU:
the record layout ((imgbuf,), (label,)) with b'__len__' / b'__keys__', the
restricted record decoder, the partition per rank (the reference's :326 reset
not reproduced), the thumbnail (pinned to the reference's ImageFromList by
tests/golden/loader.npz) and size bucketing for batched extraction."""
import io
import os
import pickle
import sys

import numpy as np
import pytest
from PIL import Image

from research_image_retrieval_amd import records as R
from research_image_retrieval_amd.dataset import imthumbnail

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import inputs as I  # noqa: E402

SIZES = [(97, 130), (240, 180), (64, 64), (333, 211), (150, 401), (240, 180), (333, 211)]


def _jpegs():
    rs = np.random.RandomState(5)
    out = []
    for h, w in SIZES:
        a = rs.randint(0, 256, size=(h, w, 3), dtype=np.uint8)
        b = io.BytesIO()
        Image.fromarray(a).save(b, format="JPEG", quality=90)
        out.append(b.getvalue())
    return out


@pytest.fixture(params=["dict", "file"])
def store(request, tmp_path):
    items = R.build_records(_jpegs(), labels=[10 + i for i in range(len(SIZES))])
    if request.param == "dict":
        return R.DictRecordStore(items)
    return R.FileRecordStore.write(str(tmp_path / "gallery"), items)


def test_gldv2_records_round_trip(store):
    ds = R.GLDV2Records(store)
    assert len(ds) == len(SIZES)
    jp = _jpegs()
    for i in range(len(ds)):
        img, label = ds[i]
        assert label == 10 + i
        ref = Image.open(io.BytesIO(jp[i])).convert("RGB")
        assert np.array_equal(np.asarray(img), np.asarray(ref))
    sub = R.GLDV2Records(store, pool=[4, 1])
    assert len(sub) == 2 and sub[0][1] == 14 and sub[1][1] == 11


def test_record_layout_matches_reference_reader(store):
    """The values are exactly what the reference's read_lmdb unpacks:
    pickle.loads(v)[0][0] = image bytes, [1][0] = label (configdataset.py:291-300)."""
    keys = pickle.loads(store.get(b"__keys__"))
    assert pickle.loads(store.get(b"__len__")) == len(SIZES) == len(keys)
    v = pickle.loads(store.get(keys[2]))
    assert v[0][0] == _jpegs()[2] and v[1][0] == 12


def test_record_decoder_refuses_code():
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    with pytest.raises(pickle.UnpicklingError):
        R.loads_record(pickle.dumps(((Evil(),), (0,))))
    assert R.loads_record(pickle.dumps(((b"x",), (np.int64(3),))))[1][0] == 3


def test_distractor_partition_and_thumbnail(store):
    n = len(SIZES)
    seen = []
    for rank in range(3):
        lo, hi = R.partition_for_rank(n, 3, rank)
        ds = R.DistractorRecords(store, imsize=100, partition=(lo, hi))
        assert len(ds) == hi - lo
        jp = _jpegs()
        for j in range(len(ds)):
            want = np.asarray(imthumbnail(Image.open(io.BytesIO(jp[lo + j])).convert("RGB"), 100))
            got = ds[j].numpy()
            assert np.array_equal(got, want)  # records [lo, hi), not [0, hi - lo) (reference :326)
            assert ds.thumb_size(j) == got.shape[:2]
            seen.append(lo + j)
    assert seen == list(range(n))
    with pytest.raises(ValueError):
        R.DistractorRecords(store, partition=(3, n + 1))


def test_size_buckets_group_equal_sizes(store):
    ds = R.DistractorRecords(store, imsize=150)
    sb = R.SizeBuckets(ds, batch_size=2)
    flat = sorted(i for b in sb for i in b)
    assert flat == list(range(len(SIZES)))
    for b in sb:
        assert len(b) <= 2 and len({ds.thumb_size(i) for i in b}) == 1


def test_lmdb_store_needs_lmdb():
    try:
        import lmdb  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            R.LmdbRecordStore("/nonexistent")
