"""Host-side loader (dataset.py) against the reference's ImageFromList outputs
(tests/golden/loader.npz, made by make_golden.py from dataset/ImageFromList.py
with Image.ANTIALIAS restored as LANCZOS), the gnd reader and the revisitop
config restatement."""
import os
import pickle
import sys

import numpy as np
import pytest

from research_image_retrieval_amd import dataset as D

GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)
import inputs as I  # noqa: E402


@pytest.mark.parametrize("imsize", [None, 100, 57])
@pytest.mark.parametrize("use_bb", [0, 1])
def test_image_from_list_matches_reference(tmp_path, imsize, use_bb):
    fx = np.load(os.path.join(GOLD, "loader.npz"))
    paths = I.write_pngs(I.loader_images(int(fx["seed"])), str(tmp_path))
    ds = D.ImageFromList(paths, imsize=imsize, bbox=I.LOADER_BBOXES if use_bb else None)
    for i in range(len(ds)):
        got = np.asarray(ds[i])
        assert np.array_equal(got, fx[f"im{imsize}_b{use_bb}_{i}"]), (imsize, use_bb, i)
    t = D.ImageFromList(paths, imsize=imsize, transforms=D.ToUint8HWC())[0]
    assert t.dtype.is_floating_point is False and t.shape[-1] == 3


def test_revisited_config_and_loaders(tmp_path):
    I.write_fake_revisited(str(tmp_path))
    cfg = D.RoxfordAndRparis("ROxford5k", str(tmp_path))
    assert cfg["n"] == 5 and cfg["nq"] == 2 and cfg["dataset"] == "roxford5k"
    assert cfg["qim_fname"][1].endswith(os.path.join("roxford5k", "jpg", "im3.jpg"))
    ql, gl = D.revisited_loaders(cfg, imsize=100, num_workers=0)
    qs = [b for b in ql]
    gs = [b for b in gl]
    assert len(qs) == 2 and len(gs) == 5
    assert all(b.shape[0] == 1 and b.shape[-1] == 3 and max(b.shape[1:3]) <= 100 for b in gs)
    # the bbox query keeps its crop's share of imsize
    assert max(qs[0].shape[1:3]) <= 100 * 120 / 130 + 1
    with pytest.raises(ValueError):
        D.RoxfordAndRparis("holidays", str(tmp_path))


def test_gnd_reader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    p = os.path.join(str(tmp_path), "gnd_bad.pkl")
    with open(p, "wb") as f:
        pickle.dump({"imlist": [], "x": Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        D.load_gnd(p)
