"""dataset — host-side image loading for the revisited Oxford/Paris protocol
(SURVEY.md §8f row 1), feeding the GPU extractor.

Restates the reference's loader behaviour:
  * pil_loader / ImageFromList.__getitem__   (dataset/ImageFromList.py:9-12, 40-57)
    RGB decode, optional query bbox crop, `thumbnail` so that the longest side
    is <= imsize (for a cropped query: imsize * max(crop) / max(full image));
  * imthumbnail                               (dataset/ImageFromList.py:20-22)
    with Image.LANCZOS: the reference's Image.ANTIALIAS was LANCZOS's alias and
    no longer exists in Pillow >= 10;
  * RoxfordAndRparis(dataset, dir_main)       (dataset/configdataset.py:27-57)
    the gnd_<dataset>.pkl config with image file lists.

What changes for the GPU path: instead of ToTensor+Normalize on the CPU
(dataset/configdataset.py:417), `ToUint8HWC` hands the decoded pixels over as
uint8 [H,W,3]; the extractor normalises them inside its first kernel
(rr_preprocess_u8).  Images keep their own size, so loaders run at batch 1,
as the reference's extract_vectors requires (utils/helpfunc.py:18-48).
"""
import os
import pickle

import numpy as np
import torch
import torch.utils.data as data
from PIL import Image, ImageFile

ImageFile.LOAD_TRUNCATED_IMAGES = True

DEFAULT_IMSIZE = 1024  # config/__init__.py:8


def pil_loader(path):
    with open(path, "rb") as f:
        img = Image.open(f)
        return img.convert("RGB")


def imthumbnail(img, imsize):
    img.thumbnail((imsize, imsize), Image.LANCZOS)
    return img


class ToUint8HWC:
    """PIL RGB image -> torch.uint8 [H, W, 3] (normalisation happens on the GPU)."""

    def __call__(self, img):
        return torch.from_numpy(np.asarray(img, dtype=np.uint8).copy())


class ImageFromList(data.Dataset):
    """Same constructor and item semantics as dataset/ImageFromList.py:30-57."""

    def __init__(self, Image_paths=None, transforms=None, imsize=None, bbox=None, loader=pil_loader):
        super().__init__()
        self.Image_paths = Image_paths
        self.transforms = transforms
        self.bbox = bbox
        self.imsize = imsize
        self.loader = loader
        self.len = len(Image_paths)

    def __getitem__(self, index):
        img = self.loader(self.Image_paths[index])
        full = max(img.size)
        if self.bbox is not None:
            img = img.crop(self.bbox[index])
        if self.imsize is not None:
            if self.bbox is not None:
                img = imthumbnail(img, self.imsize * max(img.size) / full)
            else:
                img = imthumbnail(img, self.imsize)
        if self.transforms is not None:
            img = self.transforms(img)
        return img

    def __len__(self):
        return self.len


class _GndUnpickler(pickle.Unpickler):
    """The revisitop gnd files hold dicts, lists, strings and numpy arrays;
    nothing else may be constructed while reading them."""

    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar"), ("builtins", "set"), ("builtins", "frozenset"),
                ("collections", "OrderedDict")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"gnd file: refusing to construct {module}.{name}")


def load_gnd(path):
    with open(path, "rb") as f:
        return _GndUnpickler(f).load()


def RoxfordAndRparis(dataset, dir_main):
    """dataset/configdataset.py:27-57: gnd config + image paths."""
    dataset = dataset.lower()
    if dataset not in ("oxford5k", "paris6k", "roxford5k", "rparis6k"):
        raise ValueError("Unknown dataset: {}!".format(dataset))
    gnd_fname = os.path.join(dir_main, dataset, "gnd_{}.pkl".format(dataset))
    cfg = load_gnd(gnd_fname)
    cfg["gnd_fname"] = gnd_fname
    cfg["ext"] = ".jpg"
    cfg["qext"] = ".jpg"
    cfg["dir_data"] = os.path.join(dir_main, dataset)
    cfg["dir_images"] = os.path.join(cfg["dir_data"], "jpg")
    cfg["n"] = len(cfg["imlist"])
    cfg["nq"] = len(cfg["qimlist"])
    cfg["im_fname"] = [os.path.join(cfg["dir_images"], name + ".jpg") for name in cfg["imlist"]]
    cfg["qim_fname"] = [os.path.join(cfg["dir_images"], name + ".jpg") for name in cfg["qimlist"]]
    cfg["dataset"] = dataset
    return cfg


def _first(batch):
    return batch[0].unsqueeze(0)


def revisited_loaders(cfg, imsize=DEFAULT_IMSIZE, num_workers=4):
    """(query loader, gallery loader) for the revisitop protocol: queries are
    cropped to gnd[i]['bbx'] and thumbnailed proportionally, gallery images
    thumbnailed to imsize; uint8 [1,H,W,3] batches for extract_vectors."""
    bbxs = [tuple(cfg["gnd"][i]["bbx"]) for i in range(cfg["nq"])]
    q = ImageFromList(cfg["qim_fname"], transforms=ToUint8HWC(), imsize=imsize, bbox=bbxs)
    g = ImageFromList(cfg["im_fname"], transforms=ToUint8HWC(), imsize=imsize)
    mk = lambda ds: data.DataLoader(ds, batch_size=1, shuffle=False, num_workers=num_workers,  # noqa: E731
                                    collate_fn=_first, pin_memory=False)
    return mk(q), mk(g)
