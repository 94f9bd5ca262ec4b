"""Deterministic inputs for the golden fixtures (numpy RandomState streams are
stable across numpy versions), shared by make_golden.py and the tests so large
inputs are regenerated from seeds instead of being committed."""
import os

import numpy as np
import torch
import torch.nn.functional as F


def normed(rs, n, d):
    x = rs.standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def rank_inputs(seed, nq, n, d):
    """Queries/gallery with planted near-duplicates and exact duplicate rows
    (exact score ties), as SURVEY.md §8c fixture (iv) asks."""
    rs = np.random.RandomState(seed)
    q = normed(rs, nq, d)
    g = normed(rs, n, d)
    for i in range(min(nq, 6)):
        j = rs.randint(n)
        v = q[i] + 0.05 * rs.standard_normal(d).astype(np.float32)
        g[j] = v / np.linalg.norm(v)
        g[(j + 7) % n] = g[j]  # exact tie
    return q, g


def feature_map(seed, b, c, h, w):
    """Non-negative post-ReLU-like backbone output, NCHW float32."""
    rs = np.random.RandomState(seed)
    x = np.maximum(rs.standard_normal((b, c, h, w)), 0).astype(np.float32)
    x[x == 0] = 0.0
    return x


def map_inputs(seed, nq=70, n=4993, nper=(5, 8, 6)):
    """ROxford5k-shaped synthetic ground truth + score-sorted ranks [N,Q]."""
    rs = np.random.RandomState(seed)
    gnd = []
    scores = rs.standard_normal((nq, n)).astype(np.float32)
    for i in range(nq):
        perm = rs.permutation(n)
        e, h, j = perm[: nper[0]], perm[nper[0]: nper[0] + nper[1]], perm[nper[0] + nper[1]: sum(nper)]
        if i % 9 == 3:
            e = e[:0]  # some queries without easy positives (excluded from Easy mAP)
        gnd.append({"easy": e.astype(np.int64), "hard": h.astype(np.int64), "junk": j.astype(np.int64)})
        # lift one easy and one hard positive into the top so truncated lists see them
        if len(e):
            scores[i, e[0]] = 9.0
        scores[i, h[0]] = 8.5
        scores[i, j[0]] = 8.9
    ranks = np.argsort(-scores, axis=1, kind="stable").T.copy()  # [N, Q]
    return gnd, ranks


def tiny_net_weights(seed, cin=3, cmid=32, dout=16):
    rs = np.random.RandomState(seed)
    w = (rs.standard_normal((cmid, cin, 3, 3)) * np.sqrt(2.0 / (cin * 9))).astype(np.float32)
    b = (rs.standard_normal(cmid) * 0.1).astype(np.float32)
    pw = (rs.uniform(-1, 1, (dout, cmid)) / np.sqrt(cmid)).astype(np.float32)
    pb = (rs.uniform(-1, 1, dout) / np.sqrt(cmid)).astype(np.float32)
    return w, b, pw, pb


class TinyNetRef(torch.nn.Module):
    """A small networks-style extractor (conv3x3/2 + ReLU -> gem -> Linear ->
    F.normalize) used to exercise extract_vectors' multi-scale logic."""

    def __init__(self, seed):
        super().__init__()
        w, b, pw, pb = (torch.from_numpy(a) for a in tiny_net_weights(seed))
        self.w, self.b, self.pw, self.pb = w, b, pw, pb
        self.outputdim = pw.shape[0]

    @torch.no_grad()
    def forward_test(self, x):
        x = F.relu(F.conv2d(x, self.w, self.b, 2, 1))
        x = F.avg_pool2d(x.clamp(min=1e-6).pow(3.0), (x.size(-2), x.size(-1))).pow(1.0 / 3.0).flatten(1)
        return F.normalize(F.linear(x, self.pw, self.pb), dim=-1)


def tiny_images(seed):
    rs = np.random.RandomState(seed)
    sizes = [(80, 96), (60, 50), (30, 40), (120, 100)]
    return [torch.from_numpy(rs.standard_normal((1, 3, h, w)).astype(np.float32)) for h, w in sizes]


def vit_state_dict(seed, width, layers, heads, patch, res, out_dim):
    """Seeded weights for networks/model.py:VisionTransformer (CLIP layout)."""
    rs = np.random.RandomState(seed)
    sc = width ** -0.5
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    sd = {"conv1.weight": t(rs.standard_normal((width, 3, patch, patch)) * (1.0 / np.sqrt(3 * patch * patch))),
          "class_embedding": t(rs.standard_normal(width) * sc),
          "positional_embedding": t(rs.standard_normal(((res // patch) ** 2 + 1, width)) * sc),
          "ln_pre.weight": t(1 + 0.1 * rs.standard_normal(width)), "ln_pre.bias": t(0.1 * rs.standard_normal(width))}
    for L in range(layers):
        p = f"transformer.resblocks.{L}."
        sd[p + "attn.in_proj_weight"] = t(rs.standard_normal((3 * width, width)) * sc)
        sd[p + "attn.in_proj_bias"] = t(0.02 * rs.standard_normal(3 * width))
        sd[p + "attn.out_proj.weight"] = t(rs.standard_normal((width, width)) * sc)
        sd[p + "attn.out_proj.bias"] = t(0.02 * rs.standard_normal(width))
        sd[p + "ln_1.weight"] = t(1 + 0.1 * rs.standard_normal(width))
        sd[p + "ln_1.bias"] = t(0.1 * rs.standard_normal(width))
        sd[p + "mlp.c_fc.weight"] = t(rs.standard_normal((4 * width, width)) * sc)
        sd[p + "mlp.c_fc.bias"] = t(0.02 * rs.standard_normal(4 * width))
        sd[p + "mlp.c_proj.weight"] = t(rs.standard_normal((width, 4 * width)) * (0.5 / np.sqrt(4 * width)))
        sd[p + "mlp.c_proj.bias"] = t(0.02 * rs.standard_normal(width))
        sd[p + "ln_2.weight"] = t(1 + 0.1 * rs.standard_normal(width))
        sd[p + "ln_2.bias"] = t(0.1 * rs.standard_normal(width))
    sd["ln_post.weight"] = t(1 + 0.1 * rs.standard_normal(width))
    sd["ln_post.bias"] = t(0.1 * rs.standard_normal(width))
    sd["proj"] = t(rs.standard_normal((width, out_dim)) * sc)
    return sd


# ResNet_DOLG trunk fixture (networks/backbone.py:218-274): weight seed and
# (input seed, batch, H, W) of each case
TRUNK_WEIGHT_SEED = 81
TRUNK_CASES = {"b2_224": (82, 2, 224, 224), "b1_odd": (83, 1, 100, 132)}


def trunk_input(seed, b, h, w):
    """Normalised-pixel-like NCHW fp32 input for the trunk fixture."""
    rs = np.random.RandomState(seed)
    return torch.from_numpy(rs.standard_normal((b, 3, h, w)).astype(np.float32))


def loader_images(seed=61):
    """Deterministic RGB images of assorted sizes and aspect ratios (uint8
    HWC): smooth gradients plus noise, so resampling filters matter."""
    rs = np.random.RandomState(seed)
    out = []
    for h, w in [(97, 130), (240, 180), (64, 64), (333, 211), (150, 401)]:
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
        base = np.stack([(np.sin(xx / (7 + 3 * c)) + np.cos(yy / (5 + 2 * c))) * 60 + 128 for c in range(3)], -1)
        out.append(np.clip(base + rs.randint(-30, 31, size=(h, w, 3)), 0, 255).astype(np.uint8))
    return out


# query boxes (x0, y0, x1, y1) in the revisitop gnd['bbx'] convention (floats)
LOADER_BBOXES = [(10.5, 7.25, 120.0, 90.0), (0.0, 0.0, 180.0, 240.0), (3.0, 5.0, 40.0, 61.0),
                 (50.2, 20.7, 200.9, 300.1), (100.0, 10.0, 390.5, 149.0)]


def write_pngs(imgs, directory):
    from PIL import Image
    paths = []
    for i, a in enumerate(imgs):
        p = os.path.join(directory, f"img{i}.png")
        Image.fromarray(a).save(p)
        paths.append(p)
    return paths


def write_fake_revisited(root, name="roxford5k"):
    """A 5-image revisitop-layout dataset (jpg/ + gnd_<name>.pkl) with two
    bbox queries, for the loader / full-resolution extraction tests."""
    import pickle
    from PIL import Image
    d = os.path.join(root, name, "jpg")
    os.makedirs(d)
    for i, a in enumerate(loader_images(61)):
        Image.fromarray(a).save(os.path.join(d, f"im{i}.jpg"), quality=95)
    e = np.array([], dtype=np.int64)
    gnd = [{"bbx": np.array(LOADER_BBOXES[0]), "easy": np.array([1, 3]), "hard": np.array([4]), "junk": e},
           {"bbx": np.array(LOADER_BBOXES[3]), "easy": np.array([0]), "hard": e, "junk": np.array([2])}]
    cfg = {"imlist": [f"im{i}" for i in range(5)], "qimlist": ["im0", "im3"], "gnd": gnd}
    with open(os.path.join(root, name, f"gnd_{name}.pkl"), "wb") as f:
        pickle.dump(cfg, f)
    return cfg


# ROxford5k-like full-resolution images (width, height) before the loader's
# thumbnail(1024): landscape / portrait 4:3, larger photos that get
# thumbnailed, a 3:2 photo, and a small one that stays as it is
FULLRES_SIZES = [(1024, 768), (768, 1024), (1280, 960), (1600, 1066), (700, 525), (2048, 1365)]
FULLRES_BBOXES = [(120.5, 80.25, 900.0, 700.0), (300.0, 10.0, 1500.0, 1000.0)]


def write_fake_revisited_fullres(root, name="roxford5k"):
    """A revisitop-layout dataset at full resolution (config C2: imsize 1024):
    six gallery images of the sizes above, two bbox queries (images 0 and 3)."""
    import pickle
    from PIL import Image
    d = os.path.join(root, name, "jpg")
    os.makedirs(d)
    rs = np.random.RandomState(71)
    for i, (w, h) in enumerate(FULLRES_SIZES):
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
        base = np.stack([(np.sin(xx / (17 + 5 * c)) + np.cos(yy / (11 + 3 * c))) * 60 + 128 for c in range(3)], -1)
        img = np.clip(base + rs.randint(-40, 41, size=(h, w, 3)), 0, 255).astype(np.uint8)
        Image.fromarray(img).save(os.path.join(d, f"im{i}.jpg"), quality=92)
    e = np.array([], dtype=np.int64)
    gnd = [{"bbx": np.array(FULLRES_BBOXES[0]), "easy": np.array([1, 4]), "hard": np.array([2]), "junk": e},
           {"bbx": np.array(FULLRES_BBOXES[1]), "easy": np.array([5]), "hard": e, "junk": np.array([0])}]
    cfg = {"imlist": [f"im{i}" for i in range(len(FULLRES_SIZES))], "qimlist": ["im0", "im3"], "gnd": gnd}
    with open(os.path.join(root, name, f"gnd_{name}.pkl"), "wb") as f:
        pickle.dump(cfg, f)
    return cfg
