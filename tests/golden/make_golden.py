"""Generate tests/golden/*.npz from the REFERENCE's own functions.

Run in the build container only (it imports /root/reference, which does not
exist on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
torchvision is absent here, so a bare sys.modules stub satisfies the
reference modules' top-level `import torchvision` lines; none of the functions
called below touch it.  Only data (seeds, inputs, outputs) is written; no
reference source is copied.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/benchmark"
sys.path.insert(0, HERE)
import inputs as I  # noqa: E402


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tv.models = types.ModuleType("torchvision.models")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tvf = types.ModuleType("torchvision.transforms.functional")
    tv.transforms.functional = tvf
    sys.modules.update({"torchvision": tv, "torchvision.models": tv.models, "torchvision.transforms": tv.transforms,
                        "torchvision.transforms.functional": tvf})
    # lmdb (GLDv2 training reader, dataset/configdataset.py:13) is absent too;
    # the dataset package imports it at top level, nothing below uses it
    sys.modules.setdefault("lmdb", types.ModuleType("lmdb"))


def loader_fixture():
    """(viii) ImageFromList (dataset/ImageFromList.py:30-57): full-size, thumbnail
    and query-bbox crops.  Pillow >= 10 has no Image.ANTIALIAS, on which the
    reference's imthumbnail crashes; it was an alias of
    LANCZOS in the Pillow versions the code was written for, restored here."""
    import tempfile
    from PIL import Image
    if not hasattr(Image, "ANTIALIAS"):
        Image.ANTIALIAS = Image.LANCZOS
    from dataset.ImageFromList import ImageFromList
    imgs = I.loader_images(61)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        paths = I.write_pngs(imgs, d)
        for imsize in (None, 100, 57):
            for use_bb in (0, 1):
                ds = ImageFromList(paths, imsize=imsize, bbox=I.LOADER_BBOXES if use_bb else None)
                for i in range(len(ds)):
                    out[f"im{imsize}_b{use_bb}_{i}"] = np.asarray(ds[i])
    np.savez_compressed(os.path.join(HERE, "loader.npz"), seed=61, **out)


def trunk_fixture():
    """(ix) The reference's own torchvision-free ResNet-101, ResNet_DOLG
    (networks/backbone.py:218-274; ResStemIN :261-274, ResStage :244-259,
    ResBlock :327-346, BottleneckTransform :305-325), eval mode, with seeded
    torchvision-keyed weights (non-trivial BN statistics) remapped to its keys.
    Saves its (x3, x4) outputs: x4 for every case, x3 for the odd-size one."""
    import torch.nn as nn  # noqa: F401
    from networks.backbone import ResNet_DOLG
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from research_image_retrieval_amd.weights import synthetic_resnet_state_dict, to_dolg_keys
    torch.set_num_threads(8)
    net = ResNet_DOLG()
    sd = to_dolg_keys(synthetic_resnet_state_dict("resnet101", I.TRUNK_WEIGHT_SEED))
    net.load_state_dict(sd, strict=True)
    net.eval()
    out = {"weight_seed": I.TRUNK_WEIGHT_SEED}
    with torch.no_grad():
        for tag, (seed, b, h, w) in I.TRUNK_CASES.items():
            x3, x4 = net(I.trunk_input(seed, b, h, w))
            out[tag + "_x4"] = x4.numpy()
            if tag == "b1_odd":
                out[tag + "_x3"] = x3.numpy()
            out[tag + "_case"] = np.array([seed, b, h, w])
    np.savez_compressed(os.path.join(HERE, "resnet_dolg.npz"), **out)


def trunk_fixture_v15():
    """(ix-b) The same ResNet_DOLG with each stage-entry block's stride moved
    from its 1x1 `a` conv to its 3x3 `b` conv (BottleneckTransform's own
    comment, networks/backbone.py:310: "TH/C2 -> stride=2 is on 3x3"), i.e. the
    torchvision v1.5 placement of the reference's `ResNet` (networks/backbone.py
    :60-109, torchvision absent here), composed from the reference's modules.
    Only the two Conv2d modules' stride attributes change."""
    from networks.backbone import ResNet_DOLG, ResBlock
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from research_image_retrieval_amd.weights import synthetic_resnet_state_dict, to_dolg_keys
    torch.set_num_threads(8)
    net = ResNet_DOLG()
    sd = to_dolg_keys(synthetic_resnet_state_dict("resnet101", I.TRUNK_WEIGHT_SEED))
    net.load_state_dict(sd, strict=True)
    moved = 0
    for m in net.modules():
        if isinstance(m, ResBlock) and m.f.a.stride != (1, 1):
            m.f.b.stride, m.f.a.stride = m.f.a.stride, (1, 1)
            moved += 1
    assert moved == 3, moved
    net.eval()
    out = {"weight_seed": I.TRUNK_WEIGHT_SEED}
    with torch.no_grad():
        for tag, (seed, b, h, w) in I.TRUNK_CASES.items():
            x3, x4 = net(I.trunk_input(seed, b, h, w))
            out[tag + "_x4"] = x4.numpy()
            if tag == "b1_odd":
                out[tag + "_x3"] = x3.numpy()
            out[tag + "_case"] = np.array([seed, b, h, w])
    np.savez_compressed(os.path.join(HERE, "resnet_dolg_v15.npz"), **out)


def extract_fixture():
    """(vi) extract_vectors on a tiny networks-style extractor (utils/helpfunc.py:18-48):
    single scale ms=[1], single scale ms=[0.5] (the reference's len(ms) == 1
    branch never rescales by ms[0]), and three scales."""
    from utils.helpfunc import extract_vectors
    tn = I.TinyNetRef(41)
    imgs = I.tiny_images(42)
    v1 = extract_vectors(tn, imgs, ms=[1], device=torch.device("cpu"))
    v05 = extract_vectors(tn, imgs, ms=[0.5], device=torch.device("cpu"))
    v3 = extract_vectors(tn, imgs, ms=[1, 1 / np.sqrt(2), 1 / 2], device=torch.device("cpu"))
    np.savez_compressed(os.path.join(HERE, "extract.npz"), net_seed=41, img_seed=42, v1=v1.numpy(), v3=v3.numpy(),
                        v05=v05.numpy())


def main():
    _stub_torchvision()
    sys.path.insert(0, REF)
    if "--only-loader" in sys.argv:
        loader_fixture()
        return
    if "--only-trunk" in sys.argv:
        trunk_fixture()
        return
    if "--only-extract" in sys.argv:
        extract_fixture()
        return
    if "--only-trunk-v15" in sys.argv:
        trunk_fixture_v15()
        return
    loader_fixture()
    trunk_fixture()
    trunk_fixture_v15()
    from networks.RetrievalNet import gem, GeM
    from networks.backbone import pcawhitenlearn_shrinkage
    from networks.spca import ConvDimReduction
    from networks.model import VisionTransformer
    from models.gem_pooling import GeMPooling, GeMModel
    from utils.evaluate import compute_map, compute_map_and_print
    from utils.helpfunc import extract_vectors
    import torch.nn as nn
    import torch.nn.functional as F
    torch.set_num_threads(8)

    # (i) GeM pooling, both reference variants (networks/RetrievalNet.py:318-325, models/gem_pooling.py:12-23)
    x = torch.from_numpy(I.feature_map(1, 4, 64, 7, 7))
    x2 = torch.from_numpy(I.feature_map(2, 2, 2048, 7, 7))
    np.savez_compressed(os.path.join(HERE, "gem.npz"),
                        x=x.numpy(), gem=gem()(x).numpy(), gempool=GeMPooling()(x).detach().numpy(),
                        gempool_p25=GeMPooling(p=2.5)(x).detach().numpy(),
                        x2_seed=2, gem2=gem()(x2).numpy())

    # (ii) extractor tails with the trunk replaced by identity: the reference's own
    # GeM.forward_test (networks/RetrievalNet.py:337-344) and GeMModel.extract_descriptor
    # (models/gem_pooling.py:86-92); weights from seeded generators.
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from research_image_retrieval_amd.weights import synthetic_linear
    net = GeM.__new__(GeM)
    nn.Module.__init__(net)
    net.backbone = nn.Identity()
    net.pooling = gem()
    net.whiten = nn.Conv2d(2048, 2048, kernel_size=(1, 1), stride=1, padding=0, bias=True)
    ww, wb = synthetic_linear(2048, 2048, 11)
    net.whiten.weight.data = ww.view(2048, 2048, 1, 1).clone()
    net.whiten.bias.data = wb.clone()
    net.outputdim = 2048
    out_gem_net = net.forward_test(x2)
    m = GeMModel.__new__(GeMModel)
    nn.Module.__init__(m)
    m.backbone = nn.Identity()
    m.gem_pool = GeMPooling(p=3.0)
    m.feature_proj = nn.Linear(2048, 512)
    pw, pb = synthetic_linear(512, 2048, 12)
    m.feature_proj.weight.data = pw.clone()
    m.feature_proj.bias.data = pb.clone()
    out_gem_model = m.extract_descriptor(x2)
    np.savez_compressed(os.path.join(HERE, "gem_tail.npz"), x2_seed=2, whiten_seed=11, proj_seed=12,
                        gem_net=out_gem_net.numpy(), gem_model=out_gem_model.numpy())

    # (iii) PCA-whitening learn + apply (networks/backbone.py:42-58, networks/spca.py:205-227)
    rs = np.random.RandomState(3)
    A = rs.standard_normal((64, 64))
    X = rs.standard_normal((2000, 64)) @ A * 0.1 + rs.standard_normal(64)
    mean, PT = pcawhitenlearn_shrinkage(X)
    cdr = ConvDimReduction(64, 32)
    cdr.initialize_pca_whitening(X)
    Y = torch.from_numpy(rs.standard_normal((10, 64)).astype(np.float32))
    y = F.normalize(cdr(Y.view(10, 64, 1, 1)).view(10, 32), dim=-1)
    np.savez_compressed(os.path.join(HERE, "pcaw.npz"), X=X, mean=mean, PT=PT, w=cdr.weight.data.numpy(),
                        b=cdr.bias.data.numpy(), Y=Y.numpy(), y=y.detach().numpy())

    # (iv) ranker: the reference's op sequence of iris_evaluate.py:379-386
    for tag, (seed, nq, n, d) in {"rank_a": (21, 16, 20000, 512), "rank_b": (22, 8, 50000, 2048)}.items():
        q, g = I.rank_inputs(seed, nq, n, d)
        qf = F.normalize(torch.from_numpy(q), p=2, dim=1)
        gf = F.normalize(torch.from_numpy(g), p=2, dim=1)
        sim = torch.mm(qf, gf.t()).cpu().numpy()
        ranks_default = np.argsort(-sim, axis=1)           # reference behaviour (unstable kind)
        ranks_stable = np.argsort(-sim, axis=1, kind="stable")
        k = 100
        np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), seed=seed, nq=nq, n=n, d=d,
                            top_idx_stable=ranks_stable[:, :k], top_idx_default=ranks_default[:, :k],
                            top_scores=np.take_along_axis(sim, ranks_stable[:, :k], 1),
                            kth_gap=np.sort(-sim, axis=1)[:, :k + 1])

    # (v) revisited mAP (utils/evaluate.py), full ranks (li=False) and top-100 lists (li=True)
    gnd, ranks = I.map_inputs(31)
    full = compute_map_and_print("roxford5k", "g", "global", ranks, gnd, kappas=[1, 5, 10])
    lists = [ranks[:100, i] for i in range(ranks.shape[1])]
    trunc = compute_map_and_print("rparis6k", "g", "global", lists, gnd, kappas=[1, 5, 10], li=True)
    g_m = [{"ok": np.concatenate([x["easy"], x["hard"]]), "junk": x["junk"]} for x in gnd]
    mAP, aps, pr, prs = compute_map(ranks, g_m, [1, 5, 10])
    mAP2, aps2 = compute_map(ranks, g_m)
    np.savez_compressed(os.path.join(HERE, "map.npz"), seed=31, full=np.array(full), trunc=np.array(trunc),
                        medium_map=mAP, medium_aps=aps, medium_pr=pr, medium_prs=prs, medium_map_nokeeps=mAP2,
                        medium_aps_nokeeps=aps2)

    extract_fixture()

    # (vii) CLIP ViT (networks/model.py:206-243): tiny config and ViT-B/16, seeded weights
    out = {}
    for tag, cfg in {"tiny": dict(res=32, patch=8, width=128, layers=2, heads=2, out_dim=32, seed=51),
                     "b16": dict(res=224, patch=16, width=768, layers=12, heads=12, out_dim=512, seed=52)}.items():
        vit = VisionTransformer(cfg["res"], cfg["patch"], cfg["width"], cfg["layers"], cfg["heads"], cfg["out_dim"])
        sd = I.vit_state_dict(cfg["seed"], cfg["width"], cfg["layers"], cfg["heads"], cfg["patch"], cfg["res"],
                              cfg["out_dim"])
        vit.load_state_dict(sd)
        vit.eval()
        rsx = np.random.RandomState(cfg["seed"] + 100)
        xin = torch.from_numpy(rsx.standard_normal((2, 3, cfg["res"], cfg["res"])).astype(np.float32))
        with torch.no_grad():
            out[tag] = vit(xin).numpy()
        out[tag + "_cfg"] = np.array([cfg["res"], cfg["patch"], cfg["width"], cfg["layers"], cfg["heads"],
                                      cfg["out_dim"], cfg["seed"]])
    np.savez_compressed(os.path.join(HERE, "vit.npz"), **out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
