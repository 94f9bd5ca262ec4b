"""Host-side logic that needs no GPU: BN folding, key remapping, shard bounds,
weight generation determinism."""
import torch
import torch.nn.functional as F

from research_image_retrieval_amd import weights as W
from research_image_retrieval_amd.distributed import shard_bounds


def test_fold_bn_matches_conv_then_bn():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(16, 8, 3, 3, generator=g)
    bn = {"weight": torch.rand(16, generator=g) + 0.5, "bias": torch.randn(16, generator=g),
          "running_mean": torch.randn(16, generator=g), "running_var": torch.rand(16, generator=g) + 0.5}
    x = torch.randn(2, 8, 9, 9, generator=g)
    ref = F.batch_norm(F.conv2d(x, w, None, 1, 1), bn["running_mean"], bn["running_var"], bn["weight"], bn["bias"],
                       False, 0.0, W.BN_EPS)
    wf, bf = W.fold_bn(w, bn)
    out = F.conv2d(x, wf.permute(0, 3, 1, 2), bf, 1, 1)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


def test_resnet_specs_counts():
    assert len(W.resnet_conv_specs("resnet50")) == 1 + 3 * 16 + 4
    assert len(W.resnet_conv_specs("resnet101")) == 1 + 3 * 33 + 4


def test_synthetic_weights_deterministic():
    a = W.synthetic_resnet_state_dict("resnet50", 7)
    b = W.synthetic_resnet_state_dict("resnet50", 7)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert a["layer4.2.conv3.weight"].shape == (2048, 512, 1, 1)


def test_reference_key_layouts_map_to_torchvision():
    sd = W.synthetic_resnet_state_dict("resnet50", 1)
    # networks.ResNet layout (networks/backbone.py:93-101) saved under globalmodel.
    net = {}
    for k, v in sd.items():
        k2 = k.replace("conv1.", "block1.0.", 1) if k.startswith("conv1.") else k
        k2 = k2.replace("bn1.", "block1.1.", 1) if k.startswith("bn1.") else k2
        for i in range(4):
            if k2.startswith(f"layer{i + 1}."):
                k2 = f"block{i + 2}." + k2[len(f"layer{i + 1}."):]
        net["globalmodel.backbone." + k2] = v
    # Table-1 GeMModel layout (models/gem_pooling.py:44)
    seq = {}
    for k, v in sd.items():
        k2 = k.replace("conv1.", "0.", 1) if k.startswith("conv1.") else k
        k2 = k2.replace("bn1.", "1.", 1) if k.startswith("bn1.") else k2
        for i in range(4):
            if k2.startswith(f"layer{i + 1}."):
                k2 = f"{i + 4}." + k2[len(f"layer{i + 1}."):]
        seq["backbone.backbone." + k2] = v
    seq["backbone.feature_proj.weight"] = torch.zeros(1)
    for remapped in (W.to_torchvision_keys(net), W.to_torchvision_keys(seq)):
        assert set(remapped) == set(sd)
        assert all(torch.equal(remapped[k], sd[k]) for k in sd)


def test_shard_bounds_partition():
    for n in (0, 1, 7, 1_600_000, 1_600_003):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
