"""GPU parity of librr's ResNet trunk against the REFERENCE's own R101.

tests/golden/resnet_dolg.npz holds the (x3, x4) outputs of ResNet_DOLG
(networks/backbone.py:218-274; ResBlock/BottleneckTransform :305-346), the
reference's torchvision-free ResNet-101, run by make_golden.py with seeded
weights.  librr's trunk is built from the same weights in ResNet_DOLG key
layout with the stride on the 1x1 (stride_on="1x1") and checked on both conv
cores."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import embed_ref
from research_image_retrieval_amd import weights as W
from research_image_retrieval_amd.networks import ResNet

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
sys.path.insert(0, GOLD)
import inputs as I  # noqa: E402

# fp32-accurate trunk (exact-fp32 MFMA core, or the f16x2 split "h2") vs the CPU
# reference through 33 bottlenecks; fixture values are O(0.1-1), measured
# errors 1.2-5.4e-7 (round 2)
TRUNK_TOL = 2e-6


@pytest.fixture(scope="module")
def fixture():
    return np.load(os.path.join(GOLD, "resnet_dolg.npz"))


@pytest.mark.parametrize("conv_math", ["h2", "f32"])
@pytest.mark.parametrize("tag", ["b2_224", "b1_odd"])
def test_trunk_vs_reference_resnet_dolg(cuda, fixture, conv_math, tag):
    sd = W.to_dolg_keys(W.synthetic_resnet_state_dict("resnet101", int(fixture["weight_seed"])))
    net = ResNet("resnet101", state_dict=sd, device=cuda, conv_math=conv_math, stride_on="1x1")
    seed, b, h, w = (int(v) for v in fixture[tag + "_case"])
    x = I.trunk_input(seed, b, h, w).permute(0, 2, 3, 1).contiguous().to(cuda)
    x3, x4 = net.forward(x, return_x3=True)
    x4 = x4.permute(0, 3, 1, 2).cpu().numpy()
    err4 = np.abs(x4 - fixture[tag + "_x4"]).max()
    print(tag, conv_math, "max|x4 err|", err4, "max|x4|", np.abs(fixture[tag + "_x4"]).max())
    assert err4 < TRUNK_TOL
    if tag + "_x3" in fixture:
        x3 = x3.permute(0, 3, 1, 2).cpu().numpy()
        err3 = np.abs(x3 - fixture[tag + "_x3"]).max()
        print(tag, conv_math, "max|x3 err|", err3)
        assert err3 < TRUNK_TOL


@pytest.mark.parametrize("conv_math", ["h2", "f32"])
@pytest.mark.parametrize("tag", ["b2_224", "b1_odd"])
def test_trunk_v15_vs_reference_modules(cuda, conv_math, tag):
    """The default torchvision-v1.5 placement (stride on the 3x3) against
    tests/golden/resnet_dolg_v15.npz: the reference's ResNet_DOLG modules with
    each stage-entry stride moved from the 1x1 `a` conv to the 3x3 `b` conv
    (make_golden.py trunk_fixture_v15; torchvision itself is absent)."""
    fx = np.load(os.path.join(GOLD, "resnet_dolg_v15.npz"))
    sd = W.to_dolg_keys(W.synthetic_resnet_state_dict("resnet101", int(fx["weight_seed"])))
    net = ResNet("resnet101", state_dict=sd, device=cuda, conv_math=conv_math, stride_on="3x3")
    seed, b, h, w = (int(v) for v in fx[tag + "_case"])
    x = I.trunk_input(seed, b, h, w).permute(0, 2, 3, 1).contiguous().to(cuda)
    x3, x4 = net.forward(x, return_x3=True)
    err4 = np.abs(x4.permute(0, 3, 1, 2).cpu().numpy() - fx[tag + "_x4"]).max()
    print(tag, conv_math, "v1.5 max|x4 err|", err4)
    assert err4 < TRUNK_TOL
    if tag + "_x3" in fx:
        err3 = np.abs(x3.permute(0, 3, 1, 2).cpu().numpy() - fx[tag + "_x3"]).max()
        assert err3 < TRUNK_TOL


def test_trunk_v15_vs_oracle(cuda):
    """The default torchvision-v1.5 placement against the oracle, which the
    fixture above pins (it differs only in which conv carries the stride)."""
    sd = W.synthetic_resnet_state_dict("resnet101", 7)
    net = ResNet("resnet101", state_dict=sd, device=cuda)
    x = I.trunk_input(5, 2, 96, 80)
    got = net.forward(x.permute(0, 2, 3, 1).contiguous().to(cuda)).permute(0, 3, 1, 2).cpu()
    with torch.no_grad():
        ref = embed_ref.resnet_trunk(x, sd, W.RESNET_LAYERS["resnet101"])
    err = (got - ref).abs().max().item()
    print("v1.5 max|err|", err, "max|ref|", ref.abs().max().item())
    assert err < TRUNK_TOL
