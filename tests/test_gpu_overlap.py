"""The trunk's batch split across HIP streams (networks._Extractor.
forward_test_u8_streams): the overlapped schedule computes exactly what the
same parts compute one after another, and stays within the f16x2 core's
descriptor bar of the whole batch in one part (tests/test_gpu_h2.py)."""
import numpy as np
import pytest
import torch

from research_image_retrieval_amd.networks import GeM, GeMPCAw, ConvDimReduction
from research_image_retrieval_amd import weights as W

pytestmark = pytest.mark.gpu


def _net(dev, arch="resnet50"):
    net = GeM(2048, backbone=arch, seed=3, device=dev)
    pw = ConvDimReduction(2048, 2048, device=dev)
    w, b = W.synthetic_linear(2048, 2048, 8, scale=1.0 / np.sqrt(2048))
    pw.set_params(w, b)
    return GeMPCAw(net, pw)


@pytest.mark.parametrize("parts,lag,batch", [(2, 1, 24), (2, 0, 7), (3, 4, 30), (2, 99, 16)])
def test_streams_bit_identical_to_serial_parts(parts, lag, batch):
    dev = torch.device("cuda:0")
    net = _net(dev)
    rs = np.random.RandomState(parts * 100 + batch)
    imgs = torch.from_numpy(rs.randint(0, 256, size=(batch, 160, 160, 3), dtype=np.uint8)).to(dev)
    cuts = [batch * i // parts for i in range(parts + 1)]
    ref = torch.cat([net.forward_test_u8(imgs[cuts[i]:cuts[i + 1]]) for i in range(parts)])
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    for _ in range(2):  # a second pass reuses the streams' cached blocks
        out = net.forward_test_u8_streams(imgs, streams, lag=lag)
        assert out.shape == (batch, 2048)
        assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    whole = net.forward_test_u8(imgs)
    assert (out - whole).abs().max().item() <= 1e-6


def test_streams_empty_part():
    """More streams than images: an empty part is a no-op, not an error."""
    dev = torch.device("cuda:0")
    net = _net(dev)
    imgs = torch.randint(0, 256, (1, 128, 128, 3), dtype=torch.uint8, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    out = net.forward_test_u8_streams(imgs, streams, lag=1)
    ref = net.forward_test_u8(imgs)
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
