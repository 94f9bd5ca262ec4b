"""Per-conv error of librr's ResNet trunk vs the oracle, each GPU conv fed the
oracle's own input (isolates the kernel that misbehaves).
usage: python tools/diag_trunk.py [arch] [H] [W] [stride_on] [B]"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import embed_ref  # noqa: E402
from research_image_retrieval_amd import ops  # noqa: E402
from research_image_retrieval_amd import weights as W  # noqa: E402
from research_image_retrieval_amd.networks import ResNet  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else "resnet101"
H = int(sys.argv[2]) if len(sys.argv) > 2 else 224
Wd = int(sys.argv[3]) if len(sys.argv) > 3 else 224
so = sys.argv[4] if len(sys.argv) > 4 else "3x3"
B = int(sys.argv[5]) if len(sys.argv) > 5 else 1
dev = torch.device("cuda:0")
sd = W.synthetic_resnet_state_dict(arch, 0)
net = ResNet(arch, state_dict=sd, device=dev, stride_on=so)
rs = np.random.RandomState(1234)
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, H, Wd, 3), dtype=np.uint8))
x = embed_ref.normalize_u8(imgs)
torch.set_num_threads(16)
nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(dev)  # noqa: E731
nchw = lambda t: t.permute(0, 3, 1, 2).cpu()  # noqa: E731
bn = embed_ref._bn


def rep(name, got, ref):
    e = (got - ref).abs().max().item()
    flag = "  <<<" if e > 1e-5 * max(1.0, ref.abs().max().item()) else ""
    print(f"{name:28s} {tuple(ref.shape)} err {e:.2e} max {ref.abs().max().item():.3f}{flag}", flush=True)


if os.environ.get("DIAG_CHAIN"):
    # chained: GPU chain vs oracle chain per block, and each GPU conv's error on
    # the GPU chain's own input (oracle conv run on that same input)
    with torch.no_grad():
        g = ops.preprocess_u8(imgs.to(dev), out_c=4)
        r = x
        g = net._conv(g, "conv1", 2, 3, True)
        rep("conv1 (own input)", nchw(g), F.relu(bn(F.conv2d(nchw(ops.preprocess_u8(imgs.to(dev), out_c=4))[:, :3],
                                                                sd["conv1.weight"], None, 2, 3), sd, "bn1")))
        g = ops.maxpool2d(g, 3, 2, 1)
        r = F.max_pool2d(F.relu(bn(F.conv2d(r, sd["conv1.weight"], None, 2, 3), sd, "bn1")), 3, 2, 1)
        rep("chain stem", nchw(g), r)
        for li, nb in enumerate(W.RESNET_LAYERS[arch]):
            for bi in range(nb):
                p = f"layer{li + 1}.{bi}"
                s1, s2 = W.block_strides(2 if (bi == 0 and li > 0) else 1, so)
                gi = nchw(g)
                gid = net._conv(g, p + ".downsample.0", s1 * s2, 0, False) if bi == 0 else g
                g1 = net._conv(g, p + ".conv1", s1, 0, True)
                g2 = net._conv(g1, p + ".conv2", s2, 1, True)
                g3 = net._conv(g2, p + ".conv3", 1, 0, True, residual=gid)
                o1 = F.relu(bn(F.conv2d(gi, sd[p + ".conv1.weight"], None, s1), sd, p + ".bn1"))
                rep(p + ".conv1 (own in)", nchw(g1), o1)
                o2 = F.relu(bn(F.conv2d(nchw(g1), sd[p + ".conv2.weight"], None, s2, 1), sd, p + ".bn2"))
                rep(p + ".conv2 (own in)", nchw(g2), o2)
                oid = bn(F.conv2d(gi, sd[p + ".downsample.0.weight"], None, s1 * s2), sd,
                         p + ".downsample.1") if bi == 0 else gi
                o3 = F.relu(oid + bn(F.conv2d(nchw(g2), sd[p + ".conv3.weight"]), sd, p + ".bn3"))
                rep(p + ".conv3 (own in)", nchw(g3), o3)
                idn = r
                if bi == 0:
                    idn = bn(F.conv2d(r, sd[p + ".downsample.0.weight"], None, s1 * s2), sd, p + ".downsample.1")
                y = F.relu(bn(F.conv2d(r, sd[p + ".conv1.weight"], None, s1), sd, p + ".bn1"))
                y = F.relu(bn(F.conv2d(y, sd[p + ".conv2.weight"], None, s2, 1), sd, p + ".bn2"))
                r = F.relu(idn + bn(F.conv2d(y, sd[p + ".conv3.weight"]), sd, p + ".bn3"))
                g = g3
                rep("chain " + p, nchw(g), r)
    sys.exit(0)

with torch.no_grad():
    xu = ops.preprocess_u8(imgs.to(dev), out_c=4)
    rep("preprocess", nchw(xu)[:, :3], x)
    y = F.relu(bn(F.conv2d(x, sd["conv1.weight"], None, 2, 3), sd, "bn1"))
    rep("conv1", nchw(net._conv(nhwc(F.pad(x, (0, 0, 0, 0, 0, 1))), "conv1", 2, 3, True)), y)
    xin = F.max_pool2d(y, 3, 2, 1)
    rep("maxpool", nchw(ops.maxpool2d(nhwc(y), 3, 2, 1)), xin)
    for li, nb in enumerate(W.RESNET_LAYERS[arch]):
        for bi in range(nb):
            p = f"layer{li + 1}.{bi}"
            s1, s2 = W.block_strides(2 if (bi == 0 and li > 0) else 1, so)
            idn = xin
            if bi == 0:
                idn = bn(F.conv2d(xin, sd[p + ".downsample.0.weight"], None, s1 * s2), sd, p + ".downsample.1")
                rep(p + ".downsample", nchw(net._conv(nhwc(xin), p + ".downsample.0", s1 * s2, 0, False)), idn)
            y1 = F.relu(bn(F.conv2d(xin, sd[p + ".conv1.weight"], None, s1), sd, p + ".bn1"))
            rep(p + ".conv1", nchw(net._conv(nhwc(xin), p + ".conv1", s1, 0, True)), y1)
            y2 = F.relu(bn(F.conv2d(y1, sd[p + ".conv2.weight"], None, s2, 1), sd, p + ".bn2"))
            rep(p + ".conv2", nchw(net._conv(nhwc(y1), p + ".conv2", s2, 1, True)), y2)
            y3 = F.relu(idn + bn(F.conv2d(y2, sd[p + ".conv3.weight"]), sd, p + ".bn3"))
            rep(p + ".conv3+res", nchw(net._conv(nhwc(y2), p + ".conv3", 1, 0, True, residual=nhwc(idn))), y3)
            xin = y3
