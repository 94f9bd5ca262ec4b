"""Backbone weights: seeded synthetic torchvision-keyed state dicts, local
checkpoint loading, reference key-layout remaps and eval-mode BN folding.

No network access exists (pretrained=True/'v1'/'v2' in the reference downloads
ImageNet weights, networks/backbone.py:63-72, models/gem_pooling.py:35-38), so
weights come either from a LOCAL torchvision-keyed file or from a seeded
generator.  The generator uses numpy RandomState (stream-stable across numpy
versions) so the oracle, the tests and bench.py all rebuild identical weights
from a seed.
"""
import collections

import numpy as np
import torch

# torchvision resnet{50,101} bottleneck counts (networks/backbone.py:63-72 via
# torchvision.models.resnet50/101; models/gem_pooling.py:34-38)
RESNET_LAYERS = {"resnet50": (3, 4, 6, 3), "resnet101": (3, 4, 23, 3), "resnet152": (3, 8, 36, 3)}
BN_EPS = 1e-5
# Where a downsampling bottleneck puts its stride: "3x3" = torchvision v1.5
# (conv2), "1x1" = MSRA / pycls, the reference's own torchvision-free R101
# (networks/backbone.py:310-312: BottleneckTransform.a carries the stride).
STRIDE_ON = ("3x3", "1x1")


def block_strides(stride, stride_on):
    """(conv1 stride, conv2 stride) of a bottleneck whose block stride is `stride`."""
    if stride_on not in STRIDE_ON:
        raise ValueError(f"stride_on must be one of {STRIDE_ON}")
    return (1, stride) if stride_on == "3x3" else (stride, 1)


def resnet_conv_specs(arch):
    """Ordered (prefix, cout, cin, k) of every conv + its BN prefix, torchvision layout."""
    layers = RESNET_LAYERS[arch]
    specs = [("conv1", "bn1", 64, 3, 7)]
    inplanes = 64
    for li, nblocks in enumerate(layers):
        planes = 64 * (2 ** li)
        for bi in range(nblocks):
            p = f"layer{li + 1}.{bi}"
            specs.append((f"{p}.conv1", f"{p}.bn1", planes, inplanes, 1))
            specs.append((f"{p}.conv2", f"{p}.bn2", planes, planes, 3))
            specs.append((f"{p}.conv3", f"{p}.bn3", planes * 4, planes, 1))
            if bi == 0:
                specs.append((f"{p}.downsample.0", f"{p}.downsample.1", planes * 4, inplanes, 1))
            inplanes = planes * 4
    return specs


def synthetic_resnet_state_dict(arch="resnet101", seed=0):
    """Seeded torchvision-keyed trunk weights (conv1..layer4; no fc).

    Convs: Kaiming-normal (fan_out, ReLU), as torchvision's init.  BatchNorm
    running statistics and affine parameters are randomised (not identity) so
    that BN folding is exercised; the last BN of every bottleneck gets a small
    gamma so activations stay O(1) through 33 residual blocks."""
    rs = np.random.RandomState(seed)
    sd = collections.OrderedDict()
    for conv, bn, cout, cin, k in resnet_conv_specs(arch):
        std = np.sqrt(2.0 / (cout * k * k))
        sd[conv + ".weight"] = torch.from_numpy((rs.standard_normal((cout, cin, k, k)) * std).astype(np.float32))
        last = bn.endswith("bn3") or bn.endswith("downsample.1")
        lo, hi = (0.05, 0.25) if last else (0.5, 1.0)
        sd[bn + ".weight"] = torch.from_numpy(rs.uniform(lo, hi, cout).astype(np.float32))
        sd[bn + ".bias"] = torch.from_numpy((rs.standard_normal(cout) * 0.05).astype(np.float32))
        sd[bn + ".running_mean"] = torch.from_numpy((rs.standard_normal(cout) * 0.05).astype(np.float32))
        sd[bn + ".running_var"] = torch.from_numpy(rs.uniform(0.5, 1.5, cout).astype(np.float32))
        sd[bn + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.int64)
    return sd


def synthetic_linear(out_dim, in_dim, seed, bias=True, scale=None):
    """Seeded Linear / 1x1-conv weights ([out,in], [out])."""
    rs = np.random.RandomState(seed)
    s = scale if scale is not None else 1.0 / np.sqrt(in_dim)
    w = torch.from_numpy((rs.uniform(-1, 1, (out_dim, in_dim)) * s).astype(np.float32))
    b = torch.from_numpy((rs.uniform(-1, 1, out_dim) * s).astype(np.float32)) if bias else None
    return w, b


# ---- reference key layouts -------------------------------------------------
# networks.ResNet (networks/backbone.py:93-101) renames children[:-2] into
# block1 = [conv1, bn1, relu, maxpool], block2..5 = layer1..4;
# GeMModel (models/gem_pooling.py:44) keeps nn.Sequential indices 0..7.
_SEQ_TO_TV = {"0": "conv1", "1": "bn1", "4": "layer1", "5": "layer2", "6": "layer3", "7": "layer4"}
_BLOCK_TO_TV = {"block2": "layer1", "block3": "layer2", "block4": "layer3", "block5": "layer4"}
# ResNet_DOLG (networks/backbone.py:218-274, blocks :305-345): stem.{conv,bn},
# s{K}.b{M}.{proj,bn} (projection shortcut), s{K}.b{M}.f.{a,a_bn,b,b_bn,c,c_bn}
_DOLG_F_TO_TV = {"a": "conv1", "a_bn": "bn1", "b": "conv2", "b_bn": "bn2", "c": "conv3", "c_bn": "bn3"}
_DOLG_SC_TO_TV = {"proj": "downsample.0", "bn": "downsample.1"}


def _dolg_to_tv(parts):
    if parts[0] == "stem" and len(parts) >= 3:
        return [{"conv": "conv1", "bn": "bn1"}.get(parts[1], "?")] + parts[2:]
    if len(parts) >= 4 and parts[0][:1] == "s" and parts[0][1:].isdigit() and parts[1][:1] == "b":
        layer = f"layer{int(parts[0][1:])}"
        blk = str(int(parts[1][1:]) - 1)
        if parts[2] == "f" and len(parts) >= 5 and parts[3] in _DOLG_F_TO_TV:
            return [layer, blk, _DOLG_F_TO_TV[parts[3]]] + parts[4:]
        if parts[2] in _DOLG_SC_TO_TV:
            return [layer, blk, _DOLG_SC_TO_TV[parts[2]]] + parts[3:]
    return None


def to_dolg_keys(sd):
    """torchvision trunk keys -> ResNet_DOLG keys (the inverse of the DOLG
    branch of to_torchvision_keys); used to load seeded weights into the
    reference's own R101 when generating the trunk fixture."""
    inv_f = {v: k for k, v in _DOLG_F_TO_TV.items()}
    out = collections.OrderedDict()
    for k, v in sd.items():
        parts = k.split(".")
        if parts[0] in ("conv1", "bn1"):
            nk = ["stem", {"conv1": "conv", "bn1": "bn"}[parts[0]]] + parts[1:]
        else:
            li, bi = int(parts[0][5:]), int(parts[1])
            head = [f"s{li}", f"b{bi + 1}"]
            if parts[2] == "downsample":
                nk = head + [{"0": "proj", "1": "bn"}[parts[3]]] + parts[4:]
            else:
                nk = head + ["f", inv_f[parts[2]]] + parts[3:]
        out[".".join(nk)] = v
    return out


def to_torchvision_keys(sd, prefix=""):
    """Map a reference checkpoint's trunk keys to torchvision keys.

    Accepts plain torchvision keys, networks-style ``backbone.block{1..5}.*``
    (e.g. ``globalmodel.backbone.block1.0.weight`` saved by the reference's
    load_checkpoint, utils/helpfunc.py:342-368), Table-1
    ``backbone.backbone.{0..7}.*`` keys and ResNet_DOLG keys
    (``stem.conv``, ``s3.b7.f.b_bn``, ``s1.b1.proj``; networks/backbone.py:218-345,
    whose bottlenecks carry the stride on the 1x1: build the trunk with
    stride_on="1x1").  Non-trunk keys are dropped."""
    out = collections.OrderedDict()
    for k, v in sd.items():
        if prefix and not k.startswith(prefix):
            continue
        k2 = k[len(prefix):]
        for lead in ("module.", "globalmodel.", "backbone.backbone.", "backbone."):
            if k2.startswith(lead):
                k2 = k2[len(lead):]
        parts = k2.split(".")
        dolg = _dolg_to_tv(parts)
        if dolg is not None:
            parts = dolg
        elif parts[0] == "block1" and len(parts) >= 3:
            parts = [{"0": "conv1", "1": "bn1"}.get(parts[1], "?")] + parts[2:]
        elif parts[0] in _BLOCK_TO_TV:
            parts = [_BLOCK_TO_TV[parts[0]]] + parts[1:]
        elif parts[0] in _SEQ_TO_TV:
            parts = [_SEQ_TO_TV[parts[0]]] + parts[1:]
        k2 = ".".join(parts)
        if k2.startswith(("conv1.", "bn1.", "layer1.", "layer2.", "layer3.", "layer4.")):
            out[k2] = v
    return out


def load_state_dict(path):
    """Load a LOCAL checkpoint without executing anything from the file."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    obj = torch.load(path, map_location="cpu", weights_only=True)
    for key in ("state_dict", "model"):
        if isinstance(obj, dict) and key in obj and isinstance(obj[key], dict):
            obj = obj[key]
    return obj


def fold_bn(conv_w, bn, eps=BN_EPS):
    """Eval-mode BN folded into the preceding bias-free conv.

    Returns (w [Cout,KH,KW,Cin] fp32 NHWC-ready, bias [Cout] fp32); the fold
    is computed in float64 then rounded once."""
    w = conv_w.double()
    g = bn["weight"].double()
    b = bn["bias"].double()
    m = bn["running_mean"].double()
    v = bn["running_var"].double()
    scale = g / torch.sqrt(v + eps)
    wf = (w * scale[:, None, None, None]).permute(0, 2, 3, 1).contiguous().float()
    bf = (b - m * scale).float()
    return wf, bf


def folded_resnet(sd, arch):
    """torchvision-keyed trunk -> ordered list of folded (name, w, b, stride, pad)."""
    def bn(prefix):
        return {k: sd[f"{prefix}.{k}"] for k in ("weight", "bias", "running_mean", "running_var")}

    out = collections.OrderedDict()
    for conv, bnp, cout, cin, k in resnet_conv_specs(arch):
        w = sd[conv + ".weight"]
        if tuple(w.shape) != (cout, cin, k, k):
            raise ValueError(f"{conv}: expected {(cout, cin, k, k)}, got {tuple(w.shape)}")
        out[conv] = fold_bn(w, bn(bnp))
    return out


def resnet_conv_flops(arch, h, w, stride_on="3x3"):
    """Algorithmic FLOPs (2*M*N*K) of every trunk conv for one h x w image,
    following networks.ResNet.forward's strides/pads."""
    def out(x, k, s, p):
        return (x + 2 * p - k) // s + 1

    flops = {}
    H, Wd = out(h, 7, 2, 3), out(w, 7, 2, 3)
    flops["conv1"] = 2 * H * Wd * 64 * 7 * 7 * 3
    H, Wd = out(H, 3, 2, 1), out(Wd, 3, 2, 1)
    inplanes = 64
    for li, nb in enumerate(RESNET_LAYERS[arch]):
        planes = 64 * 2 ** li
        for bi in range(nb):
            s = 2 if (bi == 0 and li > 0) else 1
            s1, s2 = block_strides(s, stride_on)
            p = f"layer{li + 1}.{bi}"
            H1, W1 = out(H, 1, s1, 0), out(Wd, 1, s1, 0)
            Ho, Wo = out(H1, 3, s2, 1), out(W1, 3, s2, 1)
            if bi == 0:
                flops[p + ".downsample.0"] = 2 * Ho * Wo * planes * 4 * inplanes
            flops[p + ".conv1"] = 2 * H1 * W1 * planes * inplanes
            flops[p + ".conv2"] = 2 * Ho * Wo * planes * planes * 9
            flops[p + ".conv3"] = 2 * Ho * Wo * planes * 4 * planes
            H, Wd, inplanes = Ho, Wo, planes * 4
    return flops


def resnet_conv_bytes(arch, h, w, batch, stride_on="3x3", weight_bytes=6, fused=False):
    """Algorithmic HBM bytes of every trunk conv launch for `batch` h x w
    images (the same layer walk as resnet_conv_flops): the fp32 NHWC input map
    read once (the stem's NHWC4 image: 4 channels), the fp32 output written
    once, the block's fp32 identity read once by the residual conv3, and the
    weights once per launch (`weight_bytes` per parameter: 6 = the split-bf16
    core's three bf16 planes, 4 = fp32 or the f16x2 core's two fp16 planes).
    fused (the f16x2 trunk, networks.ResNet._forward_h2): the stem writes only
    its max-pooled map (rr_stem_pool_h2), and a stage's first block computes
    conv3 and the downsample projection as one GEMM (rr_bottleneck_out_h2),
    which reads the block input at the sampled pixels and writes no projected
    identity (its bytes are split between the two names)."""
    def out(x, k, s, p):
        return (x + 2 * p - k) // s + 1

    by = {}
    H, Wd = out(h, 7, 2, 3), out(w, 7, 2, 3)
    Hp, Wp = out(H, 3, 2, 1), out(Wd, 3, 2, 1)
    by["conv1"] = batch * (h * w * 4 + (Hp * Wp if fused else H * Wd) * 64) * 4 + 64 * 7 * 7 * 4 * weight_bytes
    H, Wd = Hp, Wp
    inplanes = 64
    for li, nb in enumerate(RESNET_LAYERS[arch]):
        planes = 64 * 2 ** li
        for bi in range(nb):
            s = 2 if (bi == 0 and li > 0) else 1
            s1, s2 = block_strides(s, stride_on)
            p = f"layer{li + 1}.{bi}"
            H1, W1 = out(H, 1, s1, 0), out(Wd, 1, s1, 0)
            Ho, Wo = out(H1, 3, s2, 1), out(W1, 3, s2, 1)
            x_in = H * Wd * inplanes
            wd_by = planes * 4 * inplanes * weight_bytes
            if bi == 0 and fused:
                by[p + ".downsample.0"] = batch * Ho * Wo * inplanes * 4 + wd_by
            elif bi == 0:
                by[p + ".downsample.0"] = batch * (x_in + Ho * Wo * planes * 4) * 4 + wd_by
            by[p + ".conv1"] = batch * (x_in + H1 * W1 * planes) * 4 + planes * inplanes * weight_bytes
            by[p + ".conv2"] = batch * (H1 * W1 * planes + Ho * Wo * planes) * 4 + planes * planes * 9 * weight_bytes
            n_res = 0 if (bi == 0 and fused) else 1  # the identity map read by the residual epilogue
            by[p + ".conv3"] = batch * (Ho * Wo * planes + (1 + n_res) * Ho * Wo * planes * 4) * 4 + \
                planes * 4 * planes * weight_bytes
            H, Wd, inplanes = Ho, Wo, planes * 4
    return by


def synthetic_vit_state_dict(width=768, layers=12, heads=12, patch=16, res=224, out_dim=512, seed=0):
    """Seeded CLIP-layout ViT weights (networks/model.py:206-243 key names)."""
    rs = np.random.RandomState(seed)
    sc = width ** -0.5
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))  # noqa: E731
    sd = collections.OrderedDict()
    sd["conv1.weight"] = t(rs.standard_normal((width, 3, patch, patch)) / np.sqrt(3 * patch * patch))
    sd["class_embedding"] = t(rs.standard_normal(width) * sc)
    sd["positional_embedding"] = t(rs.standard_normal(((res // patch) ** 2 + 1, width)) * sc)
    sd["ln_pre.weight"], sd["ln_pre.bias"] = t(np.ones(width)), t(np.zeros(width))
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        sd[p + "attn.in_proj_weight"] = t(rs.standard_normal((3 * width, width)) * sc)
        sd[p + "attn.in_proj_bias"] = t(np.zeros(3 * width))
        sd[p + "attn.out_proj.weight"] = t(rs.standard_normal((width, width)) * sc)
        sd[p + "attn.out_proj.bias"] = t(np.zeros(width))
        sd[p + "ln_1.weight"], sd[p + "ln_1.bias"] = t(np.ones(width)), t(np.zeros(width))
        sd[p + "mlp.c_fc.weight"] = t(rs.standard_normal((4 * width, width)) * sc)
        sd[p + "mlp.c_fc.bias"] = t(np.zeros(4 * width))
        sd[p + "mlp.c_proj.weight"] = t(rs.standard_normal((width, 4 * width)) * (0.5 / np.sqrt(4 * width)))
        sd[p + "mlp.c_proj.bias"] = t(np.zeros(width))
        sd[p + "ln_2.weight"], sd[p + "ln_2.bias"] = t(np.ones(width)), t(np.zeros(width))
    sd["ln_post.weight"], sd["ln_post.bias"] = t(np.ones(width)), t(np.zeros(width))
    sd["proj"] = t(rs.standard_normal((width, out_dim)) * sc)
    return sd


def vit_flops(width=768, layers=12, heads=12, patch=16, res=224, out_dim=512):
    """Algorithmic FLOPs per image: (GEMM FLOPs, attention FLOPs)."""
    L = (res // patch) ** 2 + 1
    gemm = 2 * (L - 1) * width * 3 * patch * patch
    gemm += layers * 2 * L * width * (3 * width + width + 4 * width + 4 * width)
    gemm += 2 * width * out_dim
    attn = layers * heads * 2 * (2 * L * L * (width // heads))
    return gemm, attn
