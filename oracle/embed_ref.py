"""oracle/embed_ref.py — TEST INFRASTRUCTURE: CPU restatement of the
reference extractor path, in the reference's own op order (NCHW, fp32,
unfolded eval-mode BatchNorm), used as the checker for librr's embed kernels
and as bench.py's ``cpu_baseline``.

Reference sites restated (src/benchmark/):
  * ToTensor + Normalize               dataset/configdataset.py:417
  * torchvision resnet50/101 children[:-2] (conv1, bn1, relu, maxpool,
    layer1..4; Bottleneck v1.5, stride on the 3x3)
                                       networks/backbone.py:60-109,
                                       models/gem_pooling.py:34-44
    torchvision 0.22.1 (requirements.txt:9) is not installed here.  The trunk
    is pinned through the reference's own torchvision-free R101, ResNet_DOLG
    (networks/backbone.py:218-274, ResBlock/BottleneckTransform :305-345),
    which is the same stem / maxpool / eval-BN / residual+ReLU composition at
    depth (3,4,23,3) with the stride on the 1x1 (stride_on="1x1"):
    tests/golden/resnet_dolg.npz holds its (x3, x4).  The v1.5 stride
    placement differs only in which conv of the first block of a stage
    carries stride 2.
  * gem (p=3.0 python float)           networks/RetrievalNet.py:318-325
  * GeMPooling (tensor p)              models/gem_pooling.py:12-23
  * whiten 1x1 conv + F.normalize      networks/RetrievalNet.py:337-344
  * feature_proj Linear + F.normalize  models/gem_pooling.py:58-92
  * ConvDimReduction apply             networks/spca.py:205-227
  * extract_vectors multi-scale        utils/helpfunc.py:18-48
Every piece is pinned by tests/golden fixtures generated from the reference's
own functions (tests/golden/make_golden.py).
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def normalize_u8(img_nhwc_u8, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """uint8 [B,H,W,3] -> fp32 NCHW, ToTensor().div(255) then (x - mean) / std."""
    x = img_nhwc_u8.permute(0, 3, 1, 2).float().div(255)
    m = torch.tensor(mean).view(1, 3, 1, 1)
    s = torch.tensor(std).view(1, 3, 1, 1)
    return (x - m) / s


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], sd[p + ".weight"], sd[p + ".bias"],
                        False, 0.0, BN_EPS)


def resnet_trunk(x, sd, layers, stride_on="3x3", return_x3=False):
    """ResNet forward up to layer4 (eval mode), NCHW, torchvision keys.

    stride_on="3x3": torchvision v1.5 Bottleneck (stride on conv2);
    stride_on="1x1": the reference's own ResNet_DOLG / ResBlock +
    BottleneckTransform (networks/backbone.py:218-274, :305-345; stride on the
    1x1 `a` conv; ResBlock adds bn(proj(x)) + f(x) then ReLU, :340-346).
    return_x3: also return layer3's output (ResNet_DOLG.forward returns (x3, x4))."""
    if stride_on not in ("3x3", "1x1"):
        raise ValueError("stride_on must be '3x3' or '1x1'")
    x = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], None, 2, 3), sd, "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    x3 = None
    for li, nb in enumerate(layers):
        for bi in range(nb):
            p = f"layer{li + 1}.{bi}"
            s = 2 if (bi == 0 and li > 0) else 1
            s1, s2 = (1, s) if stride_on == "3x3" else (s, 1)
            idn = x
            if bi == 0:
                idn = _bn(F.conv2d(x, sd[p + ".downsample.0.weight"], None, s), sd, p + ".downsample.1")
            y = F.relu(_bn(F.conv2d(x, sd[p + ".conv1.weight"], None, s1), sd, p + ".bn1"))
            y = F.relu(_bn(F.conv2d(y, sd[p + ".conv2.weight"], None, s2, 1), sd, p + ".bn2"))
            y = _bn(F.conv2d(y, sd[p + ".conv3.weight"]), sd, p + ".bn3")
            x = F.relu(idn + y)
        if li == 2:
            x3 = x
    return (x3, x) if return_x3 else x


def gem(x, p=3.0, eps=1e-6):
    return F.avg_pool2d(x.clamp(min=eps).pow(p), (x.size(-2), x.size(-1))).pow(1.0 / p)


def gem_net_forward_test(x, sd, layers, whiten_w, whiten_b, stride_on="3x3"):
    """networks.GeM.forward_test: trunk -> gem -> whiten 1x1 conv -> F.normalize."""
    f = resnet_trunk(x, sd, layers, stride_on)
    f = gem(f)
    f = F.conv2d(f, whiten_w.view(whiten_w.shape[0], -1, 1, 1), whiten_b).squeeze(-1).squeeze(-1)
    return F.normalize(f, dim=-1)


def gem_model_descriptor(x, sd, layers, proj_w, proj_b, p=3.0, stride_on="3x3"):
    """GeMModel.extract_descriptor: trunk -> GeMPooling -> Linear -> F.normalize(p=2, dim=1)."""
    f = resnet_trunk(x, sd, layers, stride_on)
    pt = torch.ones(1) * p
    f = F.avg_pool2d(f.clamp(min=1e-6).pow(pt), (f.size(-2), f.size(-1))).pow(1.0 / pt)
    f = F.linear(f.view(f.size(0), -1), proj_w, proj_b)
    return F.normalize(f, p=2, dim=1)


def pcawhitenlearn_ref(X, s=1.0):
    """CPU restatement of pcawhitenlearn_shrinkage (networks/backbone.py:42-58),
    in X's dtype with numpy: m = X.mean(0); Xc = X - m; Xcov = Xc^T Xc,
    symmetrised / 2N; np.linalg.eig; descending order; P = diag(lam^(s/2))^-1 V^T.
    Returns (m [1,D], P^T)."""
    import numpy as np
    n = X.shape[0]
    m = X.mean(axis=0, keepdims=True)
    xc = X - m
    cov = xc.T @ xc
    cov = (cov + cov.T) / (2 * n)
    lam, vec = np.linalg.eig(cov)
    order = np.argsort(lam)[::-1]
    lam, vec = lam[order], vec[:, order]
    proj = np.linalg.inv(np.diag(np.power(lam, 0.5 * s))) @ vec.T
    return m, proj.T


def pcaw_apply(x, w, b):
    """ConvDimReduction forward on [B,D] descriptors, then F.normalize."""
    return F.normalize(F.linear(x, w, b), dim=-1)


def extract_vectors_ref(forward_test, images, ms=(1,)):
    """utils/helpfunc.py:18-48 over a list of [1,3,H,W] tensors (batch 1)."""
    out = []
    for inp in images:
        if len(ms) == 1:
            if inp.shape[2] < 36 or inp.shape[3] < 36:
                s = max(64 / inp.shape[2], 64 / inp.shape[3])
                inp = F.interpolate(inp, scale_factor=s, mode="bilinear", align_corners=False)
            out.append(forward_test(inp).squeeze(0))
        else:
            vec = None
            drop = 0
            # (the reference starts from zeros: all scales dropped -> 0/0 = NaN)
            for s in ms:
                x = inp.clone() if s == 1 else F.interpolate(inp, scale_factor=s, mode="bilinear",
                                                             align_corners=False)
                if x.shape[2] < 36 or x.shape[3] < 36:
                    drop += 1
                    continue
                v = forward_test(x).squeeze(0)
                vec = v.clone() if vec is None else vec + v
            if vec is None:
                vec = torch.zeros(out[0].shape[0] if out else 1)
            vec = vec / (len(ms) - drop)
            out.append(F.normalize(vec, p=2, dim=0))
    return torch.stack(out, 0)


def rank_ref(q, g):
    """iris_evaluate.py:379-386: normalise, torch.mm, np.argsort(-S) (stable here)."""
    import numpy as np
    q = F.normalize(q, p=2, dim=1)
    g = F.normalize(g, p=2, dim=1)
    sim = torch.mm(q, g.t()).numpy()
    return sim, np.argsort(-sim, axis=1, kind="stable")


def vit_forward(x, sd, patch, width, layers, heads, eps=1e-5):
    """networks/model.py:206-243 (VisionTransformer.forward) restated with
    torch.nn.functional, NCHW fp32 input -> ln_post(x[:, 0]) @ proj."""
    b = x.shape[0]
    x = F.conv2d(x, sd["conv1.weight"], None, patch)
    x = x.reshape(b, width, -1).permute(0, 2, 1)
    cls = sd["class_embedding"] + torch.zeros(b, 1, width)
    x = torch.cat([cls, x], dim=1) + sd["positional_embedding"]
    x = F.layer_norm(x, (width,), sd["ln_pre.weight"], sd["ln_pre.bias"], eps)
    hd = width // heads
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        y = F.layer_norm(x, (width,), sd[p + "ln_1.weight"], sd[p + "ln_1.bias"], eps)
        qkv = F.linear(y, sd[p + "attn.in_proj_weight"], sd[p + "attn.in_proj_bias"])
        q, k, v = qkv.split(width, dim=-1)
        sh = lambda t: t.reshape(b, -1, heads, hd).transpose(1, 2)  # noqa: E731
        att = torch.softmax((sh(q) / hd ** 0.5) @ sh(k).transpose(-2, -1), dim=-1) @ sh(v)
        att = att.transpose(1, 2).reshape(b, -1, width)
        x = x + F.linear(att, sd[p + "attn.out_proj.weight"], sd[p + "attn.out_proj.bias"])
        y = F.layer_norm(x, (width,), sd[p + "ln_2.weight"], sd[p + "ln_2.bias"], eps)
        y = F.linear(y, sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"])
        y = y * torch.sigmoid(1.702 * y)
        x = x + F.linear(y, sd[p + "mlp.c_proj.weight"], sd[p + "mlp.c_proj.bias"])
    x = F.layer_norm(x[:, 0, :], (width,), sd["ln_post.weight"], sd["ln_post.bias"], eps)
    return x @ sd["proj"]
