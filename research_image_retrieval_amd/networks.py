"""networks-style extractors (reference: src/benchmark/networks/) on librr.

Every object here exposes the reference's extractor contract
(networks/RetrievalNet.py:327-344): ``.outputdim`` and
``.forward_test(x: float32 [B,3,H,W]) -> float32 [B,outputdim]`` L2-normalised,
eval-mode semantics, no autograd.  All arithmetic runs in librr's gfx950
kernels; torch only allocates device buffers.  There is no CPU path: calling
forward_test on a CPU tensor raises.
"""
import numpy as np
import torch

from . import ops
from . import weights as W

EPS_L2 = 1e-12  # F.normalize default eps (networks/RetrievalNet.py:343)


class ResNet:
    """torchvision resnet children[:-2] trunk (networks/backbone.py:60-109:
    block1 = conv1/bn1/relu/maxpool, block2..5 = layer1..4), NHWC, BN folded.

    forward(x_nhwc [B,H,W,3]) -> [B,H/32,W/32,2048] NHWC.

    conv_math: "h2" (default) runs every conv, the stem included (NHWC4
    taps, K padded to 224), on the f16x2 split core (fp32-accurate: per conv
    mean error vs float64 within 1.05x and max within 1.25x of the exact-fp32
    core's, descriptors within 2x and <= 1e-6, tests/test_gpu_h2.py; three
    fp16 MFMAs per product; weights split once here, each conv publishes max
    |y| for the next one's split scale); "f32" keeps all convs on the
    exact-fp32 MFMA core.  (The split-bf16 core, "s3", was retired in round 6.)

    stride_on: "3x3" (default) = torchvision v1.5 bottlenecks; "1x1" = the
    reference's own torchvision-free R101, ResNet_DOLG
    (networks/backbone.py:218-274, BottleneckTransform :305-325: the stride of
    a stage's first block sits on the 1x1 `a` conv).  A ResNet_DOLG state dict
    (stem.*, s{K}.b{M}.*) is accepted as is (weights.to_torchvision_keys)."""

    outputdim_block5 = 2048
    outputdim_block4 = 1024

    def __init__(self, name="resnet101", state_dict=None, seed=0, device="cuda", conv_math="h2", stride_on="3x3"):
        if conv_math not in ("h2", "f32"):
            raise ValueError("conv_math must be 'h2' or 'f32'")
        W.block_strides(1, stride_on)  # validates
        self.stride_on = stride_on
        if name not in W.RESNET_LAYERS:
            raise ValueError(f"Unsupported or unknown architecture: {name}!")
        self.name = name
        sd = W.synthetic_resnet_state_dict(name, seed) if state_dict is None else W.to_torchvision_keys(state_dict)
        self.device = torch.device(device)
        folded = W.folded_resnet(sd, name)
        # stem weights padded to 4 input channels (zero) for the NHWC4 tap path
        w1, b1 = folded["conv1"]
        folded["conv1"] = (torch.nn.functional.pad(w1, (0, 1)).contiguous(), b1)
        self.convs = {k: (w.to(self.device), b.to(self.device)) for k, (w, b) in folded.items()}
        self.layers = W.RESNET_LAYERS[name]
        self.conv_math = conv_math
        self.convs_h2 = {}
        if conv_math == "h2":
            self.convs_h2 = {k: ops.H2Conv(w) for k, (w, _) in self.convs.items()}
            # each stage's first block: conv3 + downsample as one GEMM (ops.H2Bottleneck)
            self.fuse_downsample = True
            # the stem conv + ReLU + max-pool as one launch (ops.stem_pool_h2)
            self.fuse_stem_pool = True
            self.bneck_h2 = {}
            for li in range(len(self.layers)):
                p = f"layer{li + 1}.0"
                (w3, b3), (wd, bd) = self.convs[p + ".conv3"], self.convs[p + ".downsample.0"]
                if w3.shape[0] % 256 == 0:
                    self.bneck_h2[p] = ops.H2Bottleneck(w3, b3, wd, bd)

    def _conv(self, x, name, stride, pad, relu, residual=None):
        w, b = self.convs[name]
        return ops.conv2d(x, w, b, stride, pad, residual, relu)

    def _forward_h2(self, x, return_x3, hook=None):
        """The trunk on the f16x2 core: every conv reads its input's max-|x|
        record and writes its output's (one zeroed [2 + 3 blocks, 64] tensor per
        forward); the max-pool output reuses the stem's record (every stem
        output lies in some 3x3/2 window, so the max is the same); the stem,
        its ReLU and the max-pool run as one launch (ops.stem_pool_h2), so the
        stem's full-resolution map never reaches HBM.  A stage's
        first block runs conv3 and its downsample projection as one GEMM
        (ops.bottleneck_out_h2), so the projected identity never reaches HBM.
        hook(i), if given, is called after the i-th conv launch (i = 0: the
        stem) -- the point where a caller can record a stream event."""
        cv, h2 = self.convs, self.convs_h2
        hook = hook or (lambda i: None)
        rec = ops.amax_records(2 + 3 * sum(self.layers), x.device)
        ops.amax_f32(x, rec[0])
        if self.fuse_stem_pool and h2["conv1"].cout == 64:
            x = ops.stem_pool_h2(x, rec[0], h2["conv1"], cv["conv1"][1], 2, 3, rec[1])
        else:
            x = ops.conv2d_h2(x, rec[0], h2["conv1"], cv["conv1"][1], 2, 3, None, True, rec[1])
            x = ops.maxpool2d(x, 3, 2, 1)
        hook(0)
        xa, r, x3, ci = rec[1], 2, None, 1
        for li, nb in enumerate(self.layers):
            for bi in range(nb):
                p = f"layer{li + 1}.{bi}"
                s1, s2 = W.block_strides(2 if (bi == 0 and li > 0) else 1, self.stride_on)
                d = f"{p}.downsample.0"
                fused = bi == 0 and self.fuse_downsample and p in self.bneck_h2
                idn = ops.conv2d_h2(x, xa, h2[d], cv[d][1], s1 * s2, 0, None, False) if bi == 0 and not fused else x
                y = ops.conv2d_h2(x, xa, h2[f"{p}.conv1"], cv[f"{p}.conv1"][1], s1, 0, None, True, rec[r])
                hook(ci)
                y = ops.conv2d_h2(y, rec[r], h2[f"{p}.conv2"], cv[f"{p}.conv2"][1], s2, 1, None, True, rec[r + 1])
                hook(ci + 1)
                if fused:
                    x = ops.bottleneck_out_h2(y, rec[r + 1], x, xa, self.bneck_h2[p], s1 * s2, rec[r + 2])
                else:
                    x = ops.conv2d_h2(y, rec[r + 1], h2[f"{p}.conv3"], cv[f"{p}.conv3"][1], 1, 0, idn, True,
                                      rec[r + 2])
                hook(ci + 2)
                ci += 3
                xa, r = rec[r + 2], r + 3
            if li == 2:
                x3 = x
        return (x3, x) if return_x3 else x

    def forward(self, x, return_x3=False, hook=None):
        """x: NHWC fp32 with 3 channels or 4 (zero 4th channel, preferred).
        return_x3: also return layer3's output, as ResNet_DOLG.forward's
        (x3, x4) (networks/backbone.py:236-242)."""
        if x.shape[-1] == 3:
            x = torch.nn.functional.pad(x, (0, 1))
        if self.conv_math == "h2":
            return self._forward_h2(x.contiguous(), return_x3, hook)
        x = self._conv(x, "conv1", 2, 3, True)
        x = ops.maxpool2d(x, 3, 2, 1)
        x3 = None
        for li, nb in enumerate(self.layers):
            for bi in range(nb):
                p = f"layer{li + 1}.{bi}"
                s1, s2 = W.block_strides(2 if (bi == 0 and li > 0) else 1, self.stride_on)
                idn = self._conv(x, f"{p}.downsample.0", s1 * s2, 0, False) if bi == 0 else x
                y = self._conv(x, f"{p}.conv1", s1, 0, True)
                y = self._conv(y, f"{p}.conv2", s2, 1, True)
                x = self._conv(y, f"{p}.conv3", 1, 0, True, residual=idn)
            if li == 2:
                x3 = x
        return (x3, x) if return_x3 else x

    __call__ = forward


class gem:
    """GeM pooling with python-float p (networks/RetrievalNet.py:318-325)."""

    def __init__(self, p=3.0, eps=1e-6):
        self.p = float(p)
        self.eps = float(eps)

    def __call__(self, x_nhwc):
        return ops.gem_pool(x_nhwc, self.p, self.eps)


class _Extractor:
    def eval(self):
        return self

    def train(self, mode=False):
        if mode:
            raise NotImplementedError("training is out of scope (SURVEY.md §2: row 13)")
        return self

    def to(self, *_a, **_k):
        return self

    in_channels = 3  # NHWC channel count the first layer consumes (4 = RGB + zero pad)

    def _input(self, x):
        if not isinstance(x, torch.Tensor) or not x.is_cuda:
            raise ValueError("forward_test expects a float32 [B,3,H,W] tensor on a ROCm device")
        x = x.float() if x.dtype != torch.float32 else x
        return ops.nchw_to_nhwc(x.contiguous(), out_c=self.in_channels)

    def forward_test_nhwc(self, x_nhwc):
        raise NotImplementedError

    @torch.no_grad()
    def forward_test(self, x):
        return self.forward_test_nhwc(self._input(x))

    @torch.no_grad()
    def forward_test_u8(self, img_nhwc_u8):
        """uint8 [B,H,W,3] pixels -> descriptors, with ToTensor+Normalize fused
        into the first kernel (dataset/configdataset.py:417)."""
        return self.forward_test_nhwc(ops.preprocess_u8(img_nhwc_u8, out_c=self.in_channels))

    @torch.no_grad()
    def forward_test_u8_streams(self, img_nhwc_u8, streams, lag=1):
        """forward_test_u8 with the batch cut into len(streams) contiguous parts,
        part i on HIP stream streams[i], part i + 1 held back until part i has
        launched its lag-th conv (ResNet._forward_h2's hook; lag 0 = after the
        stem).  The parts' kernels then run side by side, offset by about one
        layer, so an MFMA-bound conv of one part shares the chip with an
        HBM-bound conv of the other instead of every layer holding the chip by
        itself.  (Giving each stream's persistent kernels half the CUs, so
        that two kernels always co-run, measured slower: 68.5 vs 66.5 ms per
        1280-image embed, DESIGN.md.)  Each part is exactly
        forward_test_u8 of its images (its own
        max-|x| records for the f16x2 split scales): descriptors are
        bit-identical to running the parts one after another
        (tests/test_gpu_overlap.py) and within the split core's bar of the
        whole batch in one part.  Returns [B, outputdim] on the current stream."""
        x = img_nhwc_u8
        dev = x.device
        cur = torch.cuda.current_stream(dev)
        n = len(streams)
        b = x.shape[0]
        cuts = [b * i // n for i in range(n + 1)]
        outs, gate = [], None
        for i, s in enumerate(streams):
            if cuts[i] == cuts[i + 1]:
                continue
            s.wait_stream(cur)
            if gate is not None:
                s.wait_event(gate)
            ev = torch.cuda.Event()

            def hook(ci, ev=ev, s=s):
                if ci == lag:
                    ev.record(s)

            with torch.cuda.stream(s):
                f = self.forward_test_nhwc(ops.preprocess_u8(x[cuts[i]:cuts[i + 1]], out_c=self.in_channels),
                                           hook=hook)
            outs.append(f)
            gate = ev
        if not outs:
            return self.forward_test_u8(x)
        for s in streams:
            cur.wait_stream(s)
        for f in outs:
            f.record_stream(cur)
        return torch.cat(outs)


class GeM(_Extractor):
    """GeM network (networks/RetrievalNet.py:327-344): backbone -> gem(p=3) ->
    whiten 1x1 conv (outputdim -> 2048, +bias) -> F.normalize.

    As in the reference, the whitening conv takes ``outputdim`` input channels,
    so the network is only well-formed for outputdim == 2048 (:332)."""

    in_channels = 4

    def __init__(self, outputdim=2048, backbone="resnet101", state_dict=None, whiten=None, seed=0, device="cuda",
                 conv_math="h2"):
        if outputdim != 2048:
            raise ValueError("networks.GeM requires outputdim == 2048 (whiten is Conv2d(outputdim, 2048), "
                             "networks/RetrievalNet.py:332)")
        self.device = torch.device(device)
        self.backbone = ResNet(backbone, state_dict, seed, device, conv_math)
        self.pooling = gem()
        if whiten is None:
            ww, wb = W.synthetic_linear(2048, outputdim, seed + 1)
        else:
            ww, wb = whiten
            ww = ww.reshape(ww.shape[0], -1)
        self.whiten_w = ww.float().contiguous().to(self.device)
        self.whiten_b = wb.float().contiguous().to(self.device)
        self.outputdim = outputdim

    def forward_test_nhwc(self, x_nhwc, hook=None):
        f = self.backbone(x_nhwc, hook=hook)
        f = self.pooling(f)
        f = ops.linear(f, self.whiten_w, self.whiten_b)
        return ops.l2_normalize(f, EPS_L2, out=f)


class ConvDimReduction:
    """PCA-whitening as a frozen 1x1 conv (networks/spca.py:205-227):
    weight = P[:dim], bias = -(P m)[:dim]."""

    def __init__(self, input_dim, dim, device="cuda"):
        self.input_dim, self.dim = input_dim, dim
        self.device = torch.device(device)
        self.weight = None
        self.bias = None

    def initialize_pca_whitening(self, des):
        """Fit (m, P) on descriptors des [N, input_dim] (numpy), exactly as
        pcawhitenlearn_shrinkage (networks/backbone.py:42-58) + spca.py:215-227."""
        m, P = pcawhitenlearn_shrinkage(des, device=self.device)
        m, P = m.T, P.T
        self.weight = torch.tensor(P[: self.dim, :], dtype=torch.float32).contiguous().to(self.device)
        shift = -torch.mm(torch.tensor(P, dtype=torch.float32), torch.tensor(m, dtype=torch.float32)).squeeze()
        self.bias = shift[: self.dim].contiguous().to(self.device)
        return m.T, P.T

    def set_params(self, weight, bias):
        self.weight = weight.reshape(weight.shape[0], -1).float().contiguous().to(self.device)
        self.bias = bias.float().contiguous().to(self.device)

    def __call__(self, x):
        if self.weight is None:
            raise RuntimeError("ConvDimReduction: call initialize_pca_whitening or set_params first")
        return ops.linear(x, self.weight, self.bias)


def pcawhitenlearn_shrinkage(X, s=1.0, device="cuda"):
    """PCA whitening with shrinkage (networks/backbone.py:42-58).

    The O(n d^2) part — column mean and centred Gram Xc^T Xc — runs on the GPU
    (rr_pcaw_gram: fp32 MFMA over 8192-row slices, fp64 sums).  The d x d tail
    stays on the host exactly as the reference writes it: symmetrise / 2n,
    LAPACK geev (np.linalg.eig, so eigenvector signs follow the reference's
    solver), descending eigenvalue order, projection scaled by lambda^(-s/2),
    in X's floating dtype.  Returns (mean [1,D], P^T [D,D])."""
    if isinstance(X, torch.Tensor):
        dt = np.float64 if X.dtype == torch.float64 else np.float32
    else:
        X = np.asarray(X)
        dt = X.dtype if X.dtype in (np.float32, np.float64) else np.float32
    x = torch.as_tensor(X).to(device=device, dtype=torch.float32).contiguous()
    n = x.shape[0]
    mean64, gram = ops.pcaw_gram(x)
    gram = gram.cpu().numpy()
    cov = ((gram + gram.T) / (2 * n)).astype(dt)
    lam, vec = np.linalg.eig(cov)
    desc = np.argsort(lam)[::-1]
    lam, vec = lam[desc], vec[:, desc]
    # np.power, not `**`: numpy turns `x ** 0.5` into sqrt, 1 ulp off pow
    proj = np.linalg.inv(np.diag(np.power(lam, 0.5 * s))) @ vec.T
    return mean64.cpu().numpy()[None, :].astype(dt), proj.T


class GeMPCAw(_Extractor):
    """Config C3 extractor: networks.GeM (R101, 2048-d) -> PCA-whitening
    (ConvDimReduction) -> L2.  The reference has no caller wiring the two
    (SURVEY.md §3.4); this is the cirtorch-style composition normalise ->
    whiten -> normalise."""

    def __init__(self, net, pcaw):
        self.in_channels = net.in_channels
        self.net = net
        self.pcaw = pcaw
        self.outputdim = pcaw.dim

    def forward_test_nhwc(self, x_nhwc, hook=None):
        f = self.net.forward_test_nhwc(x_nhwc, hook=hook)
        f = self.pcaw(f)
        return ops.l2_normalize(f, EPS_L2, out=f)


class VisionTransformer(_Extractor):
    """CLIP-style ViT image tower (networks/model.py:206-243) on librr.

    forward(x) returns ``ln_post(x[:, 0]) @ proj`` as the reference does;
    forward_test(x) additionally L2-normalises (the extractor contract).
    Weights: a CLIP-layout state dict (conv1.weight, class_embedding,
    positional_embedding, ln_pre.*, transformer.resblocks.{i}.{attn.in_proj_*,
    attn.out_proj.*, ln_1.*, mlp.c_fc.*, mlp.c_proj.*, ln_2.*}, ln_post.*,
    proj).  LayerNorm eps 1e-5 (nn.LayerNorm default)."""

    def __init__(self, input_resolution=224, patch_size=16, width=768, layers=12, heads=12, output_dim=512,
                 state_dict=None, device="cuda", dtype="fp32"):
        if width % heads or width // heads != 64:
            raise ValueError("VisionTransformer: librr's fused attention needs head_dim == 64")
        if state_dict is None:
            raise ValueError("VisionTransformer needs a state_dict (no pretrained download offline)")
        self.device = torch.device(device)
        self.res, self.patch, self.width, self.layers, self.heads = input_resolution, patch_size, width, layers, heads
        self.output_dim = self.outputdim = output_dim
        self.seq = (input_resolution // patch_size) ** 2 + 1
        if self.seq > 256:
            raise ValueError("VisionTransformer: sequence longer than 256 tokens")
        t = lambda k: state_dict[k].float().contiguous().to(self.device)  # noqa: E731
        # patch conv [width, 3, p, p] -> [width][p][p][3] to match patchify's (kh, kw, c) rows
        self.conv_w = state_dict["conv1.weight"].float().permute(0, 2, 3, 1).reshape(width, -1).contiguous().to(
            self.device)
        self.cls = t("class_embedding")
        self.pos = t("positional_embedding")
        self.ln_pre = (t("ln_pre.weight"), t("ln_pre.bias"))
        self.blocks = []
        for i in range(layers):
            p = f"transformer.resblocks.{i}."
            self.blocks.append({k: t(p + k) for k in (
                "attn.in_proj_weight", "attn.in_proj_bias", "attn.out_proj.weight", "attn.out_proj.bias",
                "ln_1.weight", "ln_1.bias", "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight",
                "mlp.c_proj.bias", "ln_2.weight", "ln_2.bias")})
        self.ln_post = (t("ln_post.weight"), t("ln_post.bias"))
        self.proj_t = state_dict["proj"].float().t().contiguous().to(self.device)  # [out, width]
        if dtype not in ("fp32", "bf16"):
            raise ValueError("VisionTransformer dtype must be fp32 or bf16")
        self.dtype = dtype
        if dtype == "bf16":
            # config C4: bf16 GEMM operands (weights rounded once, RNE), fp32
            # accumulate, fp32 residual stream / LayerNorm / softmax
            self.conv_w_bf = self.conv_w.to(torch.bfloat16)
            for blk in self.blocks:
                for k in ("attn.in_proj_weight", "attn.out_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight"):
                    blk[k + ".bf16"] = blk[k].to(torch.bfloat16)
                # ln_1 / ln_2 folded into the in-proj / c_fc GEMMs (rr_linear_bf16_ln)
                if not ops.ln_fold_supported(width, dtype):
                    continue
                blk["qkv.fold"] = ops.ln_fold_weights(blk["attn.in_proj_weight"], blk["attn.in_proj_bias"],
                                                      blk["ln_1.weight"], blk["ln_1.bias"])
                blk["fc.fold"] = ops.ln_fold_weights(blk["mlp.c_fc.weight"], blk["mlp.c_fc.bias"],
                                                     blk["ln_2.weight"], blk["ln_2.bias"])
        # the LayerNorm fold needs 256-column residual rows and K <= 768 (a
        # wider model, e.g. ViT-L/14's 1024, which networks/model.py:405
        # builds, runs the LayerNorm passes)
        self.ln_fold = ops.ln_fold_supported(width, dtype)

    def _forward_bf16(self, x_nhwc, b):
        # patch rows straight to bf16; ln_pre fused into the token assembly
        p = ops.patchify(x_nhwc, self.patch, out_bf16=True)
        x = ops.vit_tokens(ops.linear_bf16(p, self.conv_w_bf), b, self.cls, self.pos, ln=self.ln_pre)
        if self.ln_fold:
            # ln_1 / ln_2 (:188-190) folded into the in-proj / c_fc GEMMs: the
            # residual GEMMs' epilogues write the bf16 rows and the row
            # statistics, so no LayerNorm pass re-reads the fp32 stream
            xb, st = ops.ln_partials_bf16(x)
            for li, blk in enumerate(self.blocks):
                qkv = ops.linear_bf16_ln_fold(xb, st, *blk["qkv.fold"])
                a = ops.attention_bf16(qkv, b, self.seq, self.heads)
                x, xb, st = ops.linear_bf16_ln_produce(a, blk["attn.out_proj.weight.bf16"], blk["attn.out_proj.bias"], x)
                y = ops.linear_bf16_ln_fold(xb, st, *blk["fc.fold"], act=2)
                if li + 1 < len(self.blocks):
                    x, xb, st = ops.linear_bf16_ln_produce(y, blk["mlp.c_proj.weight.bf16"], blk["mlp.c_proj.bias"], x)
                else:
                    # the last block's output feeds only ln_post (fp32 CLS rows):
                    # no bf16 copy or partials (they would be ~390 MB per
                    # 1280-image step that nothing reads)
                    x = ops.linear_bf16(y, blk["mlp.c_proj.weight.bf16"], blk["mlp.c_proj.bias"], residual=x)
            cls = ops.layernorm(x, *self.ln_post, rows=b, row_stride=self.seq * self.width)
            return ops.linear(cls, self.proj_t)
        for blk in self.blocks:
            y = ops.layernorm_bf16(x, blk["ln_1.weight"], blk["ln_1.bias"])
            # QKV rows in bf16 (RNE, exactly as the attention rounds fp32 rows): half the bytes
            qkv = ops.linear_bf16(y, blk["attn.in_proj_weight.bf16"], blk["attn.in_proj_bias"], out_bf16=True)
            a = ops.attention_bf16(qkv, b, self.seq, self.heads)
            x = ops.linear_bf16(a, blk["attn.out_proj.weight.bf16"], blk["attn.out_proj.bias"], residual=x)
            y = ops.layernorm_bf16(x, blk["ln_2.weight"], blk["ln_2.bias"])
            y = ops.linear_bf16(y, blk["mlp.c_fc.weight.bf16"], blk["mlp.c_fc.bias"], act=2, out_bf16=True)
            x = ops.linear_bf16(y, blk["mlp.c_proj.weight.bf16"], blk["mlp.c_proj.bias"], residual=x)
        cls = ops.layernorm(x, *self.ln_post, rows=b, row_stride=self.seq * self.width)
        return ops.linear(cls, self.proj_t)

    def forward_nhwc(self, x_nhwc):
        b, h, w, _ = x_nhwc.shape
        if self.dtype == "bf16" and h == self.res and w == self.res:
            return self._forward_bf16(x_nhwc, b)
        if h != self.res or w != self.res:
            raise ValueError(f"VisionTransformer: fixed {self.res}x{self.res} input (positional embedding has "
                             f"{self.seq} tokens; networks/model.py:228)")
        x = ops.linear(ops.patchify(x_nhwc, self.patch), self.conv_w)
        x = ops.vit_tokens(x, b, self.cls, self.pos, ln=self.ln_pre)
        for blk in self.blocks:
            y = ops.layernorm(x, blk["ln_1.weight"], blk["ln_1.bias"])
            qkv = ops.linear(y, blk["attn.in_proj_weight"], blk["attn.in_proj_bias"])
            a = ops.attention(qkv, b, self.seq, self.heads)
            x = ops.linear_ex(a, blk["attn.out_proj.weight"], blk["attn.out_proj.bias"], residual=x)
            y = ops.layernorm(x, blk["ln_2.weight"], blk["ln_2.bias"])
            y = ops.linear_ex(y, blk["mlp.c_fc.weight"], blk["mlp.c_fc.bias"], act=2)
            x = ops.linear_ex(y, blk["mlp.c_proj.weight"], blk["mlp.c_proj.bias"], residual=x)
        cls = ops.layernorm(x, *self.ln_post, rows=b, row_stride=self.seq * self.width)
        return ops.linear(cls, self.proj_t)

    @torch.no_grad()
    def forward(self, x):
        return self.forward_nhwc(self._input(x))

    __call__ = forward

    def forward_test_nhwc(self, x_nhwc):
        f = self.forward_nhwc(x_nhwc)
        return ops.l2_normalize(f, EPS_L2, out=f)
