"""Table-1 style extractors and registry (reference: src/benchmark/models/).

Mirrors models/gem_pooling.py:12-143 and models/wrappers.py:18-90 for the GeM
family named by the hot path: ``get_model('gem_r50' | 'gem_r101', num_classes,
feature_dim=..., gem_p=...)`` returns a wrapper whose
``extract_global_descriptor(x)`` yields L2-normalised [B, feature_dim] fp32.
Training (``forward(x, targets)`` losses, optimizers) is out of scope
(SURVEY.md §2 row 13): ``forward`` only produces eval-mode logits.
"""
import torch

from . import ops
from . import weights as W
from .networks import ResNet, _Extractor, EPS_L2


class GeMPooling:
    """GeM with a tensor-valued p (models/gem_pooling.py:12-23).  The
    reference stores p as a 1-element Parameter; the exponent 1/p is formed
    in fp32 from it, which is what gem_pool's powf path does."""

    def __init__(self, p=3.0, eps=1e-6):
        self.p = torch.ones(1) * p
        self.eps = eps

    def __call__(self, x_nhwc):
        return ops.gem_pool(x_nhwc, float(self.p.item()), self.eps)


class GeMModel(_Extractor):
    """resnet trunk -> GeMPooling -> feature_proj Linear(2048, feature_dim)
    (models/gem_pooling.py:26-92); extract_descriptor adds F.normalize(p=2, dim=1)."""

    in_channels = 4

    def __init__(self, backbone="resnet50", pretrained=False, num_classes=1000, feature_dim=2048, gem_p=3.0,
                 state_dict=None, seed=0, device="cuda", conv_math="h2", stride_on="3x3"):
        if pretrained:
            raise ValueError("pretrained weights need a download; pass a local state_dict instead "
                             "(models/gem_pooling.py:35 defaults to pretrained=True)")
        if backbone not in ("resnet50", "resnet101"):
            raise ValueError(f"Unsupported backbone: {backbone}")
        self.device = torch.device(device)
        self.backbone = ResNet(backbone, state_dict, seed, device, conv_math=conv_math, stride_on=stride_on)
        self.gem_pool = GeMPooling(p=gem_p)
        backbone_dim = 2048
        pw, pb = _from_sd(state_dict, "feature_proj") or W.synthetic_linear(feature_dim, backbone_dim, seed + 2)
        self.proj_w = pw.float().contiguous().to(self.device)
        self.proj_b = pb.float().contiguous().to(self.device)
        cw, cb = _from_sd(state_dict, "classifier") or W.synthetic_linear(num_classes, feature_dim, seed + 3)
        self.cls_w = cw.float().contiguous().to(self.device)
        self.cls_b = cb.float().contiguous().to(self.device)
        self.feature_dim = feature_dim
        self.outputdim = feature_dim

    def extract_features_nhwc(self, x_nhwc):
        f = self.backbone(x_nhwc)
        f = self.gem_pool(f)
        return ops.linear(f, self.proj_w, self.proj_b)

    @torch.no_grad()
    def extract_features(self, x):
        return self.extract_features_nhwc(self._input(x))

    def forward_test_nhwc(self, x_nhwc):
        f = self.extract_features_nhwc(x_nhwc)
        return ops.l2_normalize(f, EPS_L2, out=f)

    @torch.no_grad()
    def extract_descriptor(self, x):
        return self.forward_test(x)

    @torch.no_grad()
    def forward(self, x, targets=None):
        feats = self.extract_features(x)
        return None, ops.linear(feats, self.cls_w, self.cls_b)

    __call__ = forward


def _from_sd(sd, name):
    if sd is None:
        return None
    for pre in ("", "backbone.", "module.backbone."):
        k = f"{pre}{name}.weight"
        if k in sd:
            return sd[k], sd[f"{pre}{name}.bias"]
    return None


class GeMWrapper(_Extractor):
    """models/gem_pooling.py:95-119: training-loop facade over GeMModel."""

    in_channels = 4

    def __init__(self, num_classes, backbone="resnet50", feature_dim=2048, gem_p=3.0, **kw):
        self.backbone = GeMModel(backbone=backbone, num_classes=num_classes, feature_dim=feature_dim, gem_p=gem_p,
                                 **kw)
        self.outputdim = feature_dim

    def forward_test_nhwc(self, x_nhwc):
        return self.backbone.forward_test_nhwc(x_nhwc)

    @torch.no_grad()
    def forward(self, x, targets=None):
        return self.backbone(x)

    __call__ = forward

    @torch.no_grad()
    def extract_global_descriptor(self, x):
        return self.backbone.extract_descriptor(x)


def get_gem_model(num_classes, backbone="resnet50", **kwargs):
    return GeMWrapper(num_classes=num_classes, backbone=backbone, **kwargs)


MODEL_REGISTRY = {
    "gem_r50": lambda num_classes, **kw: get_gem_model(num_classes, backbone="resnet50", **kw),
    "gem_r101": lambda num_classes, **kw: get_gem_model(num_classes, backbone="resnet101", **kw),
}

# Other Table-1 methods exist in the reference registry (models/wrappers.py:22-50)
# but are outside this build's hot path.
OUT_OF_SCOPE = ("delg_r50", "delg_r101", "token_r50", "token_r101", "how_vlad_r50", "how_vlad_r101",
                "how_asmk_r50", "how_asmk_r101", "senet_g2_50", "senet_g2_101", "sosnet_r50", "sosnet_r101",
                "spoc_r50", "spoc_r101")


def get_model(model_name, num_classes, **kwargs):
    """Factory by name (models/wrappers.py:74-90)."""
    if model_name not in MODEL_REGISTRY:
        if model_name in OUT_OF_SCOPE:
            raise NotImplementedError(f"{model_name} is outside the accelerated hot path (SURVEY.md §2)")
        raise ValueError(f"Unknown model: {model_name}. Available models: {list(MODEL_REGISTRY)}")
    return MODEL_REGISTRY[model_name](num_classes, **kwargs)
