"""extract_vectors — the reference's extractor driver (utils/helpfunc.py:18-48)
on librr.

Same contract: ``extract_vectors(net, loader, ms=[1], device, print_freq)``
returns a CPU float32 [N, net.outputdim] in loader order, with the reference's
single-scale small-image upsampling (:24-26; a single scale ms=[s] is NOT
applied, as the reference's len(ms) == 1 branch ignores it) and multi-scale averaging
(:30-46: bilinear rescale, scales whose result is < 36 px dropped, sum /
(len(ms) - drop), L2 renormalisation).  Differences, all deliberate:
  * loaders may be BATCHED (the reference requires batch size 1);
  * a batch may be float NCHW (the reference's transformed tensors) or uint8
    NHWC pixels, which are normalised on the GPU (rr_preprocess_u8);
  * descriptors leave the device once per batch, not once per image.
"""
import torch

from . import ops

MIN_SIDE = 36
UPSAMPLE_TO = 64.0


def _nhwc(batch, device):
    if isinstance(batch, (list, tuple)):
        batch = batch[0]
    if batch.dim() == 3:
        batch = batch.unsqueeze(0)
    batch = batch.to(device, non_blocking=True)
    if batch.dtype == torch.uint8:
        if batch.shape[-1] != 3:
            raise ValueError("uint8 batches must be NHWC [B,H,W,3]")
        return ops.preprocess_u8(batch)
    return ops.nchw_to_nhwc(batch.float().contiguous())


def _rescale(x_nhwc, s):
    # F.interpolate(scale_factor=s): out = floor(in * s), source index uses 1/s
    h, w = x_nhwc.shape[1], x_nhwc.shape[2]
    oh, ow = int(float(h) * s), int(float(w) * s)
    if oh < 1 or ow < 1:
        return None
    return ops.resize_bilinear(x_nhwc, oh, ow, scale_factor=s)


def _forward(net, x_nhwc):
    if hasattr(net, "forward_test_nhwc"):
        return net.forward_test_nhwc(x_nhwc)
    return net.forward_test(x_nhwc.permute(0, 3, 1, 2).contiguous())


@torch.no_grad()
def extract_vectors(net, loader, ms=(1,), device=torch.device("cuda"), print_freq=100):
    net.eval()
    ms = list(ms)
    out = []
    done = 0
    total = len(loader.dataset) if hasattr(loader, "dataset") else None
    for batch in loader:
        x = _nhwc(batch, device)
        b, h, w = x.shape[0], x.shape[1], x.shape[2]
        if len(ms) == 1:
            # as the reference's single-scale branch (:22-27): ms[0] itself is
            # never applied, only images below 36 px are upsampled
            if h < MIN_SIDE or w < MIN_SIDE:
                x = _rescale(x, max(UPSAMPLE_TO / h, UPSAMPLE_TO / w))
            v = _forward(net, x)
        else:
            acc = None
            drop = 0
            for s in ms:
                xs = x if s == 1 else _rescale(x, s)
                if xs is None or xs.shape[1] < MIN_SIDE or xs.shape[2] < MIN_SIDE:
                    drop += 1
                    continue
                f = _forward(net, xs)
                acc = f.clone() if acc is None else acc.add_(f)
            if acc is None:
                # the reference divides a zero vector by 0 here (NaN descriptor)
                acc = torch.zeros((b, net.outputdim), dtype=torch.float32, device=x.device)
            acc.div_(len(ms) - drop)
            v = ops.l2_normalize(acc, 1e-12, out=acc)
        out.append(v.cpu())
        done += b
        if print_freq and (done // print_freq != (done - b) // print_freq or (total and done == total)):
            print("\r>>>> {}/{} done...".format(done, total if total else "?"), end="")
    if print_freq:
        print("")
    return torch.cat(out, 0) if out else torch.zeros(0, getattr(net, "outputdim", 0))
