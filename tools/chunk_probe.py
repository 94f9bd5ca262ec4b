"""Does running a ResNet stage depth-first over image chunks (so each chunk's
activations stay in the 256 MiB Infinity Cache between layers) beat running
every layer over the whole batch?  Per R101 stage, the time to push all B
images through that stage's blocks in chunks of c images (chunk = one
sequence of the stage's launches), on the f16x2 core.
usage: chunk_probe.py [B] [chunks,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from research_image_retrieval_amd import ops  # noqa: E402
from research_image_retrieval_amd import weights as W  # noqa: E402
from research_image_retrieval_amd.networks import ResNet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1280
CH = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "1280,640,320,160,80,40").split(",")]
dev = torch.device("cuda:0")
net = ResNet("resnet101", seed=0, device=dev)
cv, h2 = net.convs, net.convs_h2


def stage(li, x, xa_rec):
    """layer{li+1} on x (record xa_rec), the same launches as _forward_h2."""
    nb = net.layers[li]
    rec = ops.amax_records(3 * nb, x.device)
    xa, r = xa_rec, 0
    for bi in range(nb):
        p = f"layer{li + 1}.{bi}"
        s1, s2 = W.block_strides(2 if (bi == 0 and li > 0) else 1, net.stride_on)
        fused = bi == 0 and p in net.bneck_h2
        d = f"{p}.downsample.0"
        idn = ops.conv2d_h2(x, xa, h2[d], cv[d][1], s1 * s2, 0, None, False) if bi == 0 and not fused else x
        y = ops.conv2d_h2(x, xa, h2[f"{p}.conv1"], cv[f"{p}.conv1"][1], s1, 0, None, True, rec[r])
        y = ops.conv2d_h2(y, rec[r], h2[f"{p}.conv2"], cv[f"{p}.conv2"][1], s2, 1, None, True, rec[r + 1])
        if fused:
            x = ops.bottleneck_out_h2(y, rec[r + 1], x, xa, net.bneck_h2[p], s1 * s2, rec[r + 2])
        else:
            x = ops.conv2d_h2(y, rec[r + 1], h2[f"{p}.conv3"], cv[f"{p}.conv3"][1], 1, 0, idn, True, rec[r + 2])
        xa, r = rec[r + 2], r + 3
    return x, xa


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


x = torch.relu(torch.randn(B, 56, 56, 64, device=dev))
inputs = []
for li in range(4):
    rec = ops.amax_records(1, dev)
    ops.amax_f32(x, rec[0])
    inputs.append((x, rec))
    x, _ = stage(li, x, rec[0])
torch.cuda.synchronize()
tot = {c: 0.0 for c in CH}
for li in range(4):
    x, _ = inputs[li]
    line = []
    for c in CH:
        parts = []
        for i in range(0, B, c):
            xc = x[i:i + c].contiguous()
            rc = ops.amax_records(1, dev)
            ops.amax_f32(xc, rc[0])
            parts.append((xc, rc))

        def run():
            for xc, rc in parts:
                stage(li, xc, rc[0])
        ms = timed(run)
        tot[c] += ms
        line.append(f"c{c} {ms:7.2f} ms")
        del parts
    print(f"layer{li + 1} (x{net.layers[li]}, {tuple(x.shape[1:])}): " + " | ".join(line), flush=True)
print("sum over stages: " + " | ".join(f"c{c} {tot[c]:.2f} ms" for c in CH), flush=True)
