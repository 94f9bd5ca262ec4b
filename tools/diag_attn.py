# diagnostic: bf16-math attention vs float64 on structured inputs
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from research_image_retrieval_amd import ops
dev = torch.device("cuda:0")

def ref(qkv, b, seq, heads):
    x = qkv.bfloat16().double().view(b, seq, 3, heads, 64)
    q, k, v = x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2)
    r = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
    return r.transpose(1, 2).reshape(b * seq, heads * 64)

for seq in (32, 64, 197):
    for mode in ("zeroK", "onehotV", "rand"):
        b, heads = 1, 1
        g = torch.Generator().manual_seed(seq)
        qkv = torch.randn(b * seq, 3 * heads * 64, generator=g)
        if mode == "zeroK":
            qkv[:, 64:128] = 0
        if mode == "onehotV":
            qkv[:, 128:] = 0
            for key in range(min(seq, 64)):
                qkv[key, 128 + key] = 1.0
        out = ops.attention_bf16(qkv.to(dev), b, seq, heads).double().cpu()
        r = ref(qkv, b, seq, heads)
        d = (out - r).abs()
        print(seq, mode, "max|diff| %.3g" % d.max().item(), "rows bad", int((d.max(1).values > 1e-2).sum()),
              "cols bad", int((d.max(0).values > 1e-2).sum()), flush=True)
        if mode == "onehotV" and seq == 32:
            torch.set_printoptions(precision=3, linewidth=200)
            print("got row0", out[0, :32]); print("ref row0", r[0, :32])
