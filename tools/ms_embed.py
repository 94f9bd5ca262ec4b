"""Experiment: the C3 extractor over B images as S concurrent chunks, one HIP
stream each (desynchronises the HBM-bound and MFMA-bound layers across CUs).
usage: ms_embed.py [B] [reps] [S...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 320
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 10
SS = [int(s) for s in sys.argv[3:]] or [1, 2, 4]
dev = torch.device("cuda:0")
net = bench.build_extractor("resnet101", dev)
rs = np.random.RandomState(1234)
imgs = torch.from_numpy(rs.randint(0, 256, size=(B, 224, 224, 3), dtype=np.uint8)).to(dev)
ref = net.forward_test_u8(imgs)
torch.cuda.synchronize()
for S in SS:
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    chunks = list(imgs.chunk(S))

    def run():
        main = torch.cuda.current_stream(dev)
        outs = []
        for s, c in zip(streams, chunks):
            s.wait_stream(main)
            with torch.cuda.stream(s):
                outs.append(net.forward_test_u8(c))
        for s in streams:
            main.wait_stream(s)
        return torch.cat(outs)

    for _ in range(2):
        out = run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        out = run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / REPS * 1e3
    d = (out - ref).abs().max().item()
    print(f"S={S}: {ms:.2f} ms per {B} images ({B / ms * 1e3:.0f} img/s), max|diff| vs S=1 {d:.2e}", flush=True)
