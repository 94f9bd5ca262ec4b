"""Clock, power and temperature of the GPU while it runs the C3 bench's own
work: a child process loops the embed for ~EMB seconds, then the prefilter
ranker for ~RNK seconds, printing phase timestamps; this (parent) process
never touches the GPU and samples `rocm-smi -P -c -t --json` every ~0.5 s.
Answers: does the chip hold its clock through the trunk, or is it power /
thermal limited (then energy per FLOP, not latency hiding, sets the rate)?
usage: python tools/power_probe.py [EMB_S] [RNK_S] > out.txt"""
import json
import os
import subprocess
import sys
import time

EMB = float(sys.argv[1]) if len(sys.argv) > 1 else 12.0
RNK = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = f"""
import sys, time, numpy as np, torch
sys.path.insert(0, {R!r}); sys.path.insert(0, {R + '/tools'!r})
import bench
from research_image_retrieval_amd import ops
dev = torch.device('cuda:0'); torch.cuda.set_device(dev)
net = bench.build_extractor('resnet101', dev)
imgs = torch.from_numpy(np.random.RandomState(1234).randint(0, 256, size=(1280, 224, 224, 3), dtype=np.uint8)).to(dev)
d = net.forward_test_u8(imgs); torch.cuda.synchronize()
N = 1_600_000
gal = bench.make_gallery(N, 2048, 0, N, dev)
gbf, _ = ops.quantize_rows(gal, 'bf16'); bound = ops.prefilter_gallery_bound(gal, gbf)
lo, full = ops.ranker_workspace_bounds('prefilter', 1280, N, 2048, 100)
ws = torch.empty(max(lo, min(full, 4 << 30)), dtype=torch.uint8, device=dev)
ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=ws, max_workspace_bytes=4 << 30); torch.cuda.synchronize()
print('PHASE embed', time.time(), flush=True)
t = time.time(); n = 0
while time.time() - t < {EMB}:
    net.forward_test_u8(imgs); torch.cuda.synchronize(); n += 1
print('PHASE embed_done', time.time(), n, flush=True)
t = time.time(); n = 0
while time.time() - t < {RNK}:
    ops.cosine_topk_prefilter(d, gal, gbf, bound, 100, workspace=ws, max_workspace_bytes=4 << 30); torch.cuda.synchronize(); n += 1
print('PHASE rank_done', time.time(), n, flush=True)
"""
child = subprocess.Popen([sys.executable, "-u", "-c", CHILD], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
os.set_blocking(child.stdout.fileno(), False)
t_end = time.time() + 240
while child.poll() is None and time.time() < t_end:
    try:
        out = subprocess.run(["/opt/rocm/bin/rocm-smi", "-P", "-c", "-t", "--json"], capture_output=True, text=True,
                             timeout=10).stdout
        js = json.loads(out[out.index("{"):]) if "{" in out else {}
        card = next(iter(js.values()), {}) if js else {}
        keep = {k: v for k, v in card.items() if any(w in k.lower() for w in ("sclk", "fclk", "mclk", "power", "temperature"))}
        print(f"SAMPLE {time.time():.2f} {json.dumps(keep)}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"SAMPLE {time.time():.2f} error {e!r}", flush=True)
    try:
        for line in child.stdout:
            print(line.rstrip(), flush=True)
    except (BlockingIOError, TypeError):
        pass
    time.sleep(0.5)
if child.poll() is None:
    child.kill()
for line in child.stdout or []:
    print(line.rstrip(), flush=True)
print("child rc", child.wait(), flush=True)
