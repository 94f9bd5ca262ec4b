"""Determinism: the filter epilogues append survivors with
atomics, so the candidate order differs from run to run; the selected top-k
must not.  Every ranker, rerun on the same inputs, returns bit-identical
scores and indices; the extractor returns bit-identical descriptors.  Also
runs librr's C-ABI under the host-ASan build on the device
(tests/asan/abi_check gpu)."""
import os
import subprocess

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from research_image_retrieval_amd import ops
from research_image_retrieval_amd.networks import GeM

pytestmark = pytest.mark.gpu


def _clustered(n, d, centres, seed):
    """Landmark-like gallery: rows jittered around few centres, so many rows
    land near each query's threshold and many survivors are appended."""
    g = torch.Generator().manual_seed(seed)
    c = F.normalize(torch.randn(centres, d, generator=g), dim=1)
    rows = c[torch.randint(0, centres, (n,), generator=g)] + 0.2 * torch.randn(n, d, generator=g) / d ** 0.5
    return F.normalize(rows, dim=1), c


@pytest.mark.parametrize("ranker", ["exhaustive", "prefilter", "bf16", "fp8"])
def test_ranker_reruns_bit_identical(cuda, ranker):
    gal, c = _clustered(300_000, 256, 50, 3)
    g = gal.to(cuda)
    q = F.normalize(c[:40] + 0.05 * torch.randn(40, 256), dim=1).to(cuda)
    outs = []
    for _ in range(3):
        if ranker == "exhaustive":
            s, i = ops.cosine_topk(q, g, 100)
        elif ranker == "prefilter":
            gb, _ = ops.quantize_rows(g, "bf16")
            s, i = ops.cosine_topk_prefilter(q, g, gb, ops.prefilter_gallery_bound(g, gb), 100)
        else:
            gl, gs = ops.quantize_rows(g, ranker)
            ql, qs = ops.quantize_rows(q, ranker)
            s, i = ops.cosine_topk_lp(ql, qs, gl, gs, 100, ranker)
        outs.append((s.cpu(), i.cpu()))
    for s, i in outs[1:]:
        assert torch.equal(i, outs[0][1]) and torch.equal(s.view(torch.int32), outs[0][0].view(torch.int32))


def test_extractor_reruns_bit_identical(cuda):
    net = GeM(2048, backbone="resnet50", seed=2, device=cuda)
    rs = np.random.RandomState(9)
    img = torch.from_numpy(rs.randint(0, 256, size=(24, 96, 96, 3), dtype=np.uint8)).to(cuda)
    a = net.forward_test_u8(img)
    b = net.forward_test_u8(img)
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))


def test_abi_under_host_asan_on_device(cuda):
    """The ASan build (host code instrumented, device code unchanged) through a
    real handle: argument validation of every entry, workspace checks, small
    device calls (tests/asan/abi_check.cpp)."""
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "asan", "out", "abi_check")
    if not os.path.exists(exe):
        pytest.fail("tests/asan/out/abi_check missing: run `bash tests/asan/build.sh` before the GPU tests")
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert r.returncode == 0 and "abi_check gpu: ok" in out and "AddressSanitizer" not in out
