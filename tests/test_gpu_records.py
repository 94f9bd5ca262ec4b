"""Batched extraction from an image-record store (records.extract_records:
same-size batches after thumbnail) equals batch-1 extraction of the same
records, in record order."""
import io

import numpy as np
import pytest
import torch
from PIL import Image

from research_image_retrieval_amd import records as R
from research_image_retrieval_amd.extract import extract_vectors
from research_image_retrieval_amd.networks import GeM

pytestmark = pytest.mark.gpu


def test_extract_records_matches_batch1(cuda):
    rs = np.random.RandomState(8)
    sizes = [(300, 400), (400, 300), (300, 400), (250, 250), (400, 300), (300, 400), (120, 90), (300, 400)]
    bufs = []
    for h, w in sizes:
        b = io.BytesIO()
        Image.fromarray(rs.randint(0, 256, size=(h, w, 3), dtype=np.uint8)).save(b, format="JPEG", quality=90)
        bufs.append(b.getvalue())
    ds = R.DistractorRecords(R.DictRecordStore(R.build_records(bufs)), imsize=320)
    net = GeM(2048, backbone="resnet50", seed=4, device=cuda)
    got = R.extract_records(net, ds, batch_size=3, device=cuda)
    ref = extract_vectors(net, [ds[i].unsqueeze(0) for i in range(len(ds))], device=cuda, print_freq=0)
    err = (got - ref).abs().max().item()
    print("records batched vs batch-1 max|err|", err)
    assert got.shape == (len(sizes), 2048) and err < 1e-6
