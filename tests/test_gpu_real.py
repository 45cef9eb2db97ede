"""GPU parity on a real photograph: the reference's own resource image album.jpg (1500x1500,
decoded pixels in tests/golden/album_1500x1500.png) through the SHAPE_METHOD seed stage and the
exact flood -- the interrupt-dense regime real images put the flood in -- bit-exact
against the oracles."""
import os

import numpy as np
import pytest

from oracle import shape_oracle as so
from oracle import ws_oracle

pytestmark = pytest.mark.gpu

PNG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "album_1500x1500.png")


def test_album_shape_stage_and_flood(seg):
    import torch
    from PIL import Image

    rgb = np.asarray(Image.open(PNG).convert("RGB"))
    img = np.ascontiguousarray(rgb[..., ::-1])
    H, W = img.shape[:2]
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(img).to(dev)
    mk = torch.empty((H, W), dtype=torch.int32, device=dev)
    depth, ncomp = seg.shape_markers_dev(t, mk)
    want = so.shape_stages(img)
    assert (depth, ncomp) == (want["depth"], want["ncomp"])
    assert np.array_equal(mk.cpu().numpy(), want["markers"])
    lab = torch.empty_like(mk)
    seg.watershed_dev(t, mk, lab)
    torch.cuda.synchronize()
    assert np.array_equal(lab.cpu().numpy(), ws_oracle.watershed(img, want["markers"]))
