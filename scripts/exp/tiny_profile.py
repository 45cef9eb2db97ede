"""Experiment (MSEGMENT_LIB=scripts/exp/libmsegment_tinyprof.so): s_memtime phase split of the
one-wave tiny-batch loop on the real photograph's flood.  diag[0..6] = gather (incl. load
latency), resolve rounds, cut words, wave_rank, commit stores, tails, batch formation."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

import msegment  # noqa: E402

rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
img = np.ascontiguousarray(rgb[..., ::-1])
H, W = img.shape[:2]
dev = torch.device("cuda", 0)
seg = msegment.Segmenter(0)
t = torch.from_numpy(img).to(dev)
mk = torch.empty((H, W), dtype=torch.int32, device=dev)
lab = torch.empty_like(mk)
d, n = seg.shape_markers_dev(t, mk)
seg.set_diag(True)
seg.watershed_dev(t, mk, lab)
torch.cuda.synchronize()
st = seg.stats()
names = ["gather", "resolve", "cuts", "wave_rank", "commit", "tails", "form_batch"]
b = st["batches"]
print("batches", b, "pops", st["pops"])
for k, nm in enumerate(names):
    print("%-10s %10.0f cycles/batch" % (nm, st["diag"][k] / max(b, 1)))
