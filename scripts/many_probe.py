"""The many-floods batch line of bench.py alone (bench.many_floods_line): K notConnectedMarkers
floods of SxS per batch call.  usage: python scripts/many_probe.py [K] [S] [cpu]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import json  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
import msegment  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
seg = msegment.Segmenter(0)
out = bench.many_floods_line(seg, torch.cuda.synchronize, torch.device("cuda", 0), K, S=S, cpu="cpu" in sys.argv)
print(json.dumps(out), flush=True)
seg.close()
