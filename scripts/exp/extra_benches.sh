#!/bin/bash
# round-end extra bench lines: config 4 frame on one GPU, the NC and shape pipelines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-xb}; mkdir -p "$OUT"
timeout -k 10 400 python bench.py --size 16384 --seed 3 --stress-steps 0 --batch-frames 1 > "$OUT/c4.txt" 2>&1; echo "c4 rc=$?"; grep -o '"value": [0-9.]*' "$OUT/c4.txt" | head -1
timeout -k 10 400 python bench.py --pipeline shape --stress-steps 0 > "$OUT/shape.txt" 2>&1; echo "shape rc=$?"; grep -o '"value": [0-9.]*' "$OUT/shape.txt" | head -1
timeout -k 10 500 python bench.py --pipeline nc --stress-steps 0 > "$OUT/nc.txt" 2>&1; echo "nc rc=$?"; grep -o '"value": [0-9.]*' "$OUT/nc.txt" | head -1
