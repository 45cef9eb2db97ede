#!/bin/bash
# GPU suite + inflight stress without diagnostics + default bench (one gpurun call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-vf}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/tests.txt" 2>&1; rc=$?; tail -3 "$OUT/tests.txt"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u scripts/stress_inflight_dev.py 100 8 8 4096 > "$OUT/stress.txt" 2>&1; rc=$?; tail -2 "$OUT/stress.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.txt" 2>&1; rc=$?; grep -o '"value": [0-9.]*, "unit": "Mpx/s", "n_gpus"' "$OUT/bench.txt"; exit $rc
