#!/bin/bash
# streaming-kernel variants at three sizes + GPU tests + inflight stress (one gpurun call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-sc}; mkdir -p "$OUT"
for S in 4096 8192 16384; do bash scripts/exp/run_stream.sh ${1:-sc}_$S $S | grep -E "avg|DIFF" || exit 3; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/tests.txt" 2>&1; rc=$?; tail -3 "$OUT/tests.txt"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python -u scripts/stress_inflight_dev.py 20 8 8 4096 > "$OUT/stress.txt" 2>&1; rc=$?; tail -2 "$OUT/stress.txt"; exit $rc
