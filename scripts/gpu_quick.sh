#!/bin/bash
# Fast GPU iteration: parity tests + one bench line (no profiler).  usage: scripts/gpu_quick.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-quick}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) echo "STOP"; exit $rc ;; esac
timeout -k 10 600 python bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 3 "$OUT/bench.log" | cut -c1-3000
