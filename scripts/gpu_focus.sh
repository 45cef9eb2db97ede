#!/bin/bash
# Focused GPU pass: named pytest selection (-k EXPR) then one bench line.  usage: scripts/gpu_focus.sh <tag> <-k expr> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-focus}; K=${2:-fast}; shift 2 || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 5 "$OUT/pytest_gpu.log"
case $rc in 0|1|5) ;; *) echo "STOP"; exit $rc ;; esac
if [ -n "${SPEC_PHASES:-}" ]; then
  MSEGMENT_LIB=$PWD/opencv-msegment_amd/msegment/libmsegment_specprof.so timeout -k 10 300 python scripts/spec_phases.py $SPEC_PHASES > "$OUT/spec_phases.log" 2>&1
  rc=$?; echo "spec_phases rc=$rc"; cat "$OUT/spec_phases.log" | cut -c1-400
  case $rc in 0|1) ;; *) echo "STOP"; exit $rc ;; esac
fi
timeout -k 10 600 python bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; python scripts/bench_summary.py "$OUT/bench.log"
