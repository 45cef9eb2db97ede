#!/bin/bash
# shape pipeline bench (+ kernel trace): scripts/shape_bench.sh <tag> [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-shape}; shift || true
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --pipeline shape --steps 5 --warmup 2 "$@" > "$OUT/bench.log" 2>&1; rc=$?
tail -3 "$OUT/bench.log" | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --pipeline shape --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass "$@" > "$OUT/rocprof.log" 2>&1; rc=$?
find "$OUT/prof" -name '*kernel_stats*' -exec cp {} "$OUT/" \;
exit $rc
