#!/bin/bash
# Side bench lines with their parity: the marker-stage pipelines at 4096^2 (against the pipeline
# digests) and config 2 (1024^2, SURVEY seed 1, against mosaic_1024x1024_s1).
# usage: scripts/gpu_sides.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sides}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
S="--batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4"
timeout -k 10 300 python bench.py --size 1024 --steps 20 $S > "$OUT/bench_1024.log" 2>&1 || exit $?
grep -v amdgpu "$OUT/bench_1024.log" | tail -1 | cut -c1-260; grep -o '"parity": "[^"]*"' "$OUT/bench_1024.log" | tail -1
for p in shape color nc; do
  timeout -k 10 400 python bench.py --pipeline $p $S > "$OUT/bench_$p.log" 2>&1 || exit $?
  grep -v amdgpu "$OUT/bench_$p.log" | tail -1 | cut -c1-200; grep -o '"parity": "[^"]*"' "$OUT/bench_$p.log" | tail -1
done
