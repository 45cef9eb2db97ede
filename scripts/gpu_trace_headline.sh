#!/bin/bash
# Headline step under a kernel trace: where the step's time goes between kernels (idle gaps) on
# this box, plus the headline repeated to show its run-to-run spread.
# usage: scripts/gpu_trace_headline.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-trace}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --no-hwq4 --many-frames 0"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 $ARGS > "$OUT/headline_$k.log" 2>&1 || exit $?
  grep -o '"value": [0-9.]*, "unit": "Mpx/s", "n_gpus": 1, "steps": 30, "warmup": 3, "ms_per_step": [0-9.]*' "$OUT/headline_$k.log"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- python bench.py --steps 10 --warmup 3 $ARGS > "$OUT/trace.log" 2>&1 || exit $?
CSV=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
cp "$CSV" "$OUT/kernel_trace.csv"
python scripts/trace_steps.py "$OUT/kernel_trace.csv" 3 10 > "$OUT/busy.txt" 2>&1
head -40 "$OUT/busy.txt"
