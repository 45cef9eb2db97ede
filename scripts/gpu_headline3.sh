#!/bin/bash
# The headline line of bench.py (no side lines) three times back to back, and the bare-loop probe
# beside it: does bench.py's timing now match the library's own per-frame time?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-h3}; mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --no-hwq4 --many-frames 0 --correlation="
for k in 1 2 3; do
  timeout -k 10 200 python bench.py $ARGS > "$OUT/headline_$k.log" 2>&1 || exit $?
  grep -o '"value": [0-9.]*, "unit": "Mpx/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' "$OUT/headline_$k.log"
done
timeout -k 10 120 python scripts/headline_spread.py 2 30 | grep -v amdgpu.ids
