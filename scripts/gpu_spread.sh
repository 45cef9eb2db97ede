#!/bin/bash
# The headline's run-to-run spread: per-process vs per-context vs per-period (scripts/headline_spread.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-spread}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout 30 rocm-smi --showclocks > "$OUT/clocks_before.txt" 2>&1
for k in 1 2 3 4; do timeout -k 10 120 python scripts/headline_spread.py 4 30 || exit $?; done 2>&1 | grep -v amdgpu.ids | tee "$OUT/spread.txt"
for k in 1 2; do timeout -k 10 120 python scripts/headline_spread.py 4 30 fresh || exit $?; done 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/spread.txt"
timeout 30 rocm-smi --showclocks > "$OUT/clocks_after.txt" 2>&1
grep -i -E "sclk|mclk|fclk" "$OUT/clocks_after.txt" | head -8
