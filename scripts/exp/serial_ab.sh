#!/bin/bash
# serial-loop A/B: spec_check on the album frames (flood times) for the tree and a base build,
# then the GPU parity / spec / stress tests on the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-sab}; mkdir -p "$OUT"
for v in tree base tree base; do
  if [ $v = base ]; then export MSEGMENT_LIB=$PWD/build/ab/libmsegment_base.so; else unset MSEGMENT_LIB; fi
  timeout -k 10 200 python -u scripts/spec_check.py album > "$OUT/$v.txt" 2>&1; rc=$?
  echo "== $v rc=$rc"; grep -iE "album|ms" "$OUT/$v.txt" | tail -4
  [ $rc -eq 0 ] || exit $rc
done
unset MSEGMENT_LIB
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_stress.py > "$OUT/t.txt" 2>&1; rc=$?; tail -2 "$OUT/t.txt"; exit $rc
