#!/bin/bash
# A/B of an alternative library build against a base build on one box: the GPU test suite on the
# variant, then scripts/ab_kernels.sh (headline bench, per-kernel averages, interleaved, two
# repetitions) and scripts/regime_probe.py (album / mosaic+noise / random floods vs the C oracle)
# for both.  usage: scripts/ab_variant.sh <tag> <variant.so> <base.so> [kernels]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; VAR=$2; BASE=$3; K=${4:-k_commit_fast,k_resolve,k_scan}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
MSEGMENT_LIB=$(realpath "$VAR") timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_variant.log" 2>&1
rc=$?; echo "pytest variant rc=$rc"; tail -3 "$OUT/pytest_variant.log"
case $rc in 0|1) ;; *) exit $rc ;; esac
AB_ARGS="--stress-steps 0 --batch-frames 1 --no-hwq4" scripts/ab_kernels.sh "$TAG" "$K" "$BASE" "$VAR" || exit $?
for lib in "$BASE" "$VAR"; do
  name=$(basename "$lib" .so)
  MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 200 python scripts/regime_probe.py 1 > "$OUT/regime_$name.log" 2>&1
  rc=$?; echo "regime $name rc=$rc"; grep -v amdgpu.ids "$OUT/regime_$name.log"
  [ $rc -eq 0 ] || exit $rc
done
