#!/bin/bash
# A/B timing of library builds on one box: scripts/ab_bench.sh <tag> <lib1.so> <lib2.so> ... ;
# each build runs bench.py (no CPU baseline, no profile pass) twice, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 300 python bench.py ${AB_ARGS:-} --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass --stress-steps 0 --batch-frames 1 --many-frames 0 --correlation= \
      > "$OUT/$name.$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; exit $rc; }
    printf "%s rep%d %s\n" "$name" "$rep" "$(grep -o '"value": [0-9.]*' "$OUT/$name.$rep.log")"
  done
done
