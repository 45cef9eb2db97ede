#!/bin/bash
# A/B of the serial-regime thresholds (SERIAL_RUN, SERIAL_SWITCH in ws_kernels.hip): builds
# libmsegment_<v>.so for each variant v given, on the regime probe (every frame against the
# oracle) and the NC / colour pipelines at 4096^2 (each against its digest).
# usage: scripts/ab_serial_policy.sh <tag> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=$1; shift
L=$PWD/opencv-msegment_amd/msegment
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
bash scripts/ab_libs.sh $TAG "$*" --oracle album_shape nc_mosaic_noise_1024_s100 random_4096_s2 mosaic_noise_4096_s2 || exit 1
S="--batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 --correlation="
for p in nc color; do
  for lib in libmsegment $(for v in "$@"; do echo libmsegment_$v; done); do
    MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --pipeline $p $S > $O/bench_${p}_$lib.log 2>&1 || exit 1
    echo "$lib $p $(grep -o '"value": [0-9.]*' $O/bench_${p}_$lib.log | head -1) $(grep -o '"parity": "[^"]*"' $O/bench_${p}_$lib.log | tail -1)"
  done
done
