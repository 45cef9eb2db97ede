#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/opencv-msegment_amd/msegment
O=gpurun_out/r06om; mkdir -p $O
export TMPDIR=/tmp
MSEGMENT_LIB=$L/libmsegment_om.so timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_om.log 2>&1 || { tail -30 $O/pytest_om.log; exit 1; }
tail -1 $O/pytest_om.log
bash scripts/ab_libs.sh r06om om --oracle album_shape nc_mosaic_noise_1024_s100 random_4096_s2 mosaic_noise_4096_s2 || exit 1
S="--batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 --correlation="
for lib in libmsegment libmsegment_om; do
  for p in nc color; do
    MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --pipeline $p $S > $O/bench_${p}_$lib.log 2>&1 || exit 1
    echo "$lib $p $(grep -o '"value": [0-9.]*' $O/bench_${p}_$lib.log | head -1) $(grep -o '"parity": "[^"]*"' $O/bench_${p}_$lib.log | tail -1)"
  done
done
bash scripts/ab_many.sh r06om 1024 $L/libmsegment.so $L/libmsegment_om.so || exit 1
bash scripts/ab_bench.sh r06om $L/libmsegment.so $L/libmsegment_om.so
