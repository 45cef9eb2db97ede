#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
L=$PWD/opencv-msegment_amd/msegment
O=gpurun_out/r06ty; mkdir -p $O
export TMPDIR=/tmp
MSEGMENT_LIB=$L/libmsegment_ty.so timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/pytest_ty.log 2>&1 || { tail -30 $O/pytest_ty.log; exit 1; }
tail -1 $O/pytest_ty.log
bash scripts/ab_libs.sh r06ty ty --oracle album_shape nc_mosaic_noise_1024_s100 random_4096_s2 mosaic_noise_4096_s2 || exit 1
S="--batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 --correlation="
for lib in libmsegment libmsegment_ty; do
  for p in nc color; do
    MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --pipeline $p $S > $O/bench_${p}_$lib.log 2>&1 || exit 1
    echo "$lib $p $(grep -o '"value": [0-9.]*' $O/bench_${p}_$lib.log | head -1) $(grep -o '"parity": "[^"]*"' $O/bench_${p}_$lib.log | tail -1)"
  done
done
bash scripts/ab_bench.sh r06ty $L/libmsegment.so $L/libmsegment_ty.so
for lib in libmsegment libmsegment_ty; do
  echo "== regime split $lib"
  MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python scripts/regime_split.py album_shape nc_mosaic_noise_1024_s100 color_mosaic_2048_s2 > $O/split_$lib.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/split_$lib.log
done
