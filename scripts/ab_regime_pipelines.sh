#!/bin/bash
# A/B of library builds on the serial-regime floods: the regime split of the pipelines' floods
# (scripts/regime_split.py: album.jpg shape seeds, NC seeds 1024^2, the NC and colour pipelines'
# 4096^2 floods) per build, then the regime probe with --oracle (bit-exactness) and the headline.
# usage: scripts/ab_regime_pipelines.sh <tag> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 400 python scripts/regime_split.py album_shape nc_mosaic_noise_1024_s100 nc_mosaic_4096_s2 color_mosaic_4096_s2 > "$O/split_$n.log" 2>&1 || { echo "STOP $n"; tail -5 "$O/split_$n.log"; exit 1; }
  echo "== $n"; grep -v amdgpu "$O/split_$n.log" | cut -c1-200
done
for lib in "$@"; do
  n=$(basename "$lib" .so)
  MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 400 python -u scripts/spec_probe.py --oracle album_shape nc_mosaic_noise_1024_s100 random_4096_s2 mosaic_noise_4096_s2 > "$O/probe_$n.log" 2>&1 || { echo "STOP probe $n"; exit 1; }
  echo "== probe $n"; grep -v amdgpu "$O/probe_$n.log" | sed 's/|.*|/|/' | cut -c1-160
done
