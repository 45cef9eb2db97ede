#!/bin/bash
# A/B of serial_loop's calm-cascade exit: flood times (spec_check) for the tree and alternative builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-sea}; mkdir -p "$OUT"; shift
for v in tree "$@"; do
  if [ $v = tree ]; then unset MSEGMENT_LIB; else export MSEGMENT_LIB=$PWD/$v; fi
  n=$(basename $v .so)
  timeout -k 10 300 python -u scripts/spec_check.py nc_mosaic_1024_s2 nc_mosaic_noise_1024_s2 mosaic_noise_1024_s1 random_512_s3 > "$OUT/$n.txt" 2>&1 || exit 3
  timeout -k 10 200 python -u scripts/spec_check.py album >> "$OUT/$n.txt" 2>&1 || exit 4
  echo "== $n"; grep "|" "$OUT/$n.txt" | sed -E 's/ +gens.*\| spec=0/ | spec=0/' | cut -c1-120
done
