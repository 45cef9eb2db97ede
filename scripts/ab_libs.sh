#!/bin/bash
# A/B of alternative builds of libmsegment on the regime probe (scripts/spec_probe.py), interleaved
# with the tree's own library.  usage: scripts/ab_libs.sh <tag> "<lib suffixes>" [frame names...]
# e.g. scripts/ab_libs.sh r05n "k1 k3" random_4096_s2  (runs libmsegment.so, _k1, _k3, libmsegment.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}; VARS=${2:-}; shift 2 || true
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
P=${*:-"random_4096_s2 mosaic_noise_4096_s2 album_shape"}
L=$PWD/opencv-msegment_amd/msegment
run() {
  local name=$1 lib=$2
  MSEGMENT_LIB=$lib timeout -k 10 300 python -u scripts/spec_probe.py $P > "$O/probe_$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"; cut -c1-220 "$O/probe_$name.log" | grep -v amdgpu.ids
  [ $rc -eq 0 ] || exit $rc
}
run base "$L/libmsegment.so"
for v in $VARS; do run "$v" "$L/libmsegment_$v.so"; done
run base2 "$L/libmsegment.so"
echo done
