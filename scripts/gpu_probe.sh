#!/bin/bash
# Regime probe for gpurun: flood time and engine counters per frame (scripts/spec_probe.py), with
# the C oracle's time and a parity check.  usage: scripts/gpu_probe.sh <tag> [frame names...]
# Optional: PROBE_TESTS="<pytest files>" runs those GPU tests first; PROBE_PREV=1 repeats the probe
# on opencv-msegment_amd/msegment/libmsegment_prev.so (an A/B against the previous build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-probe}; shift || true
O=gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
P=${*:-"album_shape nc_mosaic_noise_1024_s1 random_1024_s3 mosaic_noise_1024_s1 random_4096_s2 mosaic_noise_4096_s2"}
L=$PWD/opencv-msegment_amd/msegment
if [ -n "${PROBE_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PROBE_TESTS -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python -u scripts/spec_probe.py --oracle $P > "$O/probe.log" 2>&1
rc=$?; echo "probe rc=$rc"; cut -c1-400 "$O/probe.log"; [ $rc -eq 0 ] || exit $rc
if [ -n "${PROBE_PREV:-}" ]; then
  MSEGMENT_LIB=$L/libmsegment_prev.so timeout -k 10 500 python -u scripts/spec_probe.py $P > "$O/probe_prev.log" 2>&1
  rc=$?; echo "probe_prev rc=$rc"; cut -c1-400 "$O/probe_prev.log"; [ $rc -eq 0 ] || exit $rc
fi
echo done
