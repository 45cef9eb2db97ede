#!/bin/bash
# Stencil probe: event-timed sizes + rocprofv3 kernel trace of the same run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-stencil}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python scripts/stencil_probe.py > "$OUT/probe.log" 2>&1; rc=$?; cat "$OUT/probe.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python scripts/stencil_probe.py > "$OUT/rocprof.log" 2>&1; rc=$?
find "$OUT/prof" -name '*kernel_stats*' -exec cat {} \; | cut -c1-200 | head -8
exit $rc
