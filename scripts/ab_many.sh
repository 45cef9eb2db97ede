#!/bin/bash
# A/B of library builds on the many-floods kernel: K notConnectedMarkers floods of 1024^2 per call
# (scripts/many_probe.py, every frame checked against the C oracle), builds interleaved twice.
# usage: scripts/ab_many.sh <tag> <K> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 300 python scripts/many_probe.py "$K" 1024 cpu > "$OUT/$name.$K.$rep.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; tail -3 "$OUT/$name.$K.$rep.log"; exit $rc; }
    python - "$OUT/$name.$K.$rep.log" "$name" "$rep" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "rep", sys.argv[3], d["value"], "Mpx/s", d["ms_per_step"], "ms", d.get("parity"))
PY
  done
done
