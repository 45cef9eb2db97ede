#!/bin/bash
# A/B of library builds with the profile pass on: value + per-kernel avg.  usage: scripts/ab_kernels.sh <tag> <kernel> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    MSEGMENT_LIB=$(realpath "$lib") timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${AB_ARGS:-} > "$OUT/$name.$rep.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "STOP $name rc=$rc"; tail -3 "$OUT/$name.$rep.log"; exit $rc; }
    python - "$OUT/$name.$rep.log" "$name" "$rep" "$K" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {x["kernel"]: x["avg_us"] for x in d["kernels"]}
print("%-14s rep%s value %9.2f  %s  parity %s" % (sys.argv[2], sys.argv[3], d["value"],
      "  ".join("%s %s us" % (k, ks.get(k)) for k in sys.argv[4].split(",")), d["parity"]))
PY
  done
done
