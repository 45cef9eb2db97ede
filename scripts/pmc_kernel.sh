#!/bin/bash
# PMC counters (one group per rocprofv3 run, kernel trace only) for a short bench run.
# usage: scripts/pmc_kernel.sh <tag> "<ctr group 1>" "<ctr group 2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for ctr in "$@"; do
  name=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass > "$OUT/$name.log" 2>&1
  rc=$?; echo "$name rc=$rc"
  case $rc in 0) ;; 124|137|134|139) echo STOP; exit $rc ;; *) ;; esac
done
