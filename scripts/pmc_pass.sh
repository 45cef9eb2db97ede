#!/bin/bash
# Separate rocprofv3 PMC passes (one counter group per run, kernel-trace only; no sys/runtime
# tracing) over a short bench run.  usage: scripts/pmc_pass.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $ctr | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/$name" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass > "$OUT/$name.log" 2>&1
  rc=$?; echo "$name rc=$rc"
  case $rc in 0) ;; *) echo STOP; exit $rc ;; esac
done
