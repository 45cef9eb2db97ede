#!/bin/bash
# inflight stress (8 floods of 4096^2, GPU_MAX_HW_QUEUES=16, diag on) for the in-tree library and
# alternative builds; usage: scripts/exp/stress_ab.sh <tag> <steps> <alt .so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export GPU_MAX_HW_QUEUES=16 STRESS_DIAG=1
steps=$2; shift 2
for v in tree "$@"; do
  if [ $v = tree ]; then unset MSEGMENT_LIB; else export MSEGMENT_LIB=$PWD/$v; fi
  n=$(basename $v)
  timeout -k 10 200 python -u scripts/stress_inflight_dev.py $steps 8 8 4096 0 > "$OUT/$n.txt" 2>&1; rc=$?
  echo "$n rc=$rc: $(grep -c 'error' "$OUT/$n.txt") error lines; $(tail -1 "$OUT/$n.txt")"
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
