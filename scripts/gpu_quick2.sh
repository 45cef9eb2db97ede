#!/bin/bash
# GPU pass: smoke -> GPU tests (per-test time limit) -> default bench line.  Each GPU step has its
# own limit; a crash/abort/timeout stops the script.  usage: scripts/gpu_quick2.sh <tag> [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "$OUT/$name.log"
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit "$rc" ;; esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ -n "$K" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K"
else
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
fi
[ -z "${NO_BENCH:-}" ] && step bench 600 python bench.py
echo "== done"
