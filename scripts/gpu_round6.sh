#!/bin/bash
# Round-6 GPU pass: GPU tests, the default bench line (N=1), and the N > 1 path rehearsed on the
# box's one GPU (MSEG_BENCH_SHARED_GPU: 2 ranks on GPU 0, gloo collectives).  Each step has its own
# time limit; a crash / abort / timeout (rc not in {0,1}) stops the script.
# usage: scripts/gpu_round6.sh <tag> [pytest -k expression]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 6 "$OUT/$name.log" | cut -c1-1500
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit "$rc" ;; esac
}
if [ -n "$K" ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K"
else
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
[ -z "${NO_BENCH:-}" ] && run bench 600 python bench.py
[ -z "${NO_REHEARSAL:-}" ] && run bench_n2_shared 400 env MSEG_BENCH_SHARED_GPU=1 python bench.py --gpus 2 --steps 5 --warmup 2
echo "== done"
