#!/bin/bash
# GPU validation pass for gpurun: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/abort/timeout (rc not in {0,1}) stops the script.
# usage: scripts/gpu_check.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 8 "$OUT/$name.log"
  case $rc in 0|1|5) return 0 ;; *) echo "STOP after $name (rc=$rc)"; exit "$rc" ;; esac
}
if [ -z "${PROF_ONLY:-}" ]; then
  run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
  run pytest_gpu 900 python -m pytest tests -m gpu -x -q
  run bench 600 python bench.py "$@"
  [ -n "${EXTRA_BENCH:-}" ] && run bench_extra 600 python bench.py $EXTRA_BENCH
fi
# the profiled command is the headline's single-flood path only (--batch-frames 1: no concurrent
# floods, whose overlapping kernels would inflate the per-launch durations and traffic)
PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --no-hwq4 --many-frames 0 --correlation="
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py $PROF_ARGS
find "$OUT/prof" -name '*stats*' -exec cp {} "$OUT/" \; 2>/dev/null
# HBM traffic: one counter group per rocprofv3 run, kernel trace only (MI355X_MICROARCH.md)
for ctr in FETCH_SIZE WRITE_SIZE; do
  run pmc_$ctr 600 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$ctr" -o run -- python bench.py $PROF_ARGS
done
# the library these counters (and the bench line) come from, for the PMC files' notes
BID=$(python -c "import sys; sys.path.insert(0, 'opencv-msegment_amd'); from msegment import _lib; print(_lib.load().msg_build_id().decode())")
python scripts/pmc_summary.py "$OUT" "$OUT/pmc_latest.json" "$TAG, libmsegment build $BID; single-flood command" $PROF_ARGS > "$OUT/pmc_summary.log" 2>&1
# the config-3 stress variants (speculative engine, serial pops): kernel stats and HBM traffic
if [ -n "${STRESS_PROF:-}" ]; then
  for kind in mosaic_noise random; do
    SARGS="--kind $kind --steps 1 --warmup 1 --no-cpu-baseline --no-profile-pass --batch-frames 0 --stress-steps 0 --no-hwq4 --many-frames 0 --correlation="
    run rocprof_$kind 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$kind" -o run -- python bench.py $SARGS
    find "$OUT/prof_$kind" -name '*kernel_stats*' -exec cp {} "$OUT/${kind}_kernel_stats.csv" \; 2>/dev/null
    for ctr in FETCH_SIZE WRITE_SIZE; do
      run pmc_${kind}_$ctr 900 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$kind/pmc_$ctr" -o run -- python bench.py $SARGS
    done
    python scripts/pmc_summary.py "$OUT/pmc_$kind" "$OUT/pmc_stress_$kind.json" \
      "$TAG, libmsegment build $BID: config-3 stress variant $kind as the main step" $SARGS > "$OUT/pmc_summary_$kind.log" 2>&1
  done
fi
echo "== done"
