#!/bin/bash
# r06c: GPU tests, the correlation line alone, then the headline trace and the side lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06c
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 4 "$OUT/pytest_gpu.log"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py --steps 3 --batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 > "$OUT/bench_corr.log" 2>&1 || exit $?
python -c "
import json; d=json.loads([l for l in open('$OUT/bench_corr.log') if l.startswith('{')][-1])
print(json.dumps(d['correlation'], indent=0)[:3000])"
bash scripts/gpu_trace_headline.sh r06c || exit $?
bash scripts/gpu_sides.sh r06c
