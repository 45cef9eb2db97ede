#!/bin/bash
# rocprofv3 kernel trace of build/exp/stream_variants; prints per (kernel, grid) average durations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-stream}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- ./build/exp/stream_variants ${2:-4096} > "$OUT/run.log" 2>&1
rc=$?; grep -v "^[EW]2" "$OUT/run.log" | tail -20; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    d[(r["Kernel_Name"][:60], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", ""))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
for k, v in d.items():
    v = sorted(v)[2:]  # drop the first launches' warm-up outliers
    print("%-62s grid %-9s n %3d  avg %8.2f us  min %8.2f" % (k[0], k[1], len(v), sum(v) / len(v), v[0]))
PY
