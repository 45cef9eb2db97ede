#!/bin/bash
# FETCH_SIZE / WRITE-free calibration (scripts/exp/fetch_calib.hip): one --pmc pass, per-kernel averages
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-fcal}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/p" -o run -- ./build/exp/fetch_calib > "$OUT/log.txt" 2>&1
rc=$?; grep expected "$OUT/log.txt"
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        tot[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, v in tot.items():
    print("%-12s FETCH_SIZE per launch: %s KiB" % (k, " ".join("%.0f" % x for x in v)))
PY
exit $rc
