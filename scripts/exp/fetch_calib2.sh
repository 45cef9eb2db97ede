#!/bin/bash
# timing + EA read-request counters of scripts/exp/fetch_calib.hip (separate rocprofv3 runs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-fcal2}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/t" -o run -- ./build/exp/fetch_calib > "$OUT/t.log" 2>&1 || exit 3
find "$OUT/t" -name '*kernel_stats*' -exec cut -d, -f1-4 {} \;
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$OUT/p" -o run -- ./build/exp/fetch_calib > "$OUT/p.log" 2>&1
rc=$?; tail -3 "$OUT/p.log" | cut -c1-200
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        tot[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(tot.items()):
    print("%-12s %-24s %s" % (k[0], k[1], " ".join("%.0f" % x for x in v)))
PY
exit $rc
