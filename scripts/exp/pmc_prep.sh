#!/bin/bash
# one rocprofv3 SQ-counter pass over a short bench run (kernel trace only), per-kernel sums
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-pmcp}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH} --output-format csv -d "$OUT/p" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass --stress-steps 0 --batch-frames 1 > "$OUT/log.txt" 2>&1
rc=$?; echo rc=$rc
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
f = glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True)
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for fn in f:
    for r in csv.DictReader(open(fn)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("msg::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in tot.items():
    if any(x in k for x in ("k_prep", "k_resolve", "k_scatter", "k_untile", "k_scan")):
        print(k[:30], {c: "%.3g" % v for c, v in sorted(d.items())})
PY
exit $rc
