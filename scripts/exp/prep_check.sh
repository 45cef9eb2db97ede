#!/bin/bash
# parity tests + bench kernel times + one WRITE_SIZE pass (k_prep work)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-pc}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > "$OUT/t.txt" 2>&1; rc=$?; tail -2 "$OUT/t.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stress-steps 0 --batch-frames 1 > "$OUT/b.txt" 2>&1 || exit 4
python3 -c "
import json
for l in open('$OUT/b.txt'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], [(k['kernel'], k['avg_us']) for k in d['kernels']])
"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/p" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass --stress-steps 0 --batch-frames 1 > "$OUT/p.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(list)
for fn in glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].split()[-1]
        if "prep" in k or "untile" in k: tot[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(tot.items()):
    print(k, "%.1f MB avg" % (sum(v) / len(v) * 1024 / 1e6))
PY
