#!/bin/bash
# interleaved bench A/B (kernel averages) of the tree and an alternative build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${1:-bab}; mkdir -p "$OUT"
for v in tree alt tree alt; do
  if [ $v = alt ]; then export MSEGMENT_LIB=$PWD/$2; else unset MSEGMENT_LIB; fi
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --stress-steps 0 --batch-frames 1 > "$OUT/$v.txt" 2>&1 || exit 3
  python3 -c "
import json
for l in open('$OUT/$v.txt'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['value'], [(k['kernel'], k['avg_us']) for k in d['kernels'] if k['kernel'] in ('k_prep','k_untile')])
"
done
