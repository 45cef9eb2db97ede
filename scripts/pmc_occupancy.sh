#!/bin/bash
# Stall / occupancy / L2 counters of the flood kernels, one counter group per rocprofv3 run
# (kernel trace only).  usage: scripts/pmc_occupancy.sh <tag>; then scripts/pmc_table.py <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcocc}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
CGROUPS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
        "TCC_HIT_sum TCC_MISS_sum"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES")
i=0
for g in "${CGROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/g$i" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass --batch-frames 0 --stress-steps 0 --no-hwq4 --many-frames 0 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
# the per-dispatch counter files are large: keep the per-kernel table only
python scripts/pmc_table.py "$OUT" "$OUT/table.json" > "$OUT/table.txt" 2>&1 && rm -rf "$OUT"/g[0-9]*/
