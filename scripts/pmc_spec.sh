#!/bin/bash
# Issue / stall counters of k_spec_round on one regime-probe frame, one counter group per
# rocprofv3 run (kernel trace only).  usage: scripts/pmc_spec.sh <tag> <frame>; then
# python scripts/pmc_table.py gpurun_out/<tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcspec}; FRAME=${2:-random_4096_s2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
CGROUPS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES"
        "TCC_HIT_sum TCC_MISS_sum")
i=0
for g in "${CGROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $g --output-format csv -d "$OUT/g$i" -o run -- \
      python scripts/spec_probe.py $FRAME > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_table.py $OUT $OUT/pmc_table.json > $OUT/pmc_table.txt 2>&1
rm -rf "$OUT"/g[0-9]*/
