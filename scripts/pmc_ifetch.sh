#!/bin/bash
# Instruction-fetch counters of the regime probe's kernels (is a round's cold start instruction
# fetch?): the counter list of this GPU, then one SQ group over one frame.
# usage: scripts/pmc_ifetch.sh <tag> <frame>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmcif}; FRAME=${2:-mosaic_noise_1024_s1}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1
grep -o "SQ_IFETCH[A-Z_]*\|SQC_ICACHE[A-Z_]*\|SQ_WAIT_INST[A-Z_]*" "$OUT/counters.txt" | sort -u > "$OUT/ifetch_counters.txt" || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY \
    --output-format csv -d "$OUT/g1" -o run -- python scripts/spec_probe.py $FRAME > "$OUT/g1.log" 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_table.py "$OUT" "$OUT/table.json" > "$OUT/table.txt" 2>&1 && rm -rf "$OUT"/g1/
