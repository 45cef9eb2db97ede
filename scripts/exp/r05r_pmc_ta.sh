# Address-path counters of the headline flood's kernels (is k_resolve bound by the per-CU
# texture-address / L1 path of its scattered loads?): one counter group per rocprofv3 run.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05r; mkdir -p "$OUT"
CGROUPS=("GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max TA_ADDR_STALLED_BY_TC_CYCLES_sum"
        "GRBM_GUI_ACTIVE TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum"
        "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
        "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS")
i=0
for g in "${CGROUPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$OUT/g$i" -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass --batch-frames 0 --stress-steps 0 --no-hwq4 --many-frames 0 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_table.py "$OUT" "$OUT/table.json" > "$OUT/table.txt" 2>&1 && rm -rf "$OUT"/g[0-9]*/
