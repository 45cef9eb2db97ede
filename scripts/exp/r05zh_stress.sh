# Round-5 concurrency stress on the final kernels (k_resolve's dependency dropping changed its wait
# logic): floods of 4096^2 and 1024^2 with 8 in flight against the same frames flooded one at a
# time (4800 + 4800 floods), then the host-buffer batch against the oracle.
set -u
export TMPDIR=/tmp
O=gpurun_out/r05zh; mkdir -p $O
timeout -k 10 700 python -u scripts/stress_inflight_dev.py 600 8 8 4096 > $O/stress_inflight_4096.log 2>&1
rc=$?; echo "stress_inflight 4096 rc=$rc"; tail -1 $O/stress_inflight_4096.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/stress_inflight_dev.py 300 16 8 1024 > $O/stress_inflight_1024.log 2>&1
rc=$?; echo "stress_inflight 1024 rc=$rc"; tail -1 $O/stress_inflight_1024.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/stress_batch.py 50 8 > $O/stress_batch.log 2>&1
rc=$?; echo "stress_batch rc=$rc"; tail -1 $O/stress_batch.log; exit $rc
