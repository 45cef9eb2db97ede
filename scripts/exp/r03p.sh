set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r03p
export TMPDIR=/tmp
timeout -k 10 300 python scripts/regime_probe.py > gpurun_out/r03p/regime_probe.log 2>&1; rc=$?; echo "regime rc=$rc"; cat gpurun_out/r03p/regime_probe.log
case $rc in 0|1) ;; *) exit $rc ;; esac
PROF_ONLY=1 STRESS_PROF=1 bash scripts/gpu_check.sh r03p || exit $?
timeout -k 10 400 python bench.py --pipeline nc > gpurun_out/r03p/bench_nc.log 2>&1; rc=$?; echo "nc rc=$rc"; tail -c 600 gpurun_out/r03p/bench_nc.log
