set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r03x
L=opencv-msegment_amd/msegment
MSEGMENT_LIB=$(realpath $L/libmsegment_ctot.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03x/pytest_ctot.log 2>&1; rc=$?; echo "pytest wr rc=$rc"; tail -3 gpurun_out/r03x/pytest_ctot.log
case $rc in 0|1) ;; *) exit $rc ;; esac
AB_ARGS="--stress-steps 0 --batch-frames 1 --no-hwq4" scripts/ab_kernels.sh r03x k_commit_fast,k_resolve,k_scan $L/libmsegment_base.so $L/libmsegment_ctot.so || exit $?
for lib in base ctot; do MSEGMENT_LIB=$(realpath $L/libmsegment_$lib.so) timeout -k 10 200 python scripts/regime_probe.py 1 > gpurun_out/r03x/regime_$lib.log 2>&1; echo "regime $lib rc=$?"; grep -v amdgpu.ids gpurun_out/r03x/regime_$lib.log; done
