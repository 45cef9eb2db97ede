set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r03r
L=opencv-msegment_amd/msegment
MSEGMENT_LIB=$(realpath $L/libmsegment_cf3.so) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03r/pytest_cf3.log 2>&1; rc=$?; echo "pytest cf3 rc=$rc"; tail -3 gpurun_out/r03r/pytest_cf3.log
case $rc in 0|1) ;; *) exit $rc ;; esac
AB_ARGS="--stress-steps 0 --batch-frames 1 --no-hwq4" scripts/ab_kernels.sh r03r k_commit_fast,k_resolve,k_prep $L/libmsegment_base.so $L/libmsegment_cf3.so
