# Round-5 A/B: merged granule loads (label and push dependencies in one round trip per pass,
# switch MSEG_RES_MERGE) on top of the dependency dropping (no spills now: 119 VGPRs), against the
# tree's library.  The parity and spec test files on the variant, then ab_kernels.sh.
# (The switch was removed after the A/B: rejected, profiles/r05y_ab_merge.log.)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
MSEGMENT_LIB=$L/libmsegment_merge.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_merge.log 2>&1
rc=$?; echo "pytest merge rc=$rc"; tail -1 $O/pytest_merge.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05y k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_merge.so
