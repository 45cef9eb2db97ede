# Round-5 A/B: k_commit_fast's finalizer loading the histogram rows in the same round trip as the
# queue state (rowse, switch MSEG_CF_ROWS_EARLY) against the tree's library: parity file on the
# variant, then ab_kernels.sh.  (MSEG_CF_DESC_EARLY -- the sub-round blocks' pass-0 descriptors
# with the rows -- needed 106 VGPRs, 42 spilled at the 2-blocks-per-CU bound: not measured.)
# (Both switches were removed after the A/B: no change, profiles/r05za_ab_commit_rows.log.)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05za; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
MSEGMENT_LIB=$L/libmsegment_rowse.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_rowse.log 2>&1
rc=$?; echo "pytest rowse rc=$rc"; tail -1 $O/pytest_rowse.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05za k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_rowse.so
