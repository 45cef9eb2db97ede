# Round-5 A/B: k_commit_fast's finalizer as block 0 (fin0, switch MSEG_CF_FIN0); k_resolve dropping
# final dependencies so later passes neither reload nor wait for them (drop, MSEG_RES_DROP: 96
# VGPRs instead of 128); drop with 256-thread blocks (5 waves per SIMD); against the tree's library.
# The parity file on each variant, then ab_kernels.sh (headline + batch, per-kernel means).
set -u
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
for v in fin0 drop drop256; do
  MSEGMENT_LIB=$L/libmsegment_$v.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -1 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05w k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_fin0.so $L/libmsegment_drop.so $L/libmsegment_drop256.so
