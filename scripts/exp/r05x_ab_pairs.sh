# (applies scripts/exp/r05x_resolve_pairs.patch first; reverted after this A/B)
# Round-5 A/B of k_resolve deciding two chunks per block at once (pairs: chunks c and c + G, two
# items per thread, switch MSEG_RES_PAIRS; 128 VGPRs, 6 spilled) and of the phased gather it
# brought (tree: one chunk at a time, every item's slot / pixel words / competitors loaded in
# phases), against the committed library (head).  The parity file on both new builds (the pairs
# path runs on first runs only: its give-up test is the injected one on single chunks), then
# ab_kernels.sh.
set -u
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
for v in "" _pairs; do
  MSEGMENT_LIB=$L/libmsegment$v.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -1 $O/pytest$v.log; [ $rc -eq 0 ] || exit $rc
done
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05x k_resolve,k_commit_fast $L/libmsegment_head.so $L/libmsegment.so $L/libmsegment_pairs.so
