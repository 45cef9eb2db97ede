# Round-5 A/B of k_resolve (in-block LDS granules, merged granule loads, 1024-thread blocks) and
# k_prep4 (2 / 4 tile rows per block with a 2-row carry) builds against the tree's library:
# parity file on the two most changed variants, then ab_kernels.sh (headline + per-kernel means).
# (The variants were built from switches MSEG_RES_LDS / MSEG_RES_MERGE / MSEG_RBS / MSEG_PREP_ROLL that
# were removed after the A/B: lds became the default, the others were rejected; profiles/r05o_ab_resolve.log.)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
for v in ldsm p4; do
  MSEGMENT_LIB=$L/libmsegment_$v.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -3 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
AB_ARGS="--stress-steps 0 --batch-frames 1 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05o k_resolve,k_commit_fast,k_prep4 $L/libmsegment.so $L/libmsegment_lds.so $L/libmsegment_ldsm.so $L/libmsegment_lds1k.so $L/libmsegment_p2.so $L/libmsegment_p4.so
