# Round-5 A/B: batches capped at one k_resolve block-round (bcap, switch MSEG_BCAP) against the
# tree's library: parity file on the variant, headline + batch (ab_kernels.sh), the 16384^2 frame.
set -u
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
MSEGMENT_LIB=$L/libmsegment_bcap.so timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_bcap.log 2>&1
rc=$?; echo "pytest bcap rc=$rc"; tail -2 $O/pytest_bcap.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05u k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_bcap.so || exit $?
for lib in libmsegment libmsegment_bcap; do
  MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python bench.py --size 16384 --seed 3 --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 > $O/big_$lib.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$O/big_$lib.log').read().strip().splitlines()[-1]); print('$lib 16384', d['value'], d['parity'])"
done
