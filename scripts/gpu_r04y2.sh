# round 4: the speculative engine's workspace allocated at flood start for large frames: first
# flood of a fresh context against the next ones; spec / stress / parity tests
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04y2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/first_flood.py random_4096_s2 mosaic_noise_4096_s2 mosaic_4096_s2 random_1024_s3 > $O/first.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_batch_many.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
echo done
