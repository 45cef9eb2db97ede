# round 4: k_spec_round at one block per CU (the new default): spec / stress / parity / batch-many
# tests, regime probe, the bench line
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04sg2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_batch_many.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || exit 1
echo done
