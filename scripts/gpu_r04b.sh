# round 4: unbounded speculative cascades (cold pool) -- spec tests, then the regime probe
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py -x -q --timeout 300 > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/spec_probe.py --oracle random_1024_s3 random_2048_s2 random_4096_s2 mosaic_noise_4096_s2 album_shape nc_mosaic_noise_1024_s2 > $O/probe.log 2>&1
echo rc=$?
