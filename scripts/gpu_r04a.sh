set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/spec_probe.py --oracle random_1024_s3 random_2048_s2 random_4096_s2 mosaic_noise_4096_s2 album_shape nc_mosaic_noise_1024_s2 > gpurun_out/r04a/probe.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/r04a/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r04a/bench.log 2>&1
echo rc=$?
