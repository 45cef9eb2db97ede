# round 4: deep mode toggled off by a second cooldown (regime probe), the many-floods line at 1024
# floods per call
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/many_probe.py 1024 1024 cpu > $O/many_1024.log 2>&1 || exit 1
echo done
