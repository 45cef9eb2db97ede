# round 4: execution cap with hysteresis (long after a fallback, short again after an all-short
# generation): spec tests, the regime probe, the headline A/B against round 3
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04g; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape album_color nc_mosaic_noise_1024_s2 random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
echo "== round 3" >> $O/probe.log
MSEGMENT_LIB=$PWD/$L/libmsegment_old.so timeout -k 10 300 python -u scripts/spec_probe.py album_color nc_mosaic_noise_1024_s2 >> $O/probe.log 2>&1 || exit 1
echo done
