# round 4: execution cap policy 7 (the head long; all from round 2 once generations run deep),
# Ctl layout (k_commit_fast arrivals on their own line): tests, regime probe, headline A/B
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py tests/test_gpu_parity.py tests/test_gpu_batch_many.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape album_color nc_mosaic_noise_1024_s2 random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
bash scripts/ab_bench.sh r04i/ab $L/libmsegment_old.so $L/libmsegment.so > $O/ab.log 2>&1
echo done
