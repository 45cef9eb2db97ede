# round 4: headline bisect (round 3, the two round-4 commits, the tree) and the regime probe with
# the deep-generation criterion fixed
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
bash scripts/ab_bench.sh r04j/ab $L/libmsegment_old.so $L/libmsegment_05dc754.so $L/libmsegment_7d80a47.so $L/libmsegment.so > $O/ab.log 2>&1
echo done
