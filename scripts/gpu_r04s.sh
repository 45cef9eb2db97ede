# round 4: k_spec_round's per-record loops (promotion, replays, log copy, change marks) load 8
# records per round trip.  Spec / stress / parity tests, regime probe against the previous commit
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py tests/test_gpu_parity.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe.log 2>&1 || exit 1
MSEGMENT_LIB=$PWD/$L/libmsegment_prev.so timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_prev.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe2.log 2>&1 || exit 1
echo done
