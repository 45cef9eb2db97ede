# round 4: the top pop's gather through plain loads (libmsegment.so) against agent-scope loads
# (libmsegment_gag.so): spec / stress / parity tests, regime probe and the diag split per build
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py tests/test_gpu_parity.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
for v in tree gag tree2; do
  lib=$PWD/$L/libmsegment_$v.so; [ $v != gag ] && lib=$PWD/$L/libmsegment.so
  MSEGMENT_LIB=$lib timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_$v.log 2>&1 || exit 1
done
for v in tree gag; do
  lib=$PWD/$L/libmsegment_$v.so; [ $v != gag ] && lib=$PWD/$L/libmsegment.so
  MSEGMENT_LIB=$lib timeout -k 10 300 python -u scripts/spec_diag.py mosaic_noise_1024_s1 mosaic_noise_4096_s2 > $O/diag_$v.log 2>&1 || exit 1
done
echo done
