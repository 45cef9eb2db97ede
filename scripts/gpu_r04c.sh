# round 4: A/B of the speculative engine's cascade spill against the round-3 build
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_many.py -x -q --timeout 200 > $O/pytest_many.log 2>&1
echo "many rc=$?"
for v in old default minb1 nospill; do
  lib=$L/libmsegment_$v.so; [ $v = default ] && lib=$L/libmsegment.so
  echo "== $v" >> $O/probe.log
  MSEGMENT_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 random_4096_s2 mosaic_noise_4096_s2 >> $O/probe.log 2>&1 || exit 1
done
for v in old_specprof specprof; do
  echo "== $v" >> $O/phases.log
  MSEGMENT_LIB=$PWD/$L/libmsegment_$v.so timeout -k 10 200 python -u scripts/spec_phases.py random_1024_s3 mosaic_noise_1024_s1 mosaic_noise_4096_s2 >> $O/phases.log 2>&1 || exit 1
done
echo done
