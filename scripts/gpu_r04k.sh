# round 4: which kernel the headline regression is in (rocprof stats, round-3 build vs the tree),
# and the regime probe with the cooldown-triggered deep mode
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --no-hwq4 --many-frames 0"
for v in old new; do
  lib=$PWD/$L/libmsegment_$v.so; [ $v = new ] && lib=$PWD/$L/libmsegment.so
  MSEGMENT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py $PROF_ARGS > $O/prof_$v.log 2>&1 || exit 1
  find $O/prof_$v -name '*kernel_stats*' -exec cp {} $O/kstats_$v.csv \;
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
echo done
