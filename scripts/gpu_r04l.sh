# round 4: k_commit_fast arrival counters one per 128-B line (rocprof old vs tree), headline A/B,
# the regime probe (deep mode limited to large generations; hot-key scans 8 per LDS round trip
# against one: libmsegment_hsw1.so), the cascade phase split, and the many-floods line at 256 and
# 512 floods per call
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
PROF_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --batch-frames 1 --stress-steps 0 --no-hwq4 --many-frames 0"
for v in old new; do
  lib=$PWD/$L/libmsegment_$v.so; [ $v = new ] && lib=$PWD/$L/libmsegment.so
  MSEGMENT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python bench.py $PROF_ARGS > $O/prof_$v.log 2>&1 || exit 1
  find $O/prof_$v -name '*kernel_stats*' -exec cp {} $O/kstats_$v.csv \;
done
bash scripts/ab_bench.sh r04l $L/libmsegment_old.so $L/libmsegment.so || exit 1
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe.log 2>&1 || exit 1
MSEGMENT_LIB=$PWD/$L/libmsegment_hsw1.so timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_hsw1.log 2>&1 || exit 1
MSEGMENT_LIB=$PWD/$L/libmsegment_specprof.so timeout -k 10 300 python -u scripts/spec_phases.py random_1024_s3 mosaic_noise_1024_s1 random_4096_s2 > $O/phases.log 2>&1 || exit 1
for k in 256 512; do
  timeout -k 10 300 python -u scripts/many_probe.py $k 1024 cpu > $O/many_$k.log 2>&1 || exit 1
done
echo done
