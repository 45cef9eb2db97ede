# round 4: the execution cap with fallback generations left out of the regime judge, and the
# many-floods bench line (64 notConnectedMarkers floods per call)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
F="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
for m in 256 512 1024; do
  echo "== maxrec $m" >> $O/probe.log
  MSEG_SPEC_MAXREC=$m timeout -k 10 200 python -u scripts/spec_probe.py $F >> $O/probe.log 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --batch-frames 1 --stress-steps 0 --no-hwq4 --no-profile-pass > $O/bench_many.log 2>&1
echo "bench rc=$?"
