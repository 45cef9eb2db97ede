# round 4: when executions may run long (MSEG_SPEC_CAPMODE A/B), and the headline A/B
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
F="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
for m in 0 1 2 3 4 5; do
  echo "== capmode $m" >> $O/probe.log
  MSEG_SPEC_CAPMODE=$m timeout -k 10 300 python -u scripts/spec_probe.py $F >> $O/probe.log 2>&1 || exit 1
done
bash scripts/ab_bench.sh r04h/ab $L/libmsegment_old.so $L/libmsegment.so > $O/ab.log 2>&1
echo done
