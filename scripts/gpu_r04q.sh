# round 4: k_spec_round's LDS hot set 32 / 24 / 16 keys per lane (occupancy 2 / 2 / 3-4 waves per
# SIMD): regime probe per build
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
for v in tree q24m2 q16m3 q16m4; do
  lib=$L/libmsegment_$v.so; [ $v = tree ] && lib=$L/libmsegment.so
  MSEGMENT_LIB=$lib timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_$v.log 2>&1 || exit 1
done
echo done
