# Round-5 A/B: the serial loop (cv::watershed's own pops, in k_scan and k_serial_multi) resolving
# a popped slot from the wave's last 64 pushes or the previous bucket's ring before loading the
# queue (pcache, switch MSEG_SER_PCACHE), against the tree's library: the serial-regime GPU tests
# on the variant, the regime probe (album.jpg, NC 1024^2, random 1024^2) and 64 / 256 many floods.
set -u
# (The switch was removed after the A/B: slower, profiles/r05zg_ab_serial_push_cache.log.)
export TMPDIR=/tmp
O=gpurun_out/r05zg; mkdir -p $O
L=$PWD/opencv-msegment_amd/msegment
MSEGMENT_LIB=$L/libmsegment_pcache.so timeout -k 10 600 python -u -m pytest tests/test_gpu_batch_many.py tests/test_gpu_spec.py tests/test_gpu_real.py tests/test_gpu_parity.py -x -q -k "not 2_28" --timeout 120 --timeout-method thread > $O/pytest_pcache.log 2>&1
rc=$?; echo "pytest pcache rc=$rc"; tail -1 $O/pytest_pcache.log; [ $rc -eq 0 ] || exit $rc
scripts/ab_libs.sh r05zg "pcache" album_shape nc_mosaic_noise_1024_s1 random_1024_s3 || exit $?
for lib in libmsegment libmsegment_pcache libmsegment libmsegment_pcache; do
  MSEGMENT_LIB=$L/$lib.so timeout -k 10 300 python scripts/many_probe.py 256 1024 > $O/many_$lib.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$O/many_$lib.log').read().strip().splitlines()[-1]); print('$lib many 256', d['value'], d['ms_per_step'])"
done
