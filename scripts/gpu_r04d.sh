# round 4: windowed serial pops (ser_run_w) + many-floods batch: tests, then the serial-regime
# probe with and without the window, then the spec-cap and batch-commit A/Bs (gpu_r04c.sh)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 400 python -u -m pytest tests/test_gpu_serial.py tests/test_gpu_batch_many.py -x -q --timeout 200 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -le 1 ] || exit $rc
F="album_shape album_color nc_mosaic_noise_1024_s2 random_512_s3 mosaic_noise_1024_s1"
echo "== window" >> $O/serial.log
timeout -k 10 300 python -u scripts/serial_probe.py $F >> $O/serial.log 2>&1 || exit 1
echo "== no window" >> $O/serial.log
MSEGMENT_LIB=$PWD/$L/libmsegment_nowin.so timeout -k 10 300 python -u scripts/serial_probe.py $F >> $O/serial.log 2>&1 || exit 1
bash scripts/gpu_r04c.sh
