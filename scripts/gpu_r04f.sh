# round 4: adaptive execution cap (short, long after 8 fallbacks), compacted k_spec_round:
# GPU spec/parity/stress tests, the regime probe, the cascade-pop phase split, headline A/B
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04f; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_stress.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/spec_probe.py random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2 > $O/probe.log 2>&1 || exit 1
MSEGMENT_LIB=$PWD/$L/libmsegment_specprof.so timeout -k 10 200 python -u scripts/spec_phases.py random_1024_s3 mosaic_noise_1024_s1 > $O/phases.log 2>&1 || exit 1
bash scripts/ab_bench.sh r04f/ab $L/libmsegment_old.so $L/libmsegment.so > $O/ab.log 2>&1
echo done
echo "== many-floods, serial_loop" > $O/many.log
timeout -k 10 300 python -u scripts/many_probe.py 64 1024 >> $O/many.log 2>&1 || exit 1
echo "== many-floods, ser_run" >> $O/many.log
MSEGMENT_LIB=$PWD/$L/libmsegment_multi0.so timeout -k 10 300 python -u scripts/many_probe.py 64 1024 >> $O/many.log 2>&1 || exit 1
echo done2
