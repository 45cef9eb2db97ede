# round 4: deep mode switched off only when it ran no faster per pop than the span before it.
# Spec tests, regime probe (tree and previous commit), and the same probe under rocprofv3's kernel
# trace (a slower clock for the time-based regime judge) for both builds
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04x; mkdir -p $O
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_stress.py -x -q --timeout 300 > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe.log 2>&1 || exit 1
MSEGMENT_LIB=$L/libmsegment_prev.so timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_prev.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u scripts/spec_probe.py random_4096_s2 album_shape > $O/probe_rocprof.log 2>&1 || exit 1
MSEGMENT_LIB=$L/libmsegment_prev.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_prev -o run -- python -u scripts/spec_probe.py random_4096_s2 album_shape > $O/probe_rocprof_prev.log 2>&1 || exit 1
rm -f $O/prof/run_kernel_trace.csv $O/prof_prev/run_kernel_trace.csv
echo done
