# per-iteration kernel durations of one headline flood (rocprofv3 kernel trace)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile-pass --stress-steps 0 --batch-frames 0 --many-frames 0 --no-hwq4 > $O/bench.log 2>&1 || exit $?
f=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python scripts/trace_iters.py "$f" 1 > $O/iters.txt 2>&1
rc=$?; rm -rf $O/tr; exit $rc
