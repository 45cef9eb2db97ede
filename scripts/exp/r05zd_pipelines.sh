# Round-5 refresh of the side benches on the final kernels: config 4's 16384^2 frame on one GPU
# and the three marker-stage pipelines at 4096^2.
set -u
export TMPDIR=/tmp
O=gpurun_out/r05zd; mkdir -p $O
timeout -k 10 400 python bench.py --size 16384 --seed 3 --steps 3 --warmup 1 --batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 > $O/bench_16384.log 2>&1 || exit $?
grep -v amdgpu $O/bench_16384.log | tail -1 | cut -c1-400
for p in shape color; do
  timeout -k 10 400 python bench.py --pipeline $p --steps 3 --warmup 1 --batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 > $O/bench_$p.log 2>&1 || exit $?
  grep -v amdgpu $O/bench_$p.log | tail -1 | cut -c1-300
done
timeout -k 10 500 python bench.py --pipeline nc --batch-frames 1 --stress-steps 0 --many-frames 0 --no-hwq4 > $O/bench_nc.log 2>&1 || exit $?
grep -v amdgpu $O/bench_nc.log | tail -1 | cut -c1-300
