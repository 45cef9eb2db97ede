set -u
OUT=gpurun_out/thr3; mkdir -p $OUT
for n in base r1024 r4096 r16k r1024sw8; do
  echo "== $n"
  MSEGMENT_LIB=$PWD/scripts/exp/ab/$n.so timeout -k 10 180 python -u scripts/regime_probe.py 2 > $OUT/rp_$n.log 2>&1 || { echo STOP $n; cat $OUT/rp_$n.log | tail -5; exit 1; }
  cat $OUT/rp_$n.log
done
bash scripts/ab_bench.sh thr3 scripts/exp/ab/base.so scripts/exp/ab/r4096.so
