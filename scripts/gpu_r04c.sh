# round 4: the many-floods batch tests, then an A/B of the speculative engine's execution cap
# (MSEG_SPEC_MAXREC) against the round-3 build, then the cascade-pop phase split of both
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04d/c; mkdir -p $O
export TMPDIR=/tmp
L=opencv-msegment_amd/msegment
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch_many.py -x -q --timeout 200 > $O/pytest_many.log 2>&1
echo "many rc=$?"
F="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
echo "== old" >> $O/probe.log
MSEGMENT_LIB=$PWD/$L/libmsegment_old.so timeout -k 10 200 python -u scripts/spec_probe.py $F >> $O/probe.log 2>&1 || exit 1
for m in 256 1024 4096 8448; do
  echo "== maxrec $m" >> $O/probe.log
  MSEG_SPEC_MAXREC=$m timeout -k 10 200 python -u scripts/spec_probe.py $F >> $O/probe.log 2>&1 || exit 1
done
for v in old_specprof specprof; do
  echo "== $v" >> $O/phases.log
  MSEGMENT_LIB=$PWD/$L/libmsegment_$v.so timeout -k 10 200 python -u scripts/spec_phases.py random_1024_s3 mosaic_noise_1024_s1 >> $O/phases.log 2>&1 || exit 1
done

# config 5: the batch with each flood's commit grid a share of the chip (default) against the whole chip
for cs in 0 480; do
  echo "== commit subs $cs" >> $O/batch.log
  MSEG_BATCH_COMMIT_SUBS=$cs timeout -k 10 300 python -u bench.py --batch-only --size 4096 --kind mosaic --seed 100 --batch-frames 8 >> $O/batch.log 2>&1 || exit 1
done
echo done
