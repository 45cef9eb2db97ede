# round 4: k_spec_round grid size A/B (MSEG_SPEC_GRID; default = every block that fits at once,
# 2 per CU): regime probe per setting
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04sg; mkdir -p $O
export TMPDIR=/tmp
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_dflt.log 2>&1 || exit 1
for g in 384 256 128; do
  MSEG_SPEC_GRID=$g timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_$g.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_dflt2.log 2>&1 || exit 1
echo done
