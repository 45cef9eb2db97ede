# round 4: deep-mode A/B -- MSEG_SPEC_DEEPREC (cap of non-head executions in deep mode) and
# MSEG_SPEC_DEEPCOOL=0 (no cooldown on entering deep mode), regime probe per setting
# (both knobs were removed after this A/B: profiles/r04v_ab_deep_mode.log)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
P="random_1024_s3 mosaic_noise_1024_s1 album_shape random_4096_s2 mosaic_noise_4096_s2"
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u scripts/spec_probe.py $P > $O/probe_$tag.log 2>&1; }
run base MSEG_SPEC_DEEPCOOL=1 || exit 1
run nocool MSEG_SPEC_DEEPCOOL=0 || exit 1
run dr2048 MSEG_SPEC_DEEPREC=2048 || exit 1
run dr1024 MSEG_SPEC_DEEPREC=1024 || exit 1
run nocool_dr2048 MSEG_SPEC_DEEPCOOL=0 MSEG_SPEC_DEEPREC=2048 || exit 1
run base2 MSEG_SPEC_DEEPCOOL=1 || exit 1
echo done
