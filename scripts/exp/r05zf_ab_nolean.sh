# Round-5 A/B: k_resolve's radius-2 gather in one round trip (nolean, switch MSEG_RES_LEAN=false)
# on top of the dependency dropping, against the tree's library.
# (The switch was removed after the A/B: flat, profiles/r05zf_ab_nolean.log.)
set -u
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05zf k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_nolean.so
