# Round-5 A/B: k_resolve sleeping s_sleep(N) (64 N cycles) before each re-poll of its pending
# dependencies (switch MSEG_RES_NAP = 4 / 16 / 48), against the tree's library.
# (The switch was removed after the A/B: slower at every N, profiles/r05zk_ab_nap.log.)
set -u
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
AB_ARGS="--stress-steps 0 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05zk k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_nap4.so $L/libmsegment_nap16.so $L/libmsegment_nap48.so
