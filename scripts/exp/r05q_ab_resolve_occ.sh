# Round-5 A/B of k_resolve occupancy: 256-thread blocks at 4 (r256), 5 (w5) and 6 (w6) waves per
# SIMD (register spills at 5 and 6), and the one-round-trip gather (nolean), against the tree's
# library.  Switches MSEG_RES_WPE / MSEG_RBS / MSEG_RES_LEAN, removed after the A/B.
set -u
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
AB_ARGS="--stress-steps 0 --batch-frames 1 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05q k_resolve,k_commit_fast $L/libmsegment.so $L/libmsegment_r256.so $L/libmsegment_w5.so $L/libmsegment_w6.so $L/libmsegment_nolean.so
