# Round-5 A/B of k_prep4: 6 waves per SIMD (pw6: 80 VGPRs, 5 spilled), the per-pixel logic as selects
# (pbf: 186 VGPRs, 2 waves; pbf3: capped at 3 waves), against the tree's library.  Switches
# MSEG_PREP_WPE / MSEG_PREP_BF, removed after the A/B.
set -u
export TMPDIR=/tmp
L=$PWD/opencv-msegment_amd/msegment
AB_ARGS="--stress-steps 0 --batch-frames 1 --many-frames 0 --no-hwq4" scripts/ab_kernels.sh r05t k_prep,k_resolve $L/libmsegment.so $L/libmsegment_pw6.so $L/libmsegment_pbf.so $L/libmsegment_pbf3.so
