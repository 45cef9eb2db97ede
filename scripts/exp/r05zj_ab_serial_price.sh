# Round-5 A/B of the count-based regime judge's serial price (SPEC_SERIAL_TICKS, 10 ns ticks per
# serial pop: 80 in the tree; s100, s130 via the switch MSEG_SERIAL_TICKS) on the probe frames.
# (The switch was removed after the A/B: 80 kept, profiles/r05zj_ab_serial_price.log.)
set -u
scripts/ab_libs.sh r05zj "s100 s130" album_shape nc_mosaic_noise_1024_s1 random_1024_s3 random_4096_s2 mosaic_noise_4096_s2 mosaic_noise_1024_s1
