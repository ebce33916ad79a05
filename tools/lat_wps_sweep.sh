#!/bin/bash
# K1' waves-per-SIMD sweep (tuning of the pow_mine[_any] sub-round plan):
# time-to-block per difficulty with POW_LAT_WPS forcing 1/2/4/5 waves per SIMD (0 = the plan).
#   gcc -O2 -I include tools/ab_ttb.c -ldl -o tools/ab_ttb && tools/lat_wps_sweep.sh   (on the GPU box)
L=mpi_blockchain_amd/libpow_gpu_test.so  # the test build: it reads the switch below
for d in 13 15 17 19 21; do
  for w in 0 1 2 4 5; do
    echo "d=$d wps=$w $(POW_LAT_WPS=$w timeout -k 5 60 tools/ab_ttb $d 301 $L | tr -d '\n')"
  done
done
