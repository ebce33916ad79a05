#!/bin/bash
# K1' waves-per-SIMD sweep (tuning): time-to-block per d at each setting
L=mpi_blockchain_amd/libpow_gpu.so
for d in 13 15 17 19 21; do
  for w in 0 1 2 4 5; do
    echo "d=$d wps=$w $(POW_LAT_WPS=$w timeout -k 5 60 tools/ab_ttb $d 301 $L | tr -d '\n')"
  done
done
