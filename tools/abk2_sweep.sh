#!/bin/bash
# ab_k2 per variant in its own process, 3 alternating rounds (one context per process)
A=mpi_blockchain_amd/libpow_gpu.so; B=mpi_blockchain_amd/libpow_gpu_test.so
for r in 1 2 3; do
  for v in "$A" "$B@POW_NO_AQL=1" "$B@POW_AQL_EXP=32" "$B@POW_AQL_EXP=33" "$B@POW_AQL_EXP=4" "$B@POW_AQL_EXP=2"; do
    timeout -k 5 60 tools/ab_k2 5 "$v" || exit $?
  done
done
