#!/bin/bash
# Dispatch-path A/B, each variant in its own process, alternating rounds:
# ab_ttb (time-to-block, pow_mine_any) at d = 9 and 13, then ab_k2 (pow_hash_block).
A=mpi_blockchain_amd/libpow_gpu.so; B=mpi_blockchain_amd/libpow_gpu_test.so
V=("$A" "$B@POW_NO_AQL=1" "$B@POW_AQL_EXP=128" "$B@POW_AQL_EXP=384" "$B@POW_AQL_EXP=640" "$B@POW_AQL_EXP=512")
for r in 1 2 3; do
  for d in 9 13; do
    for v in "${V[@]}"; do timeout -k 5 60 tools/ab_ttb $d 201 "$v" || exit $?; done
  done
  for v in "${V[@]}"; do timeout -k 5 60 tools/ab_k2 5 "$v" || exit $?; done
done
