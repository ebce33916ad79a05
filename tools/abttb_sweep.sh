#!/bin/bash
# Dispatch-path A/B: the shipped library (hipLaunchKernel) against the test
# library with POW_AQL=1 (direct AQL dispatch) and other settings given as
# extra arguments (e.g. POW_AQL=1,POW_AQL_EXP=16); each variant in its own process, 3 alternating
# rounds: ab_ttb (time-to-block, pow_mine_any) at each d, then ab_k2.
#   tools/abttb_sweep.sh "9 13 17 21" [POW_AQL_EXP=... ...]
A=mpi_blockchain_amd/libpow_gpu.so; B=mpi_blockchain_amd/libpow_gpu_test.so
DS=${1:-"9 13"}; shift
V=("$A" "$B@POW_AQL=1")
for e in "$@"; do V+=("$B@$e"); done
for r in 1 2 3; do
  for d in $DS; do
    for v in "${V[@]}"; do timeout -k 5 60 tools/ab_ttb $d 201 "$v" || exit $?; done
  done
  for v in "${V[@]}"; do timeout -k 5 60 tools/ab_k2 5 "$v" || exit $?; done
done
