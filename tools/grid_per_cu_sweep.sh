#!/bin/bash
# Launch-geometry check of the K1 sweep: POW_GRID_PER_CU workgroups per CU, 5 rounds each.
#   tools/grid_per_cu_sweep.sh   (on the GPU box; tools/ab_sweep is built by __graft_entry__.build())
L=mpi_blockchain_amd/libpow_gpu_test.so  # the test build: it reads the switch below
for g in 8 4 5 6 7 8; do
  echo "grid_per_cu=$g $(POW_GRID_PER_CU=$g timeout -k 5 100 tools/ab_sweep 5 $L | tr -d '\n')"
done
