set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_g4 400 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/g4/libpow_gpu.so $R/abvar/v1/libpow_gpu.so
$S ttb_g4_d13 200 $R/tools/ab_ttb 13 301 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/g4/libpow_gpu.so
$S ttb_g4_d21 300 $R/tools/ab_ttb 21 201 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/g4/libpow_gpu.so
