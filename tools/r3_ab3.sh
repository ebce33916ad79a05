set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_placement 500 $R/tools/ab_sweep 11 $R/abvar/p3/libpow_gpu.so $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/p3n/libpow_gpu.so $R/abvar/p6/libpow_gpu.so $R/abvar/wgq8/libpow_gpu.so
