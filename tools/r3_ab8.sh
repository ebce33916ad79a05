set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_c0 400 $R/tools/ab_sweep 11 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/c0/libpow_gpu.so
