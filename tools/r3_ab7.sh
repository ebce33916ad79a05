set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S gputests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
cd /tmp && export TMPDIR=/tmp
$S ab_g4_vs_r02 400 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/base/libpow_gpu.so
