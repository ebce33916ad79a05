set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_adopt 400 $R/tools/ab_sweep 11 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/p3/libpow_gpu.so $R/abvar/base/libpow_gpu.so
$S pmc_new 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_new -o run -- $R/tools/ab_sweep 2 $R/mpi_blockchain_amd/libpow_gpu.so
cd $R
$S gputests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
