set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_wgq_order2 400 $R/tools/ab_sweep 11 $R/abvar/wgq8/libpow_gpu.so $R/abvar/wgq16/libpow_gpu.so $R/abvar/wgq4/libpow_gpu.so $R/mpi_blockchain_amd/libpow_gpu.so
$S pmc_wgq16 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_wgq16 -o run -- $R/tools/ab_sweep 2 $R/abvar/wgq16/libpow_gpu.so
