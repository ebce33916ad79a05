set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
$S node 500 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_node_gpu.py
cd /tmp && export TMPDIR=/tmp
$S ab_ilp_wgq 400 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/ilp2/libpow_gpu.so $R/abvar/wgq4/libpow_gpu.so $R/abvar/wgq8/libpow_gpu.so
$S pmc_wgq4 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_wgq4 -o run -- $R/tools/ab_sweep 2 $R/abvar/wgq4/libpow_gpu.so
$S pmc_wgq8 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_wgq8 -o run -- $R/tools/ab_sweep 2 $R/abvar/wgq8/libpow_gpu.so
$S pmc_base 120 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_base -o run -- $R/tools/ab_sweep 2 $R/mpi_blockchain_amd/libpow_gpu.so
