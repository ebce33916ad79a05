set -e
# chunks 1-3 as a loop (code 14.5 KB smaller) vs unrolled; instruction-fetch counters of both
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/avail_counters.txt 2>&1 || true
$S ab_cl 400 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/cl/libpow_gpu.so
$S pmc_if_base 90 timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_if_base -o run -- $R/tools/ab_sweep 2 $R/mpi_blockchain_amd/libpow_gpu.so
$S pmc_if_cl 90 timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_if_cl -o run -- $R/tools/ab_sweep 2 $R/abvar/cl/libpow_gpu.so
$S place_probe3 200 $R/tools/place_probe3
