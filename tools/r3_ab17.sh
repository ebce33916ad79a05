set -e
# per-wave solution stage of 256 entries, flushed at >= 192 (st) vs 128 / >= 64 (current): flush atomics and time
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_st 400 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/st/libpow_gpu.so
$S pmc_st_write 90 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d $R/gpurun_out/pmc_st_write -o run -- $R/tools/ab_sweep 2 $R/abvar/st/libpow_gpu.so
$S sustained_bench 400 python -u $R/bench.py --steps 100 --warmup 2 --no-ladder --no-cpu-baseline --no-protocol --no-group-search --no-pmc
$S prof_fullbench 900 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_fullbench -o run -- python -u $R/bench.py --no-pmc --no-cpu-baseline
