R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
B="$R/bench.py --steps 2 --warmup 1 --no-ladder --no-cpu-baseline --no-peak --no-protocol"
$S gpu_tests 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread &&
$S ab2 200 tools/ab_sweep 5 build/ab/v0/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so &&
cd /tmp && export TMPDIR=/tmp &&
$S prof_r01c_pmc4 200 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_r01c_pmc4" -o run -- python $B &&
$S prof_r01c_pmc3 200 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_r01c_pmc3" -o run -- python $B
