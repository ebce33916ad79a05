# round 4, third GPU pass: the clock and issue cycles of one-wave kernels (K2',
# K1' at d = 9) from PMC counters with the kernel trace of the same dispatches
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
S="$R/tools/gpu_step.sh"
cd /tmp && export TMPDIR=/tmp
$S k2_pmc 90 timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -f csv --kernel-include-regex pow_hash_one -d "$R/gpurun_out/k2_pmc" -o run -- "$R/tools/ab_k2" 1 "$R/mpi_blockchain_amd/libpow_gpu.so" && \
$S lat_pmc 90 timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace -f csv --kernel-include-regex pow_search_lat -d "$R/gpurun_out/lat_pmc" -o run -- "$R/tools/ab_ttb" 9 101 "$R/mpi_blockchain_amd/libpow_gpu.so"
