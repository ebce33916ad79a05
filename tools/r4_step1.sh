# round 4, first GPU pass: K2' A/B, K1 A/B (round-3 build, head, last-round trim),
# the full GPU suite, the default bench, and the rocprofv3 passes of its workload
set -o pipefail
S=tools/gpu_step.sh
$S ab_k2 120 tools/ab_k2 5 abvar/k2old/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so abvar/k2smem/libpow_gpu.so && \
$S ab_k1_trim 300 tools/ab_sweep 9 abvar/r3/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so abvar/trim/libpow_gpu.so && \
$S gputests 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread && \
$S bench_default 600 python -u bench.py && \
bash tools/profile_round.sh r04
