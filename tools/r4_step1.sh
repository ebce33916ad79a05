# round 4, first GPU pass: K2' A/B (round 3 vs head vs scalar-load form), K1 A/B
# (round-3 build, head, last-round trim), K1' time-to-block A/B (pipelined LDS
# reads vs the compiler's), the full GPU suite, the default bench, rocprofv3 passes
set -o pipefail
S=tools/gpu_step.sh
$S ab_k2 120 tools/ab_k2 5 abvar/k2old/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so abvar/k2smem/libpow_gpu.so && \
$S ab_ttb_d9 120 tools/ab_ttb 9 301 abvar/latnopipe/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so && \
$S ab_ttb_d13 120 tools/ab_ttb 13 301 abvar/latnopipe/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so && \
$S ab_ttb_d17 200 tools/ab_ttb 17 301 abvar/latnopipe/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so && \
$S ab_k1_trim 300 tools/ab_sweep 9 abvar/r3/libpow_gpu.so mpi_blockchain_amd/libpow_gpu.so abvar/trim/libpow_gpu.so && \
$S gputests 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread && \
$S bench_default 600 python -u bench.py && \
bash tools/profile_round.sh r04
