# round 4, second GPU pass: K2' one-wave order A/B, K1' time-to-block A/B with it,
# a HIP API + kernel trace of pow_hash_block calls, and the previously failing tests
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
S="$R/tools/gpu_step.sh"
R="${GRAFT_REPO_ROOT:-$(pwd)}"
(cd /tmp && export TMPDIR=/tmp && $S k2_trace 120 rocprofv3 --kernel-trace --hip-trace --stats -f csv -d "$R/gpurun_out/k2_trace" -o run -- "$R/tools/ab_k2" 1 "$R/mpi_blockchain_amd/libpow_gpu.so") && \
$S gputests2 400 python -u -m pytest tests/test_node_gpu.py tests/test_shard_gpu.py tests/test_gpu_parity.py -k "network or mixed or mutual or multiprocess or failure or single_block or parity_fuzz or digests" -v --timeout 300 --timeout-method thread
