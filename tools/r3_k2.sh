set -e
# K2' (one-block pow_hash_block: kernarg message, mapped-host digest) vs the batch path of the previous build
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S k2_old 120 env LD_LIBRARY_PATH=$R/abvar/lat4 $R/tools/k2_c
$S k2_new 120 env LD_LIBRARY_PATH=$R/mpi_blockchain_amd $R/tools/k2_c
$S k2_tests 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "single_block or digests or validation_beside or chained"
