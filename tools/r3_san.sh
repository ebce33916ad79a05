set -e
# host ASan/UBSan and TSan runs at the final round-3 build (build on the CPU first:
# tools/host_sanitize.sh build && tools/host_sanitize.sh tsan-build), the shard-union
# test, then the protocol soak
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S shard_union 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k shard_union
$S san_asan 400 bash tools/host_sanitize.sh run
$S san_tsan 600 bash tools/host_sanitize.sh tsan-run
$S soak_fork8_final 400 python -u tools/protocol_soak.py --runs 20 --ranks 8 --difficulty 5 --forced-fork
