set -e
# protocol soaks at the final round-3 build: forced-fork 8-rank networks, mutual chain requests, mixed reference + GPU networks
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S soak_fork8 400 python -u tools/protocol_soak.py --runs 30 --ranks 8 --difficulty 5 --forced-fork
$S soak_mixed 400 python -u tools/protocol_soak.py --runs 15 --ranks 2 --ref 2 --difficulty 9
