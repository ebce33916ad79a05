set -e
# end-of-round soaks: 5,000 + 2,000 (d > 32 variants forced) randomised parity cases, 60 forced-fork 8-rank networks
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S fuzz_5000 900 python -u tests/parity_fuzz.py --cases 5000 --seed 2026
$S fuzz_2000_full 600 env POW_FORCE_FULL=1 python -u tests/parity_fuzz.py --cases 2000 --seed 2027
$S soak_fork8_60 600 python -u tools/protocol_soak.py --runs 60 --ranks 8 --difficulty 5 --forced-fork
