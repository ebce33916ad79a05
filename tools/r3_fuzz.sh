set -e
# randomised GPU-vs-oracle parity (tests/parity_fuzz.py), two seeds
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S parity_fuzz_s7 600 python -u tests/parity_fuzz.py --cases 300 --seed 7
$S parity_fuzz_s11 600 python -u tests/parity_fuzz.py --cases 300 --seed 11
