set -e
# randomised parity with the d > 32 kernel variants forced (POW_FORCE_FULL=1) and with
# pow_mine[_any] on K1 only (POW_LAT_MAX=0: no latency-kernel sub-round)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S parity_fuzz_full 600 env POW_FORCE_FULL=1 python -u tests/parity_fuzz.py --cases 400 --seed 5
$S parity_fuzz_k1only 600 env POW_LAT_MAX=0 python -u tests/parity_fuzz.py --cases 400 --seed 6
