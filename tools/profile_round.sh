#!/bin/bash
# Kernel trace + PMC passes of the default bench workload (run on the GPU box).
#   tools/profile_round.sh <tag>
# Writes gpurun_out/prof_<tag>_*/ ; summaries are copied into profiles/ by hand.
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-ladder --no-cpu-baseline --no-peak --no-protocol --no-group-search --no-pmc"
S="$R/tools/gpu_step.sh"
$S prof_${tag}_kt 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof_${tag}_kt" -o run -- python $B &&
$S prof_${tag}_pmc1 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVES -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_${tag}_pmc1" -o run -- python $B &&
$S prof_${tag}_pmc2 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_${tag}_pmc2" -o run -- python $B &&
$S prof_${tag}_pmc3 300 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_${tag}_pmc3" -o run -- python $B &&
$S prof_${tag}_pmc4 300 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex pow_search -d "$R/gpurun_out/prof_${tag}_pmc4" -o run -- python $B
