set -e
# sustained 100-step bench, and kernel-trace stats of the whole default bench (all kernels) at the final build
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S bench_sustained 400 python -u $R/bench.py --steps 100 --warmup 2 --no-ladder --no-cpu-baseline --no-protocol --no-group-search --no-pmc
$S prof_fullbench 900 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_fullbench -o run -- python -u $R/bench.py --no-pmc --no-cpu-baseline
