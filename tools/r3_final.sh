set -e
# round-3 final build: bench GPU tests, the default bench (live PMC passes), then kernel-trace + PMC profile
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S benchtests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_bench_gpu.py -k "microbench or contract"
cd /tmp && export TMPDIR=/tmp
$S bench_final 900 python -u $R/bench.py
bash $R/tools/profile_round.sh r03final
