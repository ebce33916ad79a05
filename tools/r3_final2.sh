set -e
# final round-3 build: GPU tests + smoke, default bench (live PMC), kernel-trace + PMC profile
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S gputests 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp
$S bench_final 900 python -u $R/bench.py
bash $R/tools/profile_round.sh r03final
