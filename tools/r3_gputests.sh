set -e
# full GPU test suite + smoke at the current build
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd $R
$S gputests 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
