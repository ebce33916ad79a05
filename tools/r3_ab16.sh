set -e
# latency kernel with chunks 1-4 as asm groups at 4 waves per SIMD (lat4) vs without (ff2); then GPU tests + smoke
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ttb_lat4_d21 300 $R/tools/ab_ttb 21 201 $R/abvar/ff2/libpow_gpu.so $R/abvar/lat4/libpow_gpu.so
$S ttb_lat4_d20 300 $R/tools/ab_ttb 20 201 $R/abvar/ff2/libpow_gpu.so $R/abvar/lat4/libpow_gpu.so
cd $R
$S gputests 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
$S smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
