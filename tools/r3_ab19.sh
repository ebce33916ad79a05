set -e
# more chunk 1-4 round orders (e-path first family) vs the adopted order (head)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_order2 600 $R/tools/ab_sweep 11 $R/abvar/head/libpow_gpu.so $R/abvar/o4/libpow_gpu.so $R/abvar/o6/libpow_gpu.so $R/abvar/o7/libpow_gpu.so $R/abvar/o8/libpow_gpu.so
