set -e
# e-path-first round order: chunks 1-4 (o4, o8) and also chunk 0 (o4c0) vs the adopted order (head)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_order3 600 $R/tools/ab_sweep 13 $R/abvar/head/libpow_gpu.so $R/abvar/o4/libpow_gpu.so $R/abvar/o8/libpow_gpu.so $R/abvar/o4c0/libpow_gpu.so
