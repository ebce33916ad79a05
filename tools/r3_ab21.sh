set -e
# further e-path-first orders for chunks 1-4 (Maj moved into the a-path; e' between a-rotations) vs the adopted one (head)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_order4 600 $R/tools/ab_sweep 13 $R/abvar/head/libpow_gpu.so $R/abvar/o10/libpow_gpu.so $R/abvar/o11/libpow_gpu.so $R/abvar/o12/libpow_gpu.so
