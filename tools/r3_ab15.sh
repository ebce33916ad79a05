set -e
# chunk-0 schedule words 18-35 and the chunk feed-forward adds inside the asm groups (ff) vs HEAD
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_ff2 500 $R/tools/ab_sweep 9 $R/abvar/head/libpow_gpu.so $R/abvar/ff/libpow_gpu.so $R/abvar/ff2/libpow_gpu.so
