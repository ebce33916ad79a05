set -e
# chunk 1-4 round orders in the asm groups: o4 = e-path first (re Ch Maj re hk re S1 T1 e' ra ra ra S0 a'),
# o5 = both rotation triples e-first, vs the adopted order (head)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ab_order 500 $R/tools/ab_sweep 11 $R/abvar/head/libpow_gpu.so $R/abvar/o4/libpow_gpu.so $R/abvar/o5/libpow_gpu.so
