set -e
# the latency kernel's compiler-scheduled rounds (round_ordered) in the e-path-first order (lo) vs the adopted order (head)
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S ttb_lo_d13 200 $R/tools/ab_ttb 13 301 $R/abvar/head/libpow_gpu.so $R/abvar/lo/libpow_gpu.so
$S ttb_lo_d17 200 $R/tools/ab_ttb 17 301 $R/abvar/head/libpow_gpu.so $R/abvar/lo/libpow_gpu.so
$S ttb_lo_d19 300 $R/tools/ab_ttb 19 201 $R/abvar/head/libpow_gpu.so $R/abvar/lo/libpow_gpu.so
