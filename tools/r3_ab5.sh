set -e
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S place_probe 200 $R/tools/place_probe
$S ab_e64 300 $R/tools/ab_sweep 9 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/e64/libpow_gpu.so
$S ttb_lat_d13 200 $R/tools/ab_ttb 13 301 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/lat0/libpow_gpu.so $R/abvar/lat4/libpow_gpu.so
$S ttb_lat_d17 200 $R/tools/ab_ttb 17 301 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/lat0/libpow_gpu.so $R/abvar/lat4/libpow_gpu.so
$S ttb_lat_d21 300 $R/tools/ab_ttb 21 201 $R/mpi_blockchain_amd/libpow_gpu.so $R/abvar/lat0/libpow_gpu.so $R/abvar/lat4/libpow_gpu.so
cd $R
$S bench_default 900 python -u bench.py
