#!/bin/bash
# Host-code AddressSanitizer + UndefinedBehaviorSanitizer run of the C ABI and
# the protocol node.  Device code is NOT instrumented (GPU sanitizers are not
# available on this pool): -fsanitize goes behind -Xarch_host for the HIP
# library, and the consumers are built with clang so one sanitizer runtime
# (clang's, linked statically into each executable) serves the library too.
#
#   tools/host_sanitize.sh build     # here (CPU): builds into build/san/
#   tools/host_sanitize.sh run       # on the GPU box: runs the consumers
#   tools/host_sanitize.sh tsan-build / tsan-run   # ThreadSanitizer: pow_node and the
#                                                   # two-context board example, with the
#                                                   # library's host code instrumented too
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/build/san"
CLANG=/opt/rocm/llvm/bin/clang
CLANGXX=/opt/rocm/llvm/bin/clang++
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer"
MPI_INC=/opt/conda/include
MPI_LIB=/opt/conda/lib

case "${1:-}" in
build)
  mkdir -p "$O"
  C="$R/mpi_blockchain_amd/csrc"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -fPIC -shared -std=c++17 -mcode-object-version=5 \
    -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
    -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer \
    -DPOW_TEST_HOOKS -I "$R/include" -I "$C" \
    "$C/pow_api.cpp" "$C/pow_board.cpp" "$C/pow_group.cpp" "$C/pow_kernels.hip" "$C/pow_sort.hip" \
    "$C/valu_peak.hip" "$C/pow_aql.cpp" "$C/pow_test_kernels.hip" -o "$O/libpow_gpu.so" -L /opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
  $CLANG -std=c11 -O1 -g $SAN -I "$R/include" "$R/examples/mine_chain.c" \
    -L "$O" -lpow_gpu -Wl,-rpath,'$ORIGIN' -o "$O/mine_chain"
  $CLANG -std=c11 -D_POSIX_C_SOURCE=200809L -O1 -g $SAN -pthread -I "$R/include" "$R/examples/board_two_ctx.c" \
    -L "$O" -lpow_gpu -Wl,-rpath,'$ORIGIN' -o "$O/board_two_ctx"
  # round 6: pow_group_init's deadline (non-blocking init, abort of a communicator still initialising)
  $CLANG -std=c11 -D_POSIX_C_SOURCE=200809L -O1 -g $SAN -I "$R/include" "$R/examples/group_init_deadline.c" \
    -L "$O" -lpow_gpu -Wl,-rpath,'$ORIGIN' -o "$O/group_init_deadline"
  # the test build of the node (-DPOW_NODE_TEST_KNOBS): the runs below use its race-shaping switches
  $CLANGXX -std=c++17 -O1 -g $SAN -pthread -DPOW_NODE_TEST_KNOBS -I "$R/include" -I "$MPI_INC" \
    "$R/mpi_blockchain_amd/csrc/node/pow_node.cpp" -L "$O" -lpow_gpu -Wl,-rpath,'$ORIGIN' \
    "$MPI_LIB/libmpi.so" -Wl,-rpath-link,"$MPI_LIB" -o "$O/pow_node"
  echo "built $O"
  ;;
run)
  # Leaks inside the HIP runtime are not ours to judge; everything else aborts.
  export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1
  export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
  export LD_LIBRARY_PATH="$O${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}"
  "$O/mine_chain" 10 12
  POW_GRID_PER_CU=4 "$O/board_two_ctx"
  POW_TEST_RCCL_LIB="$R/tests/stub_rccl/libstub_rccl.so" "$O/group_init_deadline" 3000
  "$O/group_init_deadline" 3000
  W=$(mktemp -d)
  cd "$W"
  export LD_LIBRARY_PATH="/lib/x86_64-linux-gnu:$MPI_LIB:$LD_LIBRARY_PATH"
  # d = 9, 4 ranks; then d = 5, 6 ranks with the test pauses so forks, chain
  # migration and chain service run.  --serial-init 1: every rank finishes its
  # (sanitizer-slowed) GPU set-up before MPI_Init, so all of them take part.
  /opt/conda/bin/mpiexec -np 4 "$O/pow_node" --difficulty 9 --serial-init 1
  echo "chains d=9:"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  rm -f ./*.out
  /opt/conda/bin/mpiexec -np 6 "$O/pow_node" --difficulty 5 --serial-init 1 --hold-first 1 \
    --winner-pause-us 400 --pause-us 200 > net_d5.log
  cat net_d5.log
  echo "chains d=5:"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  echo "protocol paths taken (lost races, branch conflicts, chain requests):"
  grep -c "Perdí la carrera\|Conflicto\|TAG_CHAIN_HASH" net_d5.log || true
  rm -f ./*.out
  # the mutual chain-request case (round 3): every rank 3 blocks ahead on a private branch
  /opt/conda/bin/mpiexec -np 2 "$O/pow_node" --difficulty 9 --serial-init 1 --private-lead 3 > net_mutual.log
  cat net_mutual.log
  echo "chains (mutual requests):"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  rm -f ./*.out
  # the same 4-rank mutual case with the test library's direct AQL dispatch (POW_AQL=1)
  POW_AQL=1 /opt/conda/bin/mpiexec -np 4 "$O/pow_node" --difficulty 9 --serial-init 1 --private-lead 3 > net_mutual_aql.log
  cat net_mutual_aql.log
  echo "chains (mutual requests, direct dispatch):"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  ;;
tsan-build)
  # ThreadSanitizer on pow_node's own code (receive thread, miner thread, GPU
  # set-up thread) AND on the library's host code (-Xarch_host: the cancel
  # word, pow_cancel's epoch, the stop board's slots cross threads there);
  # device code and the HIP/HSA/MPI runtimes below are not instrumented.
  T="$O/tsan"
  mkdir -p "$T"
  C="$R/mpi_blockchain_amd/csrc"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -fPIC -shared -std=c++17 -mcode-object-version=5 \
    -Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer -DPOW_TEST_HOOKS -I "$R/include" -I "$C" \
    "$C/pow_api.cpp" "$C/pow_board.cpp" "$C/pow_group.cpp" "$C/pow_kernels.hip" "$C/pow_sort.hip" \
    "$C/valu_peak.hip" "$C/pow_aql.cpp" "$C/pow_test_kernels.hip" -o "$T/libpow_gpu.so" -L /opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
  $CLANGXX -std=c++17 -O1 -g -fsanitize=thread -pthread -DPOW_NODE_TEST_KNOBS -I "$R/include" -I "$MPI_INC" \
    "$R/mpi_blockchain_amd/csrc/node/pow_node.cpp" -L "$T" -lpow_gpu \
    -Wl,-rpath,'$ORIGIN' "$MPI_LIB/libmpi.so" -Wl,-rpath-link,"$MPI_LIB" -o "$T/pow_node_tsan"
  $CLANG -std=c11 -D_POSIX_C_SOURCE=200809L -O1 -g -fsanitize=thread -pthread -I "$R/include" \
    "$R/examples/board_two_ctx.c" -L "$T" -lpow_gpu -Wl,-rpath,'$ORIGIN' -o "$T/board_two_ctx_tsan"
  $CLANG -std=c11 -D_POSIX_C_SOURCE=200809L -O1 -g -fsanitize=thread -pthread -I "$R/include" \
    "$R/examples/group_init_deadline.c" -L "$T" -lpow_gpu -Wl,-rpath,'$ORIGIN' -o "$T/group_init_deadline_tsan"
  echo "built $T"
  ;;
tsan-run)
  T="$O/tsan"
  S="$T/tsan.supp"
  # Only the runtimes below the library are suppressed; libpow_gpu.so itself is instrumented.
  printf '%s\n' "called_from_lib:libamdhip64.so" "called_from_lib:libhsa-runtime64.so" \
    "called_from_lib:libmpi.so" > "$S"
  export TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=$S"
  export LD_LIBRARY_PATH="/lib/x86_64-linux-gnu:$MPI_LIB${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}"
  POW_GRID_PER_CU=4 "$T/board_two_ctx_tsan"
  # RCCL's own threads are not instrumented either (the bootstrap and proxy threads of the real-RCCL run)
  echo "called_from_lib:librccl.so" >> "$S"
  POW_TEST_RCCL_LIB="$R/tests/stub_rccl/libstub_rccl.so" "$T/group_init_deadline_tsan" 3000
  "$T/group_init_deadline_tsan" 3000
  W=$(mktemp -d)
  cd "$W"
  /opt/conda/bin/mpiexec -np 4 "$T/pow_node_tsan" --difficulty 9
  echo "chains d=9:"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  rm -f ./*.out
  /opt/conda/bin/mpiexec -np 6 "$T/pow_node_tsan" --difficulty 5 --hold-first 1 --winner-pause-us 400 \
    --pause-us 200 > net_d5.log
  cat net_d5.log
  echo "chains d=5:"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  echo "protocol paths taken (lost races, branch conflicts, chain requests):"
  grep -c "Perdí la carrera\|Conflicto\|TAG_CHAIN_HASH" net_d5.log || true
  rm -f ./*.out
  /opt/conda/bin/mpiexec -np 2 "$T/pow_node_tsan" --difficulty 9 --private-lead 3 > net_mutual.log
  cat net_mutual.log
  echo "chains (mutual requests):"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  rm -f ./*.out
  POW_AQL=1 /opt/conda/bin/mpiexec -np 4 "$T/pow_node_tsan" --difficulty 9 --private-lead 3 > net_mutual_aql.log
  cat net_mutual_aql.log
  echo "chains (mutual requests, direct dispatch):"; md5sum ./*.out | awk '{print $1}' | sort | uniq -c
  ;;
*)
  echo "usage: $0 build|run|tsan-build|tsan-run" >&2; exit 2;;
esac
