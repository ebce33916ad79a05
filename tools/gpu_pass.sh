#!/bin/bash
# One GPU pass made of named steps, each under its own time limit (tools/gpu_step.sh);
# a fault, abort or timeout in one step ends the pass.  Run on the GPU box:
#   /usr/local/graft/bin/gpurun -- 'bash tools/gpu_pass.sh tests bench profile'
#
# steps:
#   tests            the whole GPU suite (pytest -m gpu)
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (default: N = 1, every block of the JSON line)
#   profile          tools/profile_round.sh r06 (kernel trace + 4 PMC passes of the bench workload)
#   rehearse N T     bench.py's N > 1 path with N ranks sharing the GPU (BENCH_REHEARSAL=1), transport T
#                    (gloo | rccl_stub): the JSON line with timing, board and placement blocks
#   fuzz             randomised parity, shipped library: 1,000 cases (tests/parity_fuzz.py)
#   fuzz_big         10,000 cases, then 2,000 each on the test library: K1' asm variants
#                    (POW_LAT_WPS=4), + d > 32 variants, and K1 alone (POW_LAT_MAX=0)
#   soak_mixed       20 mixed networks: 2 reference ranks + 2 pow_node ranks (tools/protocol_soak.py)
#   queue_pressure   40 six-rank networks alone, then beside a queue-holding process (tools/queue_pressure.sh)
#   queue_ab         the null-stream A/B beside the holder, 3 rounds (tools/queue_pressure_ab.sh; build the
#                    variant first with tools/build_nullstream_variant.sh)
#   ab_k1 L...       K1 sweep A/B over libpow_gpu.so builds (tools/ab_sweep, 9 alternating windows)
#   ab_k2 L...       pow_hash_block A/B (tools/ab_k2, 5 x 200 calls)
#   ttb D L...       time-to-block A/B at difficulty D (tools/ab_ttb, 301 templates)
#   k2_trace         rocprofv3 HIP API + kernel trace of 200 pow_hash_block calls
#   pmc_onewave      PMC (clock, wave cycles, VALU) of K2' and of K1' at d = 9
#   sanitize         host ASan/UBSan then TSan runs of the C ABI, the node and pow_group_init's deadline
#                    (build them first, here: tools/host_sanitize.sh build && tools/host_sanitize.sh tsan-build)
# A/B library lists end at the next step name.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
S="$R/tools/gpu_step.sh"
L="$R/mpi_blockchain_amd/libpow_gpu.so"
STEPS=" tests smoke bench profile rehearse fuzz fuzz_big soak_mixed queue_pressure queue_ab ab_k1 ab_k2 ttb k2_trace pmc_onewave sanitize "
libs() {  # the library arguments of an A/B step
  LIBS=()
  while [ $# -gt 0 ] && [[ "$STEPS" != *" $1 "* ]]; do LIBS+=("$1"); shift; done
}
cd "$R"
while [ $# -gt 0 ]; do
  step=$1; shift
  case "$step" in
    tests) POW_NODE_LOG_DIR="$R/gpurun_out/netlogs" \
             $S gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit $? ;;
    smoke) $S smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) $S bench 900 python -u bench.py || exit $? ;;
    profile) bash "$R/tools/profile_round.sh" r06 || exit $? ;;
    rehearse) n=$1; tr=$2; shift 2
      BENCH_REHEARSAL=1 BENCH_REHEARSAL_TRANSPORT=$tr $S rehearse_${n}_$tr 900 python -u -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$n" \
        --steps 2 --warmup 1 || exit $? ;;
    fuzz) $S fuzz 900 python -u tests/parity_fuzz.py --cases 1000 --seed 404 || exit $? ;;
    fuzz_big) $S fuzz_big 900 python -u tests/parity_fuzz.py --cases 10000 --seed 4004 &&
      POW_LAT_WPS=4 $S fuzz_lat_asm 900 python -u tests/parity_fuzz.py --test-hooks --cases 2000 --seed 4005 &&
      POW_LAT_WPS=4 POW_FORCE_FULL=1 $S fuzz_lat_asm_full 900 python -u tests/parity_fuzz.py --test-hooks --cases 2000 --seed 4006 &&
      POW_LAT_MAX=0 $S fuzz_k1only 900 python -u tests/parity_fuzz.py --test-hooks --cases 2000 --seed 4007 || exit $? ;;
    soak_mixed) $S soak_mixed 900 python -u tools/protocol_soak.py --runs 20 --ranks 2 --ref 2 --difficulty 9 || exit $? ;;
    queue_pressure) bash "$R/tools/queue_pressure.sh" 40 6 || exit $? ;;
    queue_ab) bash "$R/tools/queue_pressure_ab.sh" 3 || exit $? ;;
    ab_k1) libs "$@"; shift ${#LIBS[@]}; $S ab_k1 400 tools/ab_sweep 9 "${LIBS[@]}" || exit $? ;;
    ab_k2) libs "$@"; shift ${#LIBS[@]}; $S ab_k2 200 tools/ab_k2 5 "${LIBS[@]}" || exit $? ;;
    ttb) d=$1; shift; libs "$@"; shift ${#LIBS[@]}; $S ttb_d$d 300 tools/ab_ttb "$d" 301 "${LIBS[@]}" || exit $? ;;
    k2_trace) (cd /tmp && export TMPDIR=/tmp && $S k2_trace 120 rocprofv3 --kernel-trace --hip-trace --stats -f csv \
                 -d "$R/gpurun_out/k2_trace" -o run -- "$R/tools/ab_k2" 1 "$L") || exit $? ;;
    pmc_onewave) (cd /tmp && export TMPDIR=/tmp &&
        $S k2_pmc 90 timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES \
          --kernel-trace -f csv --kernel-include-regex pow_hash_one -d "$R/gpurun_out/k2_pmc" -o run -- "$R/tools/ab_k2" 1 "$L" &&
        $S lat_pmc 90 timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES \
          --kernel-trace -f csv --kernel-include-regex pow_search_lat -d "$R/gpurun_out/lat_pmc" -o run -- "$R/tools/ab_ttb" 9 101 "$L") \
        || exit $? ;;
    sanitize) $S asan 600 bash "$R/tools/host_sanitize.sh" run && $S tsan 600 bash "$R/tools/host_sanitize.sh" tsan-run \
        || exit $? ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
