#!/bin/bash
# Run GPU steps in sequence; each under its own time limit.  A step that ends
# with a fault/abort/timeout (exit >= 124 or signal) stops the chain; a plain
# test failure (exit 1) does not.
#   tools/gpu_step.sh <name> <seconds> <command...>
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" >&2
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" >&2
tail -5 "gpurun_out/$name.log" >&2
if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then exit 100; fi
exit 0
