#!/bin/bash
# Run one GPU step under its own time limit, output to gpurun_out/<name>.log.
# A step that ends with a fault/abort/timeout (exit >= 124, or any code other
# than 0/1/5) makes this script exit 100 so an `&&` chain stops there; a plain
# test failure (exit 1) does not.
#   tools/gpu_step.sh <name> <seconds> <command...>
name=$1; secs=$2; shift 2
out="${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out"
mkdir -p "$out"
echo "== $name: $*" >&2
timeout -k 10 "$secs" "$@" > "$out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" >&2
tail -4 "$out/$name.log" >&2
if [ $rc -ge 124 ] || { [ $rc -gt 1 ] && [ $rc -ne 5 ]; }; then exit 100; fi
exit 0
