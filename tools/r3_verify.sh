#!/bin/bash
# Round-3 verification at HEAD: default bench (live PMC passes), then the
# kernel-trace + PMC profile passes (tools/profile_round.sh).
set -u
R=$GRAFT_REPO_ROOT
S=$R/tools/gpu_step.sh
cd /tmp && export TMPDIR=/tmp
$S bench_default 900 python -u $R/bench.py &&
bash $R/tools/profile_round.sh r03
