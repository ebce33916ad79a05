#!/bin/bash
# Hardware queues per process, measured: rocprofv3 --hsa-trace of
# tools/queue_trace_probe in each mode, counting the HIP runtime's
# hsa_queue_create / hsa_queue_destroy calls.  Run on the box.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
O="$R/gpurun_out/qtrace"
mkdir -p "$O"
for m in one rank valu valu_ctx; do
  timeout -k 10 120 rocprofv3 --hsa-trace -f csv -d "$O/$m" -o run -- "$R/tools/queue_trace_probe" "$m" > "$O/$m.log" 2>&1
  echo "== $m rc=$?"
  f=$(ls "$O/$m"/*hsa_api_trace.csv 2>/dev/null | head -1)
  if [ -n "$f" ]; then
    python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
key = "Function" if "Function" in rows[0] else [k for k in rows[0] if "unction" in k][0]
c = sum(r[key] == "hsa_queue_create" for r in rows)
d = sum(r[key] == "hsa_queue_destroy" for r in rows)
print(f"hsa_queue_create {c}, hsa_queue_destroy {d}, HSA calls traced {len(rows)}")
PY
  fi
  grep "^mode" "$O/$m.log"
done
