#!/bin/bash
# Where does pow_group_init's deadline path stall with RCCL itself?  Runs
# tools/gid_probe (examples/group_init_deadline.c against the shipped library)
# with NCCL_DEBUG=INFO under a time limit, and samples every thread's name,
# state and kernel wait channel every 2 s while it runs.  Run on the box.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/rccl_probe"
mkdir -p "$O"
cd /tmp
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP,ENV timeout -k 5 "${1:-40}" "$R/tools/gid_probe" 3000 > "$O/gid.log" 2>&1 &
P=$!
for i in $(seq 1 30); do
  sleep 2
  kill -0 $P 2>/dev/null || break
  C=$(pgrep -P $P | head -1)
  [ -n "$C" ] || continue
  {
    echo "== t=$((i * 2)) s pid $C"
    for t in /proc/$C/task/*; do
      printf '%s %s %s %s\n' "$(basename $t)" "$(cat $t/comm 2>/dev/null)" \
        "$(awk '{print $3}' $t/stat 2>/dev/null)" "$(cat $t/wchan 2>/dev/null)"
    done
  } >> "$O/threads.log"
done
wait $P
echo "rc=$?" >> "$O/gid.log"
tail -n 5 "$O/gid.log"
