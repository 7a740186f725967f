#!/bin/bash
# Start N ranks of a torch.distributed program (env:// rendezvous on 127.0.0.1)
# without torchrun, so no extra Python parent process touches the GPU: the
# 8-rank one-GPU rehearsal is 8 apps + 8 daemons, exactly the box's limit of 16
# processes with the GPU open. Rank 0's stdout/stderr go to this script's; the
# others' to $RANKLOG_DIR/rank<r>.log. Exit status: the first non-zero rank's.
#   tools/launch_ranks.sh N PORT prog.py [args...]
set -u
n=$1; port=$2; shift 2
logdir=${RANKLOG_DIR:-/tmp}
mkdir -p "$logdir"
pids=()
for ((r = 0; r < n; r++)); do
  if [ "$r" -eq 0 ]; then
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n MASTER_ADDR=127.0.0.1 MASTER_PORT=$port python3 -u "$@" &
  else
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$n LOCAL_WORLD_SIZE=$n MASTER_ADDR=127.0.0.1 MASTER_PORT=$port python3 -u "$@" \
      > "$logdir/rank$r.log" 2>&1 &
  fi
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do
  wait "$p"; s=$?
  if [ "$s" -ne 0 ] && [ "$rc" -eq 0 ]; then rc=$s; fi
done
exit $rc
