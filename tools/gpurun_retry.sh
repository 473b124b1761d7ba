#!/bin/bash
# Run one gpurun command, retrying ONLY when no box / slot was free (exit 3: nothing ran, nothing charged), with a
# pause between tries.  Any other outcome (success, failure, refusal) ends it.  usage: gpurun_retry.sh OUT TIMEOUT CMD
OUT=$1; TMO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "status=transient" "$OUT" && exit $rc
  sleep 150
done
exit 3
