#!/bin/bash
# Run one gpurun command, retrying ONLY when no box / slot was free (exit 3 with a "no box" / "transient" message:
# nothing ran, nothing charged), with a pause between tries.  Any other outcome ends it -- in particular an exit 3 that
# reports a GPU fault (the command ran and faulted) is never retried.  usage: gpurun_retry.sh OUT TIMEOUT CMD
OUT=$1; TMO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  echo "attempt $i rc=$rc $(date +%T)" >> "$OUT.attempts"
  if [ $rc -ne 3 ] || grep -qi "fault\|status=fail\|illegal\|abort" "$OUT" || \
     ! grep -qi "status=transient\|no box\|no free\|no slot\|try again" "$OUT"; then
    exit $rc
  fi
  sleep 150
done
exit 3
