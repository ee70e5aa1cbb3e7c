#!/bin/bash
# Runs one gpurun call, repeating it (up to 5 times, 60 s apart) only when the
# pool reports a transient infrastructure state (no box / box lost while being
# prepared: nothing ran, nothing charged).  Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 ${RETRIES:-5}); do
  out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient\|no free box\|slot(s) on this pod are busy"; then
    echo "[retry $i: transient]" >&2
    sleep ${RETRY_SLEEP:-60}
    continue
  fi
  echo "$out"
  exit $rc
done
echo "$out"
exit 3
