#!/bin/bash
# Submit one gpurun call, re-submitting it only while the pool reports no box / a
# transient infrastructure event (nothing ran, nothing charged); a call that ran is
# never repeated, whatever its result.
# usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out" && ! grep -q "status=ok\|status=fail\|status=timeout" "$out"; then
    echo "[gpurun_wait] transient (try $i), retrying in 150 s" >> "$out.tries"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
