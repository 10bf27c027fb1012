#!/bin/bash
# Run one gpurun call in the background; when the box could not be acquired
# (infrastructure-side "transient" / no free box, nothing charged, no part of
# the command ran) wait a minute and ask again, up to 8 times.  A command that
# ran and failed is never re-run.  Usage: tools/gpurun_bg.sh OUT.txt TIMEOUT 'cmd'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|backing off\|stopped responding while being prepared\|taken away by the GPU service" "$out" && ! grep -q "status=ok\|status=fail" "$out"; then
    echo "[gpurun_bg] attempt $i: box not acquired, retrying in 60 s" >> "$out.log"
    sleep 60
    continue
  fi
  echo "[gpurun_bg] done rc=$rc" >> "$out"
  exit 0
done
