#!/bin/bash
# (build container only) retry gpurun only while the pool reports no free box (transient; nothing ran, nothing charged)
CMD="$1"; TO="${2:-900}"; LOG="${3:-/tmp/gpuq.log}"
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])")
  if [ "$st" != "transient" ]; then echo "done after $i tries: $st" >> "$LOG"; exit 0; fi
  sleep 90
done
echo "gave up" >> "$LOG"
