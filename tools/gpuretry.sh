#!/bin/bash
# retry a gpurun call ONLY while the pool reports a transient / backoff state (nothing ran); never after a real run
out=$1; shift
for i in $(seq 1 12); do
  timeout 3000 /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  if grep -q "status=transient\|backing off\|no box or slot\|busy" "$out" && ! grep -q "status=ok\|status=fail\|rc=[0-9]" "$out"; then
    w=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | head -1); sleep $(( ${w:-60} + 15 ))
    continue
  fi
  break
done
echo finished >> "$out"
