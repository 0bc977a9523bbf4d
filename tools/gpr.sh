#!/bin/bash
# retry a gpurun call only while the pool had no box (nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|stopped responding while being prepared" $out && ! grep -q "status=ok" $out; then
    echo "[retry $i] $(tail -2 $out | head -1)" >> $out.retries
    sleep 150
    continue
  fi
  echo "rc=$rc" >> $out
  exit $rc
done
