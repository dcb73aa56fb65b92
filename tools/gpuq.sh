#!/bin/bash
# submit one gpurun call; resubmit only while the pool reports no box (rc 3 / transient, nothing ran)
out=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "no free box\|backing off\|stopped responding while being prepared\|are busy\|retry in a few" $out && ! grep -q "status=ok" $out; then sleep 120; continue; fi
  break
done
echo "rc=$rc" >> $out
