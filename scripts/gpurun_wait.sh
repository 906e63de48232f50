#!/bin/bash
# Host-side helper (never runs on the GPU box): submit one gpurun call and, only
# when the pool had no box for it (nothing ran, nothing charged: "no free box",
# "transient", "backing off"), wait as long as gpurun suggests and submit it
# again, up to TRIES times.  Any call that reached the box ends the loop,
# whatever its result.
T=${TIMEOUT:-900}
for i in $(seq 1 ${TRIES:-12}); do
  out=$(/usr/local/graft/bin/gpurun --timeout $T -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q -E "no free box|status=transient|backing off"; then
    w=$(echo "$out" | grep -o 'retry in [0-9]*s' | head -1 | grep -o '[0-9]*')
    w=${w:-60}; [ "$w" -lt 30 ] && w=30
    echo "[wait] attempt $i: no box; sleeping ${w}s" >&2
    sleep $((w + 5))
    continue
  fi
  echo "$out"
  exit $rc
done
echo "[wait] gave up after ${TRIES:-12} attempts" >&2
exit 3
