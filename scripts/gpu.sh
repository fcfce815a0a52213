#!/bin/bash
# gpurun wrapper: re-submits ONLY when gpurun reports an infrastructure
# "transient" status (box lost before the command ran: nothing executed, not
# charged).  Any real exit of the command is returned as is.
for attempt in $(seq 1 ${ATTEMPTS:-4}); do
  out=$(timeout 2400 /usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-1200} -- "$1" 2>&1)
  echo "$out" | tail -${TAILN:-25}
  if echo "$out" | grep -q "status=transient"; then sleep ${RETRY_SLEEP:-45}; continue; fi
  exit 0
done
