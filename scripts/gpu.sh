#!/bin/bash
# gpurun wrapper: one call (no resubmission), the tail of its output.
# Usage: GPU_TIMEOUT=1200 bash scripts/gpu.sh 'command'
out=$(timeout 2700 /usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-1200} -- "$1" 2>&1)
echo "$out" | tail -${TAILN:-25}
