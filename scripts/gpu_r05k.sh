#!/bin/bash
# Round 5: trace config-3 instance 39503 under the light-bin schedule (its 3.78e-4 status-1 answer)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/trace_instance.py 39503 3 > gpurun_out/trace_lsd_39503.txt 2>&1 || { tail -5 gpurun_out/trace_lsd_39503.txt; exit 1; }
tail -3 gpurun_out/trace_lsd_39503.txt
