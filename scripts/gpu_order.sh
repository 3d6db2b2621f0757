#!/bin/bash
# Launch order of the two register classes (light first vs heavy first) with a given library:
# timelines (times build), shard rehearsal and the headline workloads, A/B against the product.
#   usage: bash scripts/gpu_order.sh variant.so [times]   (times: timelines with libcmpc_times.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ord
export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
V=$1
python -c "import torch; p = torch.cuda.get_device_properties(0); print(p.name, p.multi_processor_count, getattr(p, 'shared_memory_per_multiprocessor', None), getattr(p, 'shared_memory_per_block_optin', None))"
if [ "$2" = "times" ]; then
  for hf in 0 65536; do
    CMPC_HEAVY_FIRST=$hf timeout -k 10 200 python -u tools/shard_anatomy.py times gpurun_out/ord/hf$hf 1 8 > gpurun_out/ord/hf$hf.log 2>&1 || { echo "times $hf failed"; tail -5 gpurun_out/ord/hf$hf.log; exit 1; }
  done
fi
for hf in 0 65536; do
  CMPC_HEAVY_FIRST=$hf timeout -k 10 200 python -u tools/shard_times.py $V 5 > gpurun_out/ord/sh_hf$hf.log 2>&1 || { echo "shards $hf failed"; tail -5 gpurun_out/ord/sh_hf$hf.log; exit 1; }
  echo "heavy first <= $hf"; tail -4 gpurun_out/ord/sh_hf$hf.log
done
TESTS=0 R=${R:-2} CASES=${CASES:-"3:65536 2:65536 2:4096 3:16384 3:8192 1:65536"} bash scripts/gpu_ab.sh $L/libcmpc.so $V $V@CMPC_HEAVY_FIRST=65536
