#!/bin/bash
# LDS bank-conflict counters of the config-3 headline for each given library (one PMC pass each)
#   usage: bash scripts/gpu_lds.sh a.so [b.so ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lds
export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename $lib .so)
  timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/lds/$tag -o run -- python bench.py --aux 0 --config 3 --steps 2 --warmup 1 --lib $lib > gpurun_out/lds/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 gpurun_out/lds/$tag.log; exit 1; }
done
echo done
