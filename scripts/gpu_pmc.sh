#!/bin/bash
# PMC counter passes for the dominant solve kernel (one rocprofv3 --pmc pass per group)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--batch 65536 --steps 2 --warmup 1 --cpu-seconds 0 --latency-batch 0"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
run() {
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i ($1) failed"; tail -5 gpurun_out/pmc/p$i.log; return 1; }
}
run "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" && \
run "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS" && \
run "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM" && \
run "GRBM_GUI_ACTIVE GRBM_COUNT"
ls gpurun_out/pmc/*/ > /dev/null
ls gpurun_out/pmc/*/
