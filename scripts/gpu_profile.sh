#!/bin/bash
# The round's measurement record on one GPU box:
#   1. the default bench line (all objects, CPU baseline)              -> gpurun_out/bench_full.json
#   2. rocprofv3 --kernel-trace --stats of the headline (config 3)     -> gpurun_out/prof/
#   3. PMC passes, each its own run (HBM bytes, instruction mix, clock) -> gpurun_out/pmc/p*/
# then tools/summarize_profile.py --tag $TAG turns them into profiles/ (run it on the CPU side).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench failed"; tail gpurun_out/bench_full.err; exit 1; }
  cat gpurun_out/bench_full.json
fi
HEAD="--aux 0 --config ${CFG:-3} ${BATCH:+--batch $BATCH}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py $HEAD --steps 5 --warmup 1 > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof.log; exit 1; }
i=0
pass() {
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc/p$i -o run -- python bench.py $HEAD --steps 2 --warmup 1 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pmc pass $i ($1) failed"; tail -5 gpurun_out/pmc/p$i.log; return 1; }
}
pass "FETCH_SIZE" && \
pass "WRITE_SIZE" && \
pass "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" && \
pass "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES" || exit 1
echo done
