#!/bin/bash
# Round 5: the block-LDL' factorization as the product (libcmpc.so) -- GPU tests, parity survey,
# N = 8 shard rehearsal, tail anatomy, stamps, A/B against the explicit inverse (libcmpc_inv.so),
# the NC 192 kernel's empty-bin span with its stream at high priority, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; grep -E "^FAILED" gpurun_out/gpu_tests.log | head -20
case $rc in 124|134|137|139) echo "tests aborted ($rc)"; exit 1;; esac
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
timeout -k 10 300 python -u tools/shard_times.py "" 5 > gpurun_out/shard_rehearsal.log 2>&1 || { tail -5 gpurun_out/shard_rehearsal.log; exit 1; }
cat gpurun_out/shard_rehearsal.log
CMPC_DIAG_LIB=$L/libcmpc_diag.so timeout -k 10 300 python tools/diag_counts.py > gpurun_out/diag_counts.txt 2>&1 || { tail -5 gpurun_out/diag_counts.txt; exit 1; }
grep -E "^cfg|max:|8 ranks" gpurun_out/diag_counts.txt
for c in 1 2; do
  timeout -k 10 120 python tools/stamps.py --config $c --batch 8192 --team 0 --lib $L/libcmpc_stamps.so > gpurun_out/stamps_cfg$c.txt 2>&1 || { tail -5 gpurun_out/stamps_cfg$c.txt; exit 1; }
  grep -E "==|per call|instance total|mean iters" gpurun_out/stamps_cfg$c.txt
done
TESTS=0 R=2 CASES="3:65536 2:4096 1:256 2:65536" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_inv.so || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/span -o run --output-format csv -- python bench.py --aux 0 --config 1 --batch 65536 --steps 5 --warmup 1 > gpurun_out/span.log 2>&1 || { tail -5 gpurun_out/span.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
tail -c 600 gpurun_out/bench_default.json
echo done
