#!/bin/bash
# Round 5: GPU tests + parity survey of the product library (ambiguity band 5 tol), the default
# bench line (warm tail, 1,024-robot closed loop) with and without the one-wave-per-CU team
# kernel, A/B of the product vs the block-LDL' variant vs Riccati for the NC 192 bin (also on
# standing batches), LDL' stamps, the NC 192 kernel's span with an empty bin.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=convex-mpc-unitree-go2_amd/cmpc/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tests/certify_sample.py gpu > gpurun_out/survey_gpu.log 2>&1 || { tail -5 gpurun_out/survey_gpu.log; exit 1; }
timeout -k 10 600 python -u tests/certify_sample.py cpu > gpurun_out/survey_cpu.log 2>&1 || { tail -5 gpurun_out/survey_cpu.log; exit 1; }
grep -E "above 1e-4|^cfg" gpurun_out/survey_cpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
LOOP="--sub-configs 0 --dynamics-steps 0 --tick-steps 0 --leg-steps 0 --api-ticks 0 --cpu-seconds 1"
CMPC_TEAM_OCC=1 timeout -k 10 300 python -u bench.py $LOOP > gpurun_out/bench_occ1.json 2> gpurun_out/bench_occ1.err || { tail -5 gpurun_out/bench_occ1.err; exit 1; }
python - <<'EOF'
import json
for f in ("bench_default", "bench_occ1"):
    a = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    w = a.get("warm_start", {}); cl = a.get("closed_loop", {}).get("robots_1024", {})
    print(f, "value %.0f ms %.3f" % (a["value"], a["ms_per_step"]),
          "warm itmax %s cold itmax %s warm p999 %s cold p999 %s" % (w.get("iters_max_warm"), w.get("iters_max_cold"), w.get("iters_p999_warm"), w.get("iters_p999_cold")),
          "loop1024 graph %.3f ms eager %.3f ms" % (cl.get("ms_per_tick_graph", -1), cl.get("ms_per_tick_eager", -1)))
EOF
TESTS=0 R=1 CASES="3:65536 2:4096" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_ldl.so $L/libcmpc_ric192.so || exit 1
timeout -k 10 120 python tools/stamps.py --config 2 --batch 8192 --team 0 --lib $L/libcmpc_ldl_stamps.so > gpurun_out/st_ldl_stamps_cfg2.txt 2>&1 || { tail -5 gpurun_out/st_ldl_stamps_cfg2.txt; exit 1; }
grep -E "==|per call|instance total|mean iters" gpurun_out/st_ldl_stamps_cfg2.txt
# standing batches (every instance NC 192): explicit inverse vs LDL vs Riccati for that bin
BENCH_ARGS=--stance-all TESTS=0 R=1 CASES="2:4096 2:16384" bash scripts/gpu_ab.sh $L/libcmpc.so $L/libcmpc_ldl.so $L/libcmpc_ric192.so || exit 1
# the NC 192 kernel's span with an empty bin (config 1 at 65,536: no NC 192 instance)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/span -o run --output-format csv -- python bench.py --aux 0 --config 1 --batch 65536 --steps 5 --warmup 1 > gpurun_out/span.log 2>&1 || { tail -5 gpurun_out/span.log; exit 1; }
echo done
