set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/test.log 2>&1; rc=$?; tail -3 gpurun_out/test.log; [ $rc -eq 0 ] || exit 1
for c in 1 2 3; do timeout -k 10 300 python bench.py --config $c --steps 10 --cpu-seconds 0 --dynamics-steps 0 --warm-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/b0_cfg$c.json 2>gpurun_out/b0_cfg$c.err || exit 1; python -c "import json;a=json.load(open('gpurun_out/b0_cfg$c.json'));print($c, a['value'], a['latency_ms_b256'], a['bin_ms_per_step'], a['bin_solves'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof0 -o run --output-format csv -- python bench.py --config 3 --steps 3 --warmup 1 --cpu-seconds 0 --latency-batch 0 --dynamics-steps 0 --warm-steps 0 --tick-steps 0 --leg-steps 0 --loop-steps 0 --api-ticks 0 > gpurun_out/prof0.log 2>&1 || exit 1
echo done
