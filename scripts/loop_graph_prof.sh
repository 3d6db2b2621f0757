set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/loop_graph.py 65536 24 > gpurun_out/lg_65536.log 2>&1 || exit 1
timeout -k 10 300 python tools/loop_graph.py 1024 200 > gpurun_out/lg_1024.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lgprof -o lg -- python tools/loop_graph.py 65536 8 > gpurun_out/lg_prof.log 2>&1 || exit 1
cat gpurun_out/lg_65536.log gpurun_out/lg_1024.log
