set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py --config 1 --batch 65536 > gpurun_out/st1.txt 2>&1 && timeout -k 10 200 python tools/stamps.py --config 2 --batch 65536 > gpurun_out/st2.txt 2>&1 && timeout -k 10 200 python tools/stamps.py --config 1 --batch 65536 --warm > gpurun_out/st3.txt 2>&1
cat gpurun_out/st1.txt gpurun_out/st2.txt gpurun_out/st3.txt
