set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.is_available(), torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t1.log 2>&1
echo "pytest exit $?" >> gpurun_out/t1.log
