set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import torch;print(torch.cuda.get_device_name(0))"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
tail -30 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tools/quick_time.py humanoid-run 1 && timeout -k 10 120 python tools/quick_time.py humanoid-run 8 && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; echo "bench rc=$?"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
