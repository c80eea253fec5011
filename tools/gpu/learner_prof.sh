cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out/lp && \
timeout -k 10 600 python -u -m pytest tests/test_learner.py tests/test_gpu_train_loop.py tests/test_gpu_adam.py tests/test_gpu_lg_gemm.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/lp/learner_tests.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lp/tr -o run -- python3 tools/quick_learner.py humanoid-run > gpurun_out/lp/tr.log 2>&1 && \
python3 tools/learner_prof.py $(find gpurun_out/lp/tr -name "*kernel_trace.csv" | head -1) 10 > gpurun_out/lp/prof.txt
