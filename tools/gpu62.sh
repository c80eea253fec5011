set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r62
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r62/kt -o run --output-format csv -- python tools/learner_trace.py > gpurun_out/r62/kt.log 2>&1 || { tail gpurun_out/r62/kt.log; exit 1; }
python tools/learner_seq.py gpurun_out/r62/kt/run_kernel_trace.csv > gpurun_out/r62/seq.txt
rm -f gpurun_out/r62/kt/run_kernel_trace.csv
wc -l gpurun_out/r62/seq.txt
