set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r45
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r45/kt -o run --output-format csv -- python tools/learner_trace.py > gpurun_out/r45/kt.log 2>&1 || { tail gpurun_out/r45/kt.log; exit 1; }
python tools/learner_prof.py gpurun_out/r45/kt/run_kernel_trace.csv 10 > gpurun_out/r45/learner.txt
rm -f gpurun_out/r45/kt/run_kernel_trace.csv
cat gpurun_out/r45/learner.txt
