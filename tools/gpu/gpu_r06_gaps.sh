# Round 6: main-queue gaps of the default bench under rocprofv3 (kernel trace only), summarised on the box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6gaps}
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wrapper --no-box-probe > gpurun_out/${TAG}_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
T=$(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1)
python tools/stream_gaps.py $T 5 > gpurun_out/${TAG}.txt
rm -f $T
cat gpurun_out/${TAG}.txt
