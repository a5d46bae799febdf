# Round 5: rocprofv3 kernel trace + stats of the default bench (5 steps): per-kernel breakdown, GEMM per shape,
# main-queue idle gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5p}
A=${PROF_ARGS:-}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wrapper --no-box-probe $A > gpurun_out/${TAG}_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
T=$(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1)
python tools/prof_summary.py $T 5 45 > gpurun_out/${TAG}_breakdown.txt
python tools/gemm_shapes_summary.py $T 5 > gpurun_out/${TAG}_gemm_shapes.txt
cp $(ls gpurun_out/${TAG}_prof/*kernel_stats.csv | head -1) gpurun_out/${TAG}_kernel_stats.csv
head -50 gpurun_out/${TAG}_breakdown.txt
cat gpurun_out/${TAG}_gemm_shapes.txt
rm -f $T
