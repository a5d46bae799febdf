# Round 5: T2I decode Linear cold vs warm (tools/dlin_warm_ab.py), then the T2I bench under rocprofv3 kernel stats
# (the decode step's per-kernel durations on the current tree)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5t}
timeout -k 10 240 python -u tools/dlin_warm_ab.py > gpurun_out/${TAG}_dlin_warm.log 2>&1 || { echo "DLIN WARM FAILED"; tail gpurun_out/${TAG}_dlin_warm.log; exit 1; }
cat gpurun_out/${TAG}_dlin_warm.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python -u bench.py --workload t2i --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench_t2i.json 2> gpurun_out/${TAG}_bench_t2i.err || { echo "T2I PROF FAILED"; tail -20 gpurun_out/${TAG}_bench_t2i.err; exit 1; }
cut -c1-600 gpurun_out/${TAG}_bench_t2i.json
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_t2i_kernel_stats.csv
head -12 gpurun_out/${TAG}_t2i_kernel_stats.csv | cut -c1-200
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
