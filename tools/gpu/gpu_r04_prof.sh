# Round 4: rocprofv3 kernel trace + stats of the default bench (5 steps) and the per-step breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r4p}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py $(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1) 5 36 > gpurun_out/${TAG}_breakdown.txt
cp $(ls gpurun_out/${TAG}_prof/*kernel_stats.csv | head -1) gpurun_out/${TAG}_kernel_stats.csv
head -60 gpurun_out/${TAG}_breakdown.txt
rm -f gpurun_out/${TAG}_prof/*kernel_trace.csv
