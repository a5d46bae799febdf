# Round 5: T2I kernel stats on the current tree (sampler rewrite), one bench run under rocprofv3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5u}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_t2i.json 2> gpurun_out/${TAG}_t2i.err || { echo "T2I PROF FAILED"; tail -20 gpurun_out/${TAG}_t2i.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_t2i_kernel_stats.csv
grep -E "cfg_sample|gen_aligner|advance|dlin" gpurun_out/${TAG}_t2i_kernel_stats.csv | cut -c1-200
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
