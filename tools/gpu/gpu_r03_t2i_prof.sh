# Round 3: per-kernel breakdown of the fused decode step (eager steps at mid-generation position)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-t2ip}
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG} -o p -- python tools/t2i_prof.py > gpurun_out/${TAG}.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}.log; exit 1; }
python tools/t2i_prof_summary.py $(ls gpurun_out/${TAG}/*kernel_trace.csv | head -1) 5 > gpurun_out/${TAG}_summary.txt
cat gpurun_out/${TAG}_summary.txt
rm -f gpurun_out/${TAG}/*kernel_trace.csv
