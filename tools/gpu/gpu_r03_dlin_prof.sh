# kernel stats of the T2I bench, fused decode Linear vs the round-2 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dlp_new -o p -- python bench.py --workload t2i --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/dlp_new.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/dlp_new.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dlp_old -o p -- python bench.py --workload t2i --no-cpu-baseline --steps 1 --warmup 1 --t2i-unfused > gpurun_out/dlp_old.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/dlp_old.log; exit 1; }
rm -f gpurun_out/dlp_*/p_kernel_trace.csv gpurun_out/dlp_*/p_*trace*.csv
echo ok
