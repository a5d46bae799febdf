# Round 5 final: (WITH_SUITE=1: the whole GPU suite + smoke + default bench, gpu_r05_suite.sh), the rocprofv3 kernel stats of the
# default bench, the MXFP8 r = 32 line (config 5) and the T2I line (config 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5f}
[ -n "$WITH_SUITE" ] && { TAG=$TAG bash tools/gpu/gpu_r05_suite.sh || exit 1; }
TAG=${TAG}p bash tools/gpu/gpu_r05_prof.sh > /dev/null || exit 1
head -6 gpurun_out/${TAG}p_breakdown.txt
timeout -k 10 600 python -u bench.py --linear-dtype mx8 --lora-r 32 --no-cpu-baseline > gpurun_out/${TAG}_mx8_r32.json 2> gpurun_out/${TAG}_mx8_r32.err || { echo "MX8 BENCH FAILED"; tail -20 gpurun_out/${TAG}_mx8_r32.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_mx8_r32.json
timeout -k 10 600 python -u bench.py --workload t2i --no-cpu-baseline > gpurun_out/${TAG}_t2i.json 2> gpurun_out/${TAG}_t2i.err || { echo "T2I BENCH FAILED"; tail -20 gpurun_out/${TAG}_t2i.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_t2i.json
