# Round 3 final tree: GPU suite + smoke, step A/B against the base library (alternating), the default bench line,
# rocprofv3 kernel stats of 5 steps and their per-step breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-fin}
NO_BENCH=1 TAG=$TAG bash tools/gpu/gpu_r03_suite.sh || exit 1
if [ -f ospo_amd/libospo_hip_base.so ]; then
  for r in 1 2; do
    for lib in base new; do
      L=$PWD/ospo_amd/libospo_hip.so; [ $lib = base ] && L=$PWD/ospo_amd/libospo_hip_base.so
      OSPO_HIP_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_ab_${lib}_$r.json 2> gpurun_out/${TAG}_ab_${lib}_$r.err || { echo "AB BENCH FAILED"; tail -5 gpurun_out/${TAG}_ab_${lib}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss'))" gpurun_out/${TAG}_ab_${lib}_$r.json "$lib $r"
    done
  done
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
python tools/prof_summary.py $(ls gpurun_out/${TAG}_prof/*kernel_trace.csv | head -1) 5 36 > gpurun_out/${TAG}_breakdown.txt
head -12 gpurun_out/${TAG}_breakdown.txt
rm -f gpurun_out/${TAG}_prof/*kernel_trace.csv
