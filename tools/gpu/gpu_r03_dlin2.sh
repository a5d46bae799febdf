# Round 3: streaming decode Linear (dlin2): generate tests, T2I bench v2 / v1 (ablation lib, OSPO_DLIN_V1) / v2, kernel breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dl2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -s > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for run in v2a v1 v2b; do
  if [ $run = v1 ]; then export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so OSPO_DLIN_V1=1; else unset OSPO_HIP_LIB OSPO_DLIN_V1; fi
  timeout -k 10 400 python -u bench.py --workload t2i --no-cpu-baseline > gpurun_out/${TAG}_t2i_$run.json 2> gpurun_out/${TAG}_t2i_$run.err || { echo "T2I BENCH $run FAILED"; tail -5 gpurun_out/${TAG}_t2i_$run.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['avg_step_us'], d['roofline']['frac'], d.get('tokens_checksum'))" gpurun_out/${TAG}_t2i_$run.json $run
done
unset OSPO_HIP_LIB OSPO_DLIN_V1
TAG=${TAG}p bash tools/gpu/gpu_r03_t2i_prof.sh
