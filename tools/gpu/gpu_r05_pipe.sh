# Round 5: the pipelined decode Linear (dlin_pipe_kernel): decode tests (bit-identity vs the unfused GEMV),
# per-shape cold/warm times against dlin_kernel (ablation library, OSPO_DLIN_PIPE=0), T2I bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5q}
PROF=${PROF:-}
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gen_tests.log 2>&1 || { echo "GEN TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_gen_tests.log | head -20; tail -5 gpurun_out/${TAG}_gen_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_gen_tests.log | tail -1
timeout -k 10 240 python -u tools/dlin_warm_ab.py > gpurun_out/${TAG}_dlin_pipe.log 2>&1 || { echo "DLIN PIPE FAILED"; tail gpurun_out/${TAG}_dlin_pipe.log; exit 1; }
OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so OSPO_DLIN_PIPE=0 timeout -k 10 240 python -u tools/dlin_warm_ab.py > gpurun_out/${TAG}_dlin_nopipe.log 2>&1 || { echo "DLIN NOPIPE FAILED"; tail gpurun_out/${TAG}_dlin_nopipe.log; exit 1; }
echo pipe; grep shape gpurun_out/${TAG}_dlin_pipe.log; echo nopipe; grep shape gpurun_out/${TAG}_dlin_nopipe.log
for i in 1 2; do
  for V in pipe nopipe; do
    if [ $V = pipe ]; then L=$PWD/ospo_amd/libospo_hip.so; else L=$PWD/ospo_amd/libospo_hip_ablation.so; fi
    OSPO_HIP_LIB=$L OSPO_DLIN_PIPE=0 timeout -k 10 300 python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_t2i_${V}_${i}.json 2> gpurun_out/${TAG}_t2i_${V}_${i}.err || { echo "T2I $V FAILED"; tail -20 gpurun_out/${TAG}_t2i_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['avg_step_us'], d['roofline']['frac'], d['tokens_checksum'])" gpurun_out/${TAG}_t2i_${V}_${i}.json $V
  done
done
[ -z "$PROF" ] && exit 0
# per-kernel decode times of the product tree (rocprofv3 kernel stats over one T2I bench run)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python -u bench.py --workload t2i --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_t2i_prof.json 2> gpurun_out/${TAG}_t2i_prof.err || { echo "T2I PROF FAILED"; tail -20 gpurun_out/${TAG}_t2i_prof.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${TAG}_t2i_kernel_stats.csv
head -8 gpurun_out/${TAG}_t2i_kernel_stats.csv | cut -c1-160
find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" -delete
