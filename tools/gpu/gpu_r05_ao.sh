# Round 5: the cached attention + o in one launch: generate tests (incl. one launch == two launches bit for
# bit), then the T2I bench A/B against two launches, 2 alternating rounds (tokens checksums must agree)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5ao}
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gen_tests.log 2>&1 || { echo "GEN TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_gen_tests.log | head -20; tail -5 gpurun_out/${TAG}_gen_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_gen_tests.log | tail -1
for i in 1 2; do
  for V in one two; do
    A=""; [ $V = one ] && A="--t2i-attn-o-one-launch"
    timeout -k 10 300 python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline $A > gpurun_out/${TAG}_t2i_${V}_${i}.json 2> gpurun_out/${TAG}_t2i_${V}_${i}.err || { echo "T2I $V FAILED"; tail -20 gpurun_out/${TAG}_t2i_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['avg_step_us'], d['roofline']['frac'], d['tokens_checksum'], d['config']['attn_o'])" gpurun_out/${TAG}_t2i_${V}_${i}.json $V
  done
done
