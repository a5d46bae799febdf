# Round 5: generate tests (sampler without scratch: tokens bit-exact vs the oracle), decode Linear split A/B, T2I bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/r5v_gen_tests.log 2>&1 || { echo "GEN TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r5v_gen_tests.log | head -20; tail -5 gpurun_out/r5v_gen_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r5v_gen_tests.log | tail -1
timeout -k 10 400 python -u tools/dlin_split_ab.py > gpurun_out/r5v_dlin_split.log 2>&1 || { echo "SPLIT AB FAILED"; tail gpurun_out/r5v_dlin_split.log; exit 1; }
grep shape gpurun_out/r5v_dlin_split.log
timeout -k 10 300 python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r5v_t2i.json 2> gpurun_out/r5v_t2i.err || { echo "T2I FAILED"; tail -20 gpurun_out/r5v_t2i.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('t2i', d['value'], d['roofline']['avg_step_us'], d['roofline']['frac'], d['tokens_checksum'])" gpurun_out/r5v_t2i.json
