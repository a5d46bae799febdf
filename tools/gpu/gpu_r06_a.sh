# Round 6, first call: the new generator test, kernel tests, smoke, and the default bench line (box probe)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6a}
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 \
  || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -30; tail -15 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['box_probe'], d.get('cpu_baseline',{}).get('value'))"
