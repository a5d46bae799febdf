set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r}
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo done
