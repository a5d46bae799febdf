# Round 3: the fixed mx8 test, smoke, the bench, its rocprofv3 kernel stats, then the PMC passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3p3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_mx8.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -k rejects > gpurun_out/${TAG}_t.log 2>&1 || { echo "TEST FAILED"; tail -20 gpurun_out/${TAG}_t.log; exit 1; }
tail -1 gpurun_out/${TAG}_t.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "SMOKE FAILED"; tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-300 gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
echo prof ok
mkdir -p gpurun_out/pmc_bench
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timer"
for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $SET | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/pmc_bench/$tag -o p -- python bench.py $ARGS > gpurun_out/pmc_bench/$tag.log 2>&1 || { echo "PMC $tag FAILED"; tail -5 gpurun_out/pmc_bench/$tag.log; exit 1; }
  echo "pmc $tag ok"
done
