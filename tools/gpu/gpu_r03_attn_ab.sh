# Round 3: attention tests on the product lib, then dK/dV A/B (base lib vs product lib, alternating): attn_bench
# and the default bench; stamps on the ablation lib
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-aab}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "flash or attn" > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for r in 1 2; do
  for lib in ${ATTN_LIBS:-base new}; do
    L=$PWD/ospo_amd/libospo_hip.so; [ $lib != new ] && L=$PWD/ospo_amd/libospo_hip_$lib.so
    OSPO_HIP_LIB=$L timeout -k 10 120 python -u tools/attn_bench.py > gpurun_out/${TAG}_ab_${lib}_$r.json 2>&1 || { echo "ATTN BENCH FAILED"; tail -5 gpurun_out/${TAG}_ab_${lib}_$r.json; exit 1; }
    echo "$lib $r $(tail -1 gpurun_out/${TAG}_ab_${lib}_$r.json | cut -c1-300)"
  done
done
timeout -k 10 120 python -u tools/attn_stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1 || { echo "STAMPS FAILED"; tail -5 gpurun_out/${TAG}_stamps.txt; exit 1; }
cat gpurun_out/${TAG}_stamps.txt
[ -n "$NO_STEP" ] && exit 0
for r in 1 2; do
  for lib in base new; do
    L=$PWD/ospo_amd/libospo_hip.so; [ $lib = base ] && L=$PWD/ospo_amd/libospo_hip_base.so
    OSPO_HIP_LIB=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_${lib}_$r.json 2> gpurun_out/${TAG}_bench_${lib}_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_bench_${lib}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('loss'))" gpurun_out/${TAG}_bench_${lib}_$r.json "$lib $r"
  done
done
