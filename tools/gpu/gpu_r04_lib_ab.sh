# Round 4: same-box step A/B of the in-tree library against ospo_amd/libospo_hip_base.so (built from the previous
# commit's sources), alternating, 2 rounds, after the GPU tests named by TESTK.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-libab}
if [ -n "$TESTK" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "$TESTK" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -5 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for r in 1 2; do
  for lib in base new; do
    L=$PWD/ospo_amd/libospo_hip.so; [ $lib = base ] && L=$PWD/ospo_amd/libospo_hip_base.so
    OSPO_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${lib}_$r.json 2> gpurun_out/${TAG}_${lib}_$r.err || { tail -5 gpurun_out/${TAG}_${lib}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/${TAG}_${lib}_$r.json "$lib $r"
  done
done
