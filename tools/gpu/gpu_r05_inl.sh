# Round 5: the w4 GEMM's split-K tail summed inside its launch: kernel tests (incl. in-launch vs fixup bit
# identity), w4_check (w4 in-launch vs the SP8 kernel + fixup), then the step A/B against the fixup launch
# (ablation library, OSPO_GEMM_FIXUP=1), 2 alternating rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5k}
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mx8.py -m gpu -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/${TAG}_kernel_tests.log 2>&1 || { echo "KERNEL TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_kernel_tests.log | head -20; tail -5 gpurun_out/${TAG}_kernel_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_kernel_tests.log | tail -1
timeout -k 10 300 python -u tools/w4_check.py > gpurun_out/${TAG}_w4_check.log 2>&1 || { echo "W4 CHECK FAILED"; tail -5 gpurun_out/${TAG}_w4_check.log; exit 1; }
tail -1 gpurun_out/${TAG}_w4_check.log
for i in 1 2; do
  for V in inl fixup; do
    if [ $V = inl ]; then L=$PWD/ospo_amd/libospo_hip.so; else L=$PWD/ospo_amd/libospo_hip_ablation.so; fi
    OSPO_HIP_LIB=$L OSPO_GEMM_FIXUP=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['loss_first_step'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
