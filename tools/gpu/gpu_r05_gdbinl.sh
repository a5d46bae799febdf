# Round 5: lora_gdb's g partials summed in the launch: kernel tests (exact integers, == the reduce launch via
# swiglu_lora_gdb, counters left zero), step parity tests, then the default bench A/B against the reduce launch
# (ablation library, OSPO_GDB_INL=1), 2 alternating rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5gi}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "gdb" > gpurun_out/${TAG}_kern.log 2>&1 || { echo "KERNEL TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_kern.log | head -20; tail -5 gpurun_out/${TAG}_kern.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_kern.log | tail -1
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -v -p no:cacheprovider -rf --timeout 300 --timeout-method thread -k "bench_config_first_step or 8_pairs or dropout_vs_oracle or gdb_gu_only" > gpurun_out/${TAG}_step.log 2>&1 || { echo "STEP TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_step.log | head -20; tail -5 gpurun_out/${TAG}_step.log; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_step.log | tail -1
for i in 1 2; do
  for V in inl launch; do
    E=""; [ $V = inl ] && E="OSPO_GDB_INL=1"
    env OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so $E timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('loss_first_step'))" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
