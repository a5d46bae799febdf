# LoRA weight-gradient products: tests, then the current tiles vs the streaming kernel at several grid sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -k "wgrad or f32acc" --timeout 120 --timeout-method thread > gpurun_out/wgrad_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/wgrad_tests.log | head; tail -3 gpurun_out/wgrad_tests.log; exit 1; }
tail -1 gpurun_out/wgrad_tests.log
for w in 0 64 128 160 256 384; do
  OSPO_WGRAD_WGS=$w timeout -k 10 120 python tools/lora_grads_bench.py 2>/dev/null | tail -1 || { echo "BENCH FAILED $w"; exit 1; }
done
