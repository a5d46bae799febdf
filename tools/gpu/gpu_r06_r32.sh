# Round 6: LoRA r = 32 fused g/dB streams -- kernel tests, r = 32 step/wrapper/MXFP8 parity, and a same-box
# A/B of the MXFP8 r = 32 bench line with the r = 32 fusion on (default) and off (--lora-variant gdb_unfused)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6r32}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gdb" > gpurun_out/${TAG}_ktests.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -40 gpurun_out/${TAG}_ktests.log; exit 1; }
tail -1 gpurun_out/${TAG}_ktests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_step.py::test_step_lora_rank_variants_vs_oracle" \
  tests/test_gpu_step.py::test_step_mx8_full_size_7b_shapes_lora_r32 \
  tests/test_gpu_step.py::test_bench_mx8_r32_30_layers_gross_errors \
  tests/test_gpu_wrapper.py::test_wrapper_shipped_config_16_pairs_r32_dropout_7b_widths_vs_oracle \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
[ -n "$SKIP_AB" ] || for v in on off on off; do
  if [ $v = on ]; then LV=""; else LV="gdb_unfused"; fi
  timeout -k 10 600 python -u bench.py --linear-dtype mx8 --lora-r 32 --no-cpu-baseline --no-wrapper --lora-variant "$LV" \
    > gpurun_out/${TAG}_mx8_${v}.json 2> gpurun_out/${TAG}_mx8_${v}.err || { echo "MX8 $v FAILED"; tail -20 gpurun_out/${TAG}_mx8_${v}.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${TAG}_mx8_${v}.json').read().splitlines()[-1]); print('mx8 r32 fusion=$v', d['value'], d['ms_per_step'], d.get('box_probe',{}).get('tflops'))"
done
[ -z "$PROF" ] || TAG=${TAG}_prof PROF_ARGS="--linear-dtype mx8 --lora-r 32" bash tools/gpu/gpu_r05_prof.sh
