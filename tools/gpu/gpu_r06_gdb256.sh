# Round 6: one-module lora_gdb groups on 256-row x 256-column workgroups -- kernel tests, the step / rank /
# shipped-config tests, the per-group micro A/B against the round-5 512-row blocks, and the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6g256}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gdb or lora" \
  > gpurun_out/${TAG}_ktests.log 2>&1 || { echo "KERNEL TESTS FAILED"; tail -40 gpurun_out/${TAG}_ktests.log; exit 1; }
tail -1 gpurun_out/${TAG}_ktests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_wrapper.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "STEP TESTS FAILED"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/gdb_bench.py 16 ",OSPO_GDB_RSB8" > gpurun_out/${TAG}_micro16.log 2>&1 || { echo "MICRO FAILED"; tail gpurun_out/${TAG}_micro16.log; exit 1; }
timeout -k 10 200 python -u tools/gdb_bench.py 32 "" > gpurun_out/${TAG}_micro32.log 2>&1 || { echo "MICRO32 FAILED"; tail gpurun_out/${TAG}_micro32.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_micro16.log gpurun_out/${TAG}_micro32.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['box_probe']['tflops'])"
