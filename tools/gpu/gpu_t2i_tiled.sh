set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -q -m gpu -p no:cacheprovider -rf --timeout 300 --timeout-method thread > gpurun_out/t1_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" gpurun_out/t1_tests.log | head -20; tail -3 gpurun_out/t1_tests.log; exit 1; }
tail -1 gpurun_out/t1_tests.log
timeout -k 10 300 python -u tools/t2i_tiled_ab.py > gpurun_out/t1_ab.jsonl 2> gpurun_out/t1_ab.err || { echo "AB FAILED"; tail -5 gpurun_out/t1_ab.err; exit 1; }
cat gpurun_out/t1_ab.jsonl
timeout -k 10 400 python bench.py --workload t2i > gpurun_out/t1_t2i.json 2> gpurun_out/t1_t2i.err || { echo "T2I BENCH FAILED"; tail -5 gpurun_out/t1_t2i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/t1_t2i.json')); print('images/s', d['value'], 'step us', d['roofline']['avg_step_us'], 'frac', d['roofline']['frac'], 'tok', d['tokens_checksum'], 'pix', d['pixels_checksum'])"
