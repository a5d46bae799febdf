set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -p no:cacheprovider -k "mx8 or gemm" --timeout 300 --timeout-method thread > gpurun_out/mx8_tests.log 2>&1 || { grep -E "^FAILED|Error" gpurun_out/mx8_tests.log | head -20; tail -5 gpurun_out/mx8_tests.log; exit 1; }
tail -1 gpurun_out/mx8_tests.log
GB_MX8=1 GB_VARIANTS=14,0 timeout -k 10 500 python tools/gemm_bench.py > gpurun_out/mx8_ab.jsonl 2> gpurun_out/mx8_ab.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --linear-dtype mx8 > gpurun_out/mx8_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/mx8_bench.json')); print('mx8 r16', d['value'], d['ms_per_step'])"
