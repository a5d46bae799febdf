# Round 6: the final tree's bench lines: default (config 2), MXFP8 r = 32 (config 5), T2I (config 4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6l}
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['box_probe']['tflops'], d['box_probe']['clock_ghz_p10_p50_p90'])"
timeout -k 10 600 python -u bench.py --linear-dtype mx8 --lora-r 32 --no-cpu-baseline > gpurun_out/${TAG}_mx8_r32.json 2> gpurun_out/${TAG}_mx8_r32.err || { echo "MX8 FAILED"; tail -20 gpurun_out/${TAG}_mx8_r32.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_mx8_r32.json').read().splitlines()[-1]); print('mx8', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('box_probe',{}).get('tflops'))"
timeout -k 10 600 python -u bench.py --workload t2i > gpurun_out/${TAG}_t2i.json 2> gpurun_out/${TAG}_t2i.err || { echo "T2I FAILED"; tail -20 gpurun_out/${TAG}_t2i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_t2i.json').read().splitlines()[-1]); print('t2i', d['value'], d['roofline']['frac'], d.get('box_probe',{}).get('tflops'))"
