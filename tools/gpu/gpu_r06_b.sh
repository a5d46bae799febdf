# Round 6: the bench-config oracle fixture (6 CPU oracle passes), the default bench line, and the step's kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r6b}
timeout -k 10 900 python -u tools/make_bench_seeds_fixture.py 2>&1 | tee gpurun_out/${TAG}_fixture.log || { echo "FIXTURE FAILED"; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['box_probe'], d.get('cpu_baseline',{}).get('value'))"
TAG=${TAG} bash tools/gpu/gpu_r05_prof.sh
