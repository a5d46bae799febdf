# Round 3 final tree: the builder-run lines of the other configs (config 5 MXFP8 r=32 and r=16, config 4 T2I,
# the drop-in wrapper workload)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for spec in "mx8_r32:--linear-dtype mx8 --lora-r 32" "mx8_r16:--linear-dtype mx8 --lora-r 16" "t2i:--workload t2i" "wrapper:--workload wrapper"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 500 python -u bench.py --no-cpu-baseline $args > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg_$tag.err || { echo "BENCH $tag FAILED"; tail -5 gpurun_out/cfg_$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))" gpurun_out/cfg_$tag.json $tag
done
