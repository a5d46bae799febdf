# Round 6: the side stream's dA workgroups per CU (1 / 2 / 4) in the step, alternating, one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for w in 2 1 4; do
    OSPO_DA_WGS_PER_CU=$w timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper --no-box-probe > gpurun_out/da_ab_w${w}_$r.json 2> gpurun_out/da_ab_w${w}_$r.err || { echo "BENCH w$w FAILED"; tail -5 gpurun_out/da_ab_w${w}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/da_ab_w${w}_$r.json').read().splitlines()[-1]); print('wgs_per_cu $w round $r', d['value'], d['ms_per_step'], d['loss_first_step'])"
  done
done
