# Round 4: the step with the w4 GEMM (ablation lib default) against the round-3 SP8 kernel (variant 27),
# same box, alternating; then the w4 isolated A/B (tools/w4_check.py timing)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-gab}
export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so
for r in 1 2; do
  for v in 27 0; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --gemm-variant $v > gpurun_out/${TAG}_v${v}_$r.json 2> gpurun_out/${TAG}_v${v}_$r.err || { echo "BENCH FAILED"; tail -5 gpurun_out/${TAG}_v${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss_first_step'))" gpurun_out/${TAG}_v${v}_$r.json "v$v r$r"
  done
done
