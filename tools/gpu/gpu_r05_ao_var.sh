# Round 5: attention + o in one launch, variants (ablation library, OSPO_ATTN_O_VAR): 0 the product form, 1 the o
# weights issued after the wait, 2 two workgroups per CU; against the two-launch step; 2 alternating rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5aov}
for i in 1 2; do
  for V in two v0 v1 v2; do
    if [ $V = two ]; then
      timeout -k 10 300 python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err || { echo "T2I $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    else
      OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so OSPO_ATTN_O_VAR=${V#v} timeout -k 10 300 python -u bench.py --workload t2i --steps 2 --warmup 1 --no-cpu-baseline --t2i-attn-o-one-launch > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err || { echo "T2I $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['avg_step_us'], d['roofline']['frac'], d['tokens_checksum'], d['config']['attn_o'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
