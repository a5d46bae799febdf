# Round 4: same-box step A/B of ablation-library knobs (env), alternating, 2 rounds.
# usage: ARMS="base OSPO_SK3_NT=1 OSPO_SK3_NT=2" TAG=x bash tools/gpu/gpu_r04_env_ab.sh
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-envab}
AL=$PWD/ospo_amd/libospo_hip_ablation.so
for r in 1 2; do
 i=0
 for arm in $ARMS; do
  E=""; [ "$arm" != base ] && E="$arm"
  env $E OSPO_HIP_LIB=$AL timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${i}_$r.json 2> gpurun_out/${TAG}_${i}_$r.err || { tail -5 gpurun_out/${TAG}_${i}_$r.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_${i}_$r.json "$arm $r"
  i=$((i+1))
 done
done
