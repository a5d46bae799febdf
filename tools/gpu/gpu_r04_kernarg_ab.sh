# Round 4: same-box step A/B of a HIP runtime setting (env), product library, alternating, 2 rounds.
# usage: ARMS="base HIP_FORCE_DEV_KERNARG=1" TAG=x bash tools/gpu/gpu_r04_kernarg_ab.sh
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-kargab}
for r in 1 2; do
 i=0
 for arm in $ARMS; do
  E=""; [ "$arm" != base ] && E="$arm"
  env $E timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${i}_$r.json 2> gpurun_out/${TAG}_${i}_$r.err || { tail -5 gpurun_out/${TAG}_${i}_$r.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/${TAG}_${i}_$r.json "$arm $r"
  i=$((i+1))
 done
done
