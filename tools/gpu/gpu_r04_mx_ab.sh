# Round 4: config-5 (MXFP8 decoder Linears, LoRA r = 32) step A/B, in-tree library against
# ospo_amd/libospo_hip_base.so (previous commit), alternating, 2 rounds.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-mxab}
for r in 1 2; do
  for lib in base new; do
    L=$PWD/ospo_amd/libospo_hip.so; [ $lib = base ] && L=$PWD/ospo_amd/libospo_hip_base.so
    OSPO_HIP_LIB=$L timeout -k 10 200 python -u bench.py --linear-dtype mx8 --lora-r 32 --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_${lib}_$r.json 2> gpurun_out/${TAG}_${lib}_$r.err || { tail -5 gpurun_out/${TAG}_${lib}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" gpurun_out/${TAG}_${lib}_$r.json "$lib $r"
  done
done
