# Round 5: same-box A/B of the default bench workload, alternating: r4hash = the round-4 dropout hash and GEMM
# epilogue (ospo_amd/libospo_hip_r4hash.so), r5nostage = the round-5 hash with the round-4 GEMM epilogue
# (libospo_hip_r5nostage.so, -DOSPO_W4_STAGE=0), new = the product library (round-5 hash + the w4 epilogue staged
# inside the last K-tile); then the reference's shipped configuration (16 pairs, LoRA r = 32) at 30 layers
# (verdict r4 item 7).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5c}
for i in 1 2; do
  for L in r4hash r5nostage new; do
    if [ $L = new ]; then unset OSPO_HIP_LIB; else export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_$L.so; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper \
      > gpurun_out/${TAG}_hash_${L}_${i}.json 2> gpurun_out/${TAG}_hash_${L}_${i}.err \
      || { echo "BENCH $L FAILED"; tail -20 gpurun_out/${TAG}_hash_${L}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['loss_first_step'])" gpurun_out/${TAG}_hash_${L}_${i}.json $L
  done
done
unset OSPO_HIP_LIB
timeout -k 10 600 python -u bench.py --pairs-per-gpu 16 --lora-r 32 --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/${TAG}_p16_r32.json 2> gpurun_out/${TAG}_p16_r32.err || { echo "BENCH p16 FAILED"; tail -20 gpurun_out/${TAG}_p16_r32.err; exit 1; }
cut -c1-600 gpurun_out/${TAG}_p16_r32.json
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('p16 r32', d['value'], d['ms_per_step'], d['drop_in_wrapper']['value'], d['roofline']['frac'])" gpurun_out/${TAG}_p16_r32.json
