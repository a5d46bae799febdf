set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "swiglu_lora_gdb or lora_gdb or lora_da" > gpurun_out/nt_tests.log 2>&1 || { tail -5 gpurun_out/nt_tests.log; exit 1; }
tail -1 gpurun_out/nt_tests.log
AL=$PWD/ospo_amd/libospo_hip_ablation.so
for r in 1 2; do
 for v in base nt_da nt_gdb unfused; do
  E=""; X=""
  [ $v = nt_da ] && E="OSPO_NT_DA=1"
  [ $v = nt_gdb ] && E="OSPO_NT_GDB=1"
  [ $v = unfused ] && X="--lora-variant swiglu_gdb_unfused"
  env $E OSPO_HIP_LIB=$AL timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper $X > gpurun_out/nt_${v}_$r.json 2> gpurun_out/nt_${v}_$r.err || { tail -5 gpurun_out/nt_${v}_$r.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/nt_${v}_$r.json "$v $r"
 done
done
