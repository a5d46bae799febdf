# Same-box A/B: the round-2 final tree (r2base/, commit 2cefa39, its own library) against this tree, alternating;
# then the lora_gdb ring-depth sweep (ablation build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  (cd r2base && timeout -k 10 400 python -u bench.py --no-cpu-baseline > ../gpurun_out/r2r3_r2_$r.json 2> ../gpurun_out/r2r3_r2_$r.err) || { echo "R2 BENCH FAILED"; tail -5 gpurun_out/r2r3_r2_$r.err; exit 1; }
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r2r3_r3_$r.json 2> gpurun_out/r2r3_r3_$r.err || { echo "R3 BENCH FAILED"; tail -5 gpurun_out/r2r3_r3_$r.err; exit 1; }
  for t in r2 r3; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d.get('loss'))" gpurun_out/r2r3_${t}_$r.json "$t $r"; done
done
for ns in 4 2 3; do
  unset OSPO_GDB_NS2 OSPO_GDB_NS3; [ $ns = 2 ] && export OSPO_GDB_NS2=1; [ $ns = 3 ] && export OSPO_GDB_NS3=1
  echo "gdb NS=$ns $(timeout -k 10 120 python -u tools/gdb_bench.py 2>&1 | grep -v amdgpu.ids)"
done
