# Round 5: lora_gdb ring depth per shape (tools/gdb_bench.py, ablation library knobs), 2 alternating rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for V in default OSPO_GDB_NS6 OSPO_GDB_NS3 OSPO_NT_GDB; do
    if [ $V = default ]; then
      timeout -k 10 120 python -u tools/gdb_bench.py > gpurun_out/r5gdb_${V}_${i}.json 2> gpurun_out/r5gdb_${V}_${i}.err || { echo "GDB $V FAILED"; tail -5 gpurun_out/r5gdb_${V}_${i}.err; exit 1; }
    else
      env $V=1 timeout -k 10 120 python -u tools/gdb_bench.py > gpurun_out/r5gdb_${V}_${i}.json 2> gpurun_out/r5gdb_${V}_${i}.err || { echo "GDB $V FAILED"; tail -5 gpurun_out/r5gdb_${V}_${i}.err; exit 1; }
    fi
    echo "$V $(cat gpurun_out/r5gdb_${V}_${i}.json)"
  done
done
