# Round 5, verdict item 1: config 3's per-GPU workload (8 pairs per GPU, M = 9600) against the 4-pair
# line on the same box, alternating, then a rocprofv3 kernel trace of the 8-pair bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5a}
for i in 1 2; do
  for P in 4 8; do
    timeout -k 10 300 python -u bench.py --pairs-per-gpu $P --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper \
      > gpurun_out/${TAG}_p${P}_${i}.json 2> gpurun_out/${TAG}_p${P}_${i}.err \
      || { echo "BENCH p$P FAILED"; tail -20 gpurun_out/${TAG}_p${P}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" gpurun_out/${TAG}_p${P}_${i}.json p$P
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof8 -o p -- python bench.py --pairs-per-gpu 8 --steps 5 --warmup 2 --no-cpu-baseline --no-wrapper > gpurun_out/${TAG}_prof8.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/${TAG}_prof8.log; exit 1; }
python tools/prof_summary.py $(ls gpurun_out/${TAG}_prof8/*kernel_trace.csv | head -1) 5 40 > gpurun_out/${TAG}_breakdown8.txt
python tools/gemm_shapes_summary.py $(ls gpurun_out/${TAG}_prof8/*kernel_trace.csv | head -1) 5 > gpurun_out/${TAG}_gemm_shapes8.txt
cp $(ls gpurun_out/${TAG}_prof8/*kernel_stats.csv | head -1) gpurun_out/${TAG}_kernel_stats8.csv
head -45 gpurun_out/${TAG}_breakdown8.txt
cat gpurun_out/${TAG}_gemm_shapes8.txt
rm -f gpurun_out/${TAG}_prof8/*kernel_trace.csv
