# HBM traffic + MFMA busy of the step's kernels, one counter group per rocprofv3 pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; PMC runs carry
# no trace domains).  Output: gpurun_out/pmc_bench/<counter>/...counter_collection.csv
# Round 5: BENCH_ARGS selects the bench configuration (e.g. "--pairs-per-gpu 8"), PMC_DIR the output directory.
set -o pipefail
D=${PMC_DIR:-gpurun_out/pmc_bench}
mkdir -p $D
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timer --no-wrapper $BENCH_ARGS"
for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  tag=$(echo $SET | cut -d' ' -f1)
  timeout -k 10 600 rocprofv3 --pmc $SET --output-format csv -d $D/$tag -o p -- python bench.py $ARGS > $D/$tag.log 2>&1 || { echo "PMC $tag FAILED"; tail -5 $D/$tag.log; exit 1; }
done
echo done
