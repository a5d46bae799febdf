# Round 5, verdict r4 item 2c: do HF's two bf16 score roundings matter for parity?  The 30-layer parity tests with the
# ablation library's unrounded-score attention (OSPO_ATTN_RAW_SCORES=1: forward and dK/dV), parity log only (their
# bounds may or may not hold: that is the measurement); then attention timing with and without the roundings.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5raw}
export OSPO_PARITY_LOG=gpurun_out/${TAG}_parity.jsonl
rm -f $OSPO_PARITY_LOG
OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so OSPO_ATTN_RAW_SCORES=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py -m gpu -v -p no:cacheprovider -rf -s --timeout 600 --timeout-method thread \
  -k "full_depth or bench_config or full_size_7b_shapes_two_layers" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || { echo "RAW TESTS ERROR rc=$rc"; tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
for V in hf raw; do
  if [ $V = raw ]; then export OSPO_ATTN_RAW_SCORES=1; else unset OSPO_ATTN_RAW_SCORES; fi
  OSPO_ATTN_WAVES=4 timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/${TAG}_attn_${V}.log 2>&1 || { echo "ATTN BENCH FAILED"; tail gpurun_out/${TAG}_attn_${V}.log; exit 1; }
  echo $V $(tail -1 gpurun_out/${TAG}_attn_${V}.log)
done
unset OSPO_ATTN_RAW_SCORES
