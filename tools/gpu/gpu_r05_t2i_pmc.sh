# Round 5, verdict r4 item 8: the T2I decode traffic over a whole 576-token image (the bench's own 575 decode
# steps at the bench's positions, eager so the counters are per dispatch), summarised -> gpurun_out/t2i_pmc_576.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T2I_PMC_TOKENS=576 bash tools/gpu/gpu_r04_t2i_pmc.sh || exit 1
# the generator's summary dict is the log's one line starting with '{' (rocprofv3 appends its own lines after it)
ARGS=$(python -c "import ast; l=[x for x in open('gpurun_out/t2i_pmc/FETCH_SIZE.log') if x.startswith('{')][-1]; d=ast.literal_eval(l); print(d['n_img'], d['prompt_len'], d['rows'])") || exit 1
python tools/t2i_pmc_summary.py gpurun_out/t2i_pmc $ARGS 2>&1 | tail -3 && cp profiles/t2i_pmc.json gpurun_out/t2i_pmc_576.json
rm -rf gpurun_out/t2i_pmc/FETCH_SIZE gpurun_out/t2i_pmc/WRITE_SIZE
