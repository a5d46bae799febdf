# Round 4: HBM traffic of the T2I decode kernels (bench generator, eager generate of T2I_PMC_TOKENS tokens), one
# counter per rocprofv3 pass, no trace domains; summary -> profiles/t2i_pmc.json (tools/t2i_pmc_summary.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t2i_pmc
export T2I_PMC_TOKENS=${T2I_PMC_TOKENS:-8}
RX="dlin_kernel|attn_cache2_kernel|cfg_sample_kernel|gen_aligner_in8_kernel|advance_kernel"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d gpurun_out/t2i_pmc/$C -o p -- python3 tools/t2i_pmc.py > gpurun_out/t2i_pmc/$C.log 2>&1 || { echo "PMC $C FAILED"; tail -5 gpurun_out/t2i_pmc/$C.log; exit 1; }
  tail -1 gpurun_out/t2i_pmc/$C.log
done
