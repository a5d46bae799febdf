"""Writes tests/golden/bench_config_seeds_oracle.npz (run on a GPU box; with --mx8 the config-5 fixture
tests/golden/bench_mx8_r32_seed_oracle.npz instead: MXFP8 Linears, LoRA r = 32, batch 0, the oracle's fp8 mode): the bf16 and fp32 oracles' per-sequence
log-probs and SimPO losses of the bench workload's batches 0, 1, 2 (tests/test_gpu_step.py bench_seed_oracle, the
HIP path's dropout masks replayed), with the digest of every weight and input that pins them to the workload
(the weights are drawn on the device by bench.simpo_setup).  The test recomputes the oracles when the digest
differs.  Output: gpurun_out/bench_config_seeds_oracle.npz (copied into tests/golden/ by hand)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from tests.test_gpu_step import bench_seed_oracle, bench_seed_runs  # noqa: E402


def main():
    t0 = time.time()
    mx8 = "--mx8" in sys.argv  # config 5: MXFP8 Linears, LoRA r = 32, batch 0 only, the oracle's fp8 mode
    setup = dict(n_seeds=1, lora_r=32, linear_dtype="mx8") if mx8 else {}
    runs, wc, dims, p, dig = bench_seed_runs(**setup)
    print(f"HIP forwards done ({time.time() - t0:.0f} s)", flush=True)
    ref = bench_seed_oracle(runs, wc, dims, p, lambda m: print(f"{m} ({time.time() - t0:.0f} s)", flush=True),
                            mx8=mx8)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", "bench_mx8_r32_seed_oracle.npz" if mx8 else "bench_config_seeds_oracle.npz")
    np.savez(out, digest=dig, hip=np.stack([r[3].float().numpy() for r in runs]), **ref)
    print("wrote", out, {k: v.tolist() for k, v in ref.items() if k.startswith("loss")}, flush=True)


if __name__ == "__main__":
    main()
