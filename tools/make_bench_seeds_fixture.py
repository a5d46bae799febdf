"""Writes tests/golden/bench_config_seeds_oracle.npz (run on a GPU box): the bf16 and fp32 oracles' per-sequence
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
    runs, wc, dims, p, dig = bench_seed_runs()
    print(f"HIP forwards done ({time.time() - t0:.0f} s)", flush=True)
    ref = bench_seed_oracle(runs, wc, dims, p, lambda m: print(f"{m} ({time.time() - t0:.0f} s)", flush=True))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", "bench_config_seeds_oracle.npz")
    np.savez(out, digest=dig, hip=np.stack([r[3].float().numpy() for r in runs]), **ref)
    print("wrote", out, {k: v.tolist() for k, v in ref.items() if k.startswith("loss")}, flush=True)


if __name__ == "__main__":
    main()
