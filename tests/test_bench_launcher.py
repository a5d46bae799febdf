"""bench.py's multi-rank launcher on CPU (gloo): ``python bench.py --gpus 2`` must start two
ranks by itself (torch.distributed.run as a child process), time the region with barrier + max
over ranks, and print ONE JSON line from rank 0 reporting n_gpus = 2.  The
stub workload exercises the same launcher / env / timing / all-reduce code as the GPU bench."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=240, env=env, cwd=ROOT)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_gpus2_launches_two_ranks():
    p = _run(["--gpus", "2", "--workload", "stub", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["steps"] == 3 and ln["warmup"] == 1
    assert ln["config"]["parallelism"] == "dp2" and ln["config"]["backend"] == "gloo"
    assert ln["config"]["pairs_per_gpu"] == 8 and ln["config"]["global_batch"] == 16  # config 3's per-GPU load
    assert ln["value"] > 0


def test_bench_single_process_default():
    p = _run(["--workload", "stub", "--steps", "2", "--warmup", "0", "--pairs-per-gpu", "3"])
    assert p.returncode == 0, p.stderr[-2000:]
    (ln,) = _json_lines(p.stdout)
    assert ln["n_gpus"] == 1 and ln["config"]["global_batch"] == 3


def test_bench_rejects_gpus_world_mismatch():
    p = _run(["--gpus", "4", "--workload", "stub"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE=2" in (p.stderr + p.stdout)


def test_t2i_traffic_field_from_committed_counter_pass():
    """The t2i line's roofline.traffic = its algorithmic bytes x the committed counter pass's measured /
    algorithmic ratio (profiles/t2i_pmc.json, written by tools/t2i_pmc_summary.py); the file's ratio is its own
    measured / algorithmic bytes and the decode kernels it counted are all present."""
    sys.path.insert(0, ROOT)
    import bench

    pmc = json.load(open(os.path.join(ROOT, "profiles", "t2i_pmc.json")))
    ratio = pmc["measured_bytes"] / pmc["algorithmic_bytes"]
    assert abs(ratio - pmc["traffic_ratio"]) < 1e-4
    assert 1.0 <= ratio < 2.0
    assert {"dlin_kernel", "attn_cache2_kernel"} <= set(pmc["per_kernel"])
    nbytes = 18_037_604_352
    assert bench.t2i_traffic(nbytes) == round(nbytes * pmc["traffic_ratio"])


def test_gemm_traffic_only_from_counter_passes_of_the_same_configuration():
    """roofline.traffic comes from the committed counter summary of the bench's own configuration (round 5: the
    8-pair and MXFP8 lines used to carry the default 4-pair line's bytes); a configuration without its own
    counter passes reports null."""
    sys.path.insert(0, ROOT)
    import bench
    default = bench.gemm_pmc_path(4, 30, 16, "bf16")
    assert os.path.basename(default) == "gemm_pmc.json" and os.path.exists(default)
    p8 = bench.gemm_pmc_path(8, 30, 16, "bf16")
    mx = bench.gemm_pmc_path(4, 30, 32, "mx8")
    assert os.path.basename(p8) == "gemm_pmc_bf16_p8_r16_l30.json"
    assert os.path.basename(mx) == "gemm_pmc_mx8_p4_r32_l30.json"
    assert len({default, p8, mx, bench.gemm_pmc_path(4, 2, 16, "bf16")}) == 4
