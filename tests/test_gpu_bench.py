"""bench.py's multi-rank path (the driver's 1/2/4/8-GPU scaling runs): ``--gpus N`` without a
launcher starts N rank processes itself, and the rank-0 JSON line reports the whole job.

Rehearsed on one MI355X with two ranks sharing the card (BENCH_DIST_BACKEND=gloo,
BENCH_SHARE_GPU=1: the barrier and the max-over-ranks reduction go through gloo; the driver's
multi-GPU runs use RCCL, one rank per GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, extra_env=None, timeout=600):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # ONE JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("split", [False, True])
def test_bench_gpus2_spawns_ranks(split):
    """--gpus 2 (weak: an independent ring per rank; --split: output rows of one shared ring):
    two ranks ran, n_gpus is 2 and value is the whole-job throughput."""
    args = ["--gpus", "2", "--steps", "6", "--warmup", "2", "--ring", "16", "--ramp-s", "0.05",
            "--no-cpu-baseline", "--no-decode-layer", "--no-other-mode", "--pipeline", "off"]
    if split:
        args.append("--split")
    d = _bench(*args, extra_env={"BENCH_DIST_BACKEND": "gloo", "BENCH_SHARE_GPU": "1"})
    assert d["n_gpus"] == 2
    assert d["scaling"] == ("strong" if split else "weak")
    assert d["config"]["ring"] == 16 and d["steps"] == 6
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value = all ranks' products / the max-over-ranks time
    per_rank_products = 16 * 6
    flops = 2.0 * 4096 * 4096 * per_rank_products * (1 if split else 2)
    if split:  # N_per_rank rows each: the job is the one shared ring
        assert d["config"]["N_per_rank"] == 2048
    got = flops / (d["ms_per_step"] * 6 / 1e3) / 1e12
    assert abs(got - d["value"]) <= 0.02 * d["value"] + 1e-3, (got, d["value"])


@pytest.mark.timeout(1100)
def test_bench_gpus2_pipeline_leg():
    """The configs[4] leg the driver's multi-GPU runs add to the line: with
    two ranks the 32 LLaMA3-8B layers run as 2 pipeline stages (here gloo + one shared MI355X;
    RCCL over xGMI, one rank per GPU, in the driver's runs), windows in flight and graph-replayed
    decode steps are timed, and the pipeline's NLL and greedy tokens equal one process bit for
    bit."""
    d = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--ring", "8", "--ramp-s", "0.05",
               "--no-cpu-baseline", "--no-decode-layer", "--no-other-mode", "--pipe-windows", "2",
               "--pipe-decode", "8", extra_env={"BENCH_DIST_BACKEND": "gloo",
                                                 "BENCH_SHARE_GPU": "1"}, timeout=1000)
    assert d["n_gpus"] == 2
    p = d["pipeline"]
    assert p["stages"] == [[0, 16], [16, 32]] and p["backend"] == "gloo"
    assert p["windows"]["ms_per_window"] > 0 and p["decode"]["ms_per_step"] > 0
    assert p["check"]["nll_bit_identical_to_one_process"], p["check"]
    assert p["check"]["tokens_identical_to_one_process"], p["check"]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("workload,bound", [("gemv_int4_g128_a8", "hbm"),
                                            ("gemm_int4_g128_a8_m2048", "mfma")])
def test_bench_act_quant_workloads(workload, bound):
    """SURVEY §8(f) row f3 measured like the other rows: the W4A8 linear (per-token 8-bit act
    fake-quant of x, quant/int_linear.py:59-60) through qlin_linear_ep_f16 — fused into the GEMV
    blocks at one token, the quantizer kernel + MFMA GEMM at a 2048-token window."""
    d = _bench("--workload", workload, "--steps", "4", "--warmup", "2", "--ramp-s", "0.05",
               "--no-cpu-baseline")
    assert d["n_gpus"] == 1 and d["config"]["workload"] == workload
    assert d["value"] > 0 and d["roofline"]["bound"] == bound and 0 < d["roofline"]["frac"] < 1
