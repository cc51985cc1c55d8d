"""CPU checks of the measurement evidence: the decode-layer traffic tool counts
every dispatch of a layer window, refuses passes without the layer's five kernel classes, and
bench.py never publishes a PMC traffic figure below the algorithmic bytes."""
import csv
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import decode_traffic  # noqa: E402

LAYER = [("void qlin_gv::gemv_fast_kernel<4, 1, 1, 0, 0, 4, 2>(qlin_gv::FastArgs)", 13.6e6),
         ("void (anonymous namespace)::attn_decode_kernel<4, true>(AttnArgs)", 2.5e6),
         ("void qlin_gv::gemv_fast_kernel<4, 1, 1, 0, 1, 2, 0>(qlin_gv::FastArgs)", 9.1e6),
         ("void qlin_gv::gemv_wq_kernel<4, 1, 0, 2>(qlin_gv::WqArgs)", 62.0e6),
         ("void qlin_gv::gemv_rows_kernel<4, 1, 0, 8, 8, 0>(qlin_gv::RowsArgs)", 31.6e6)]


def _write_pass(path, layers, layer=LAYER, prologue=3):
    """A counter_collection.csv as rocprofv3 writes it: setup dispatches, then `layers` layer
    passes (FETCH_SIZE in KiB, half the bytes: the tool's x 1024 x 2)."""
    os.makedirs(path, exist_ok=True)
    rows, did = [], 1
    for _ in range(prologue):
        rows.append((did, "void qlin_quantize_kernel<...>()", 1.0e6))
        did += 1
    for _ in range(layers):
        for name, b in layer:
            rows.append((did, name, b))
            did += 1
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Correlation_Id", "Dispatch_Id", "Kernel_Name", "Counter_Name",
                    "Counter_Value"])
        for d, name, b in rows[::-1]:  # file order need not be dispatch order
            w.writerow([d, d, name, "FETCH_SIZE", b / 2048])


def test_decode_traffic_counts_every_kernel(tmp_path):
    _write_pass(str(tmp_path / "pmc"), 12)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "decode_traffic.py"),
                    str(tmp_path / "pmc"), str(out)], check=True, capture_output=True)
    d = json.loads(out.read_text())
    assert d["kernel_classes"] == 5 and d["layers_dispatched"] == 12
    assert d["fetch_bytes_per_layer"] == pytest.approx(sum(b for _, b in LAYER))
    assert d["per_class_mean_bytes"]["gate_up_norm_silu"] == pytest.approx(62.0e6)
    assert "gemv_wq_kernel" in d["per_class_kernel"]["gate_up_norm_silu"]


def test_decode_traffic_refuses_a_four_kernel_layer(tmp_path):
    _write_pass(str(tmp_path / "pmc"), 8, layer=[LAYER[0], LAYER[1], LAYER[2], LAYER[4]])
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "decode_traffic.py"),
                        str(tmp_path / "pmc"), str(tmp_path / "o.json")], capture_output=True)
    assert r.returncode != 0 and b"five kernel classes" in r.stderr


def test_decode_traffic_refuses_ragged_windows(tmp_path):
    _write_pass(str(tmp_path / "pmc"), 6)
    rows = decode_traffic._rows(str(tmp_path / "pmc"))
    for at in (27, 17, 7):  # another kernel inside three of the six layers: no dominant shape
        rows.insert(at, (10**6 + at, "void at::native::elementwise_kernel<...>", 1.0))
    with pytest.raises(SystemExit):
        decode_traffic.layer_windows(rows)


def test_decode_traffic_leaves_out_the_eager_pass(tmp_path):
    """One eager warm-up layer with two extra host-side torch kernels among 12 replayed ones: that
    window is left out, never mixed into the bytes per layer."""
    _write_pass(str(tmp_path / "pmc"), 12)
    rows = decode_traffic._rows(str(tmp_path / "pmc"))
    rows[8:8] = [(-1, "void at::native::elementwise_kernel<...>", 5e6)] * 2  # after layer 0
    wins = decode_traffic.layer_windows(rows)
    assert len(wins) == 11 and all(len(w) == 5 for w in wins)
    assert sum(r[2] for r in wins[0]) == pytest.approx(sum(b for _, b in LAYER))


def test_bench_never_publishes_traffic_below_algorithmic_bytes():
    sys.path.insert(0, ROOT)
    import bench
    r = {}
    bench._attach_traffic(r, {"fetch_bytes_per_launch": 56.8e6, "file": "x.json"}, 116.4e6)
    assert r["traffic"] is None and "incomplete" in r["traffic_rejected"]
    r = {}
    bench._attach_traffic(r, {"fetch_bytes_per_launch": 119.7e6, "file": "x.json"}, 116.4e6)
    assert r["traffic"] == 119700000 and 1.0 <= r["traffic_ratio"] <= 1.1


def _newest(pattern):
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    assert files, pattern
    return files[-1]


def test_committed_decode_layer_pmc_has_every_kernel():
    """The newest committed decode-layer PMC pass (the file bench.py publishes as the decode
    line's roofline.traffic) has the five kernel classes and at least the layer's algorithmic
    bytes, within 10 %."""
    sys.path.insert(0, ROOT)
    import bench
    from transformers import LlamaConfig
    d = json.load(open(_newest("r*_decode_layer_int4_g128_pmc.json")))
    assert d.get("kernel_classes", 0) >= 5, d
    cfg = LlamaConfig(hidden_size=4096, intermediate_size=14336, num_attention_heads=32,
                      num_key_value_heads=8)
    algo, _ = bench.decode_layer_bytes(cfg, 513)
    assert 1.0 <= d["fetch_bytes_per_layer"] / algo <= 1.1, (d["fetch_bytes_per_layer"], algo)


def test_bench_scales_traffic_to_the_lines_launch_size():
    """A pass taken at one ring size published on a line at another (round 6: the two-rank
    rehearsal's 8-product launches carried the 64-product pass, 8.1x algorithmic) is scaled per
    product; a pass without its launch size is not published on a batched line."""
    sys.path.insert(0, ROOT)
    import bench
    algo1 = bench.algo_bytes(1, 4096, 4096, 4, 128)
    pmc = {"fetch_bytes_per_launch": 1.0145 * algo1 * 64, "products_per_launch": 64,
           "file": "x.json"}
    r = {}
    bench._attach_traffic(r, dict(pmc), algo1 * 8, 8)
    assert r["traffic_ratio"] == pytest.approx(1.0145, abs=1e-4) and "64" in r["traffic_scaled"]
    r = {}
    bench._attach_traffic(r, dict(pmc), algo1 * 64, 64)
    assert "traffic_scaled" not in r and r["traffic_ratio"] == pytest.approx(1.0145, abs=1e-4)
    r = {}
    bench._attach_traffic(r, {"fetch_bytes_per_launch": 5e8, "file": "x.json"}, algo1 * 8, 8)
    assert r["traffic"] is None and "not recorded" in r["traffic_rejected"]


@pytest.mark.parametrize("workload", ["gemv_int4_g128", "gemv_int3_g64", "gemv_int2_g64",
                                      "gemv_int3_g64_hqq", "gemv_int2_g64_hqq"])
def test_committed_ring_pmc_per_product(workload):
    """The newest committed batched-ring PMC pass of each GEMV workload reads every algorithmic
    byte once, within 10 %, per product of the launch size it records."""
    sys.path.insert(0, ROOT)
    import bench
    M, N, K, bits, group, ring, _, _ = bench.WORKLOADS[workload]
    d = json.load(open(_newest(f"r*_{workload}_batched_pmc.json")))
    assert d["products_per_launch"] == ring, d
    ratio = d["fetch_bytes_per_launch"] / ring / bench.algo_bytes(M, N, K, bits, group)
    assert 1.0 <= ratio <= 1.1, ratio
