"""Measurement tooling on the CPU: tools/traffic.py turns rocprofv3 FETCH_SIZE / WRITE_SIZE
counter rows into bytes per read per kernel (gfx950's halved FETCH_SIZE doubled), and sums a
step's multi-k k_map1 passes into the "k_map1 xN passes" entry bench.py names its dominant kernel."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"]
PASS = "void skq::k_map1<16, 4, 0, true, false>(skq::SketchParams, skq::ChainParams)"
FINAL = "void skq::k_map1<16, 4, 0, true, true>(skq::SketchParams, skq::ChainParams)"
ONE = "void skq::k_map1<16, 4, 0>(skq::SketchParams, skq::ChainParams)"


def _write(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HDR)
        for did, name, grid, val in rows:
            # two rows per dispatch (the counter per XCD instance): traffic.py adds them
            w.writerow([did, name, grid, counter, val / 2])
            w.writerow([did, name, grid, counter, val / 2])


def test_traffic_sums_multi_k_passes(tmp_path):
    g = 1000
    # two steps of three passes (1, 2, 4 kB per thread), a small sample launch, one k_bin_sum
    rows = [(1, PASS, g, 1.0 * g), (2, PASS, g, 2.0 * g), (3, FINAL, g, 4.0 * g),
            (4, PASS, g, 1.0 * g), (5, PASS, g, 2.0 * g), (6, FINAL, g, 4.0 * g),
            (7, PASS, 100, 50.0), (8, FINAL, 100, 90.0),
            (9, "skq::k_bin_sum(unsigned long*)", 64, 64.0)]
    _write(str(tmp_path / "F"), "FETCH_SIZE", rows)
    _write(str(tmp_path / "W"), "WRITE_SIZE", [(d, n, gg, v / 8) for d, n, gg, v in rows])
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), "cfg5", str(tmp_path / "F"),
                    str(tmp_path / "W"), str(out), "k_map1 x3 passes=450"], check=True, capture_output=True)
    k = json.load(open(out))["kernels"]
    mp = k["k_map1 x3 passes"]
    assert mp["dispatches"] == [2, 2]
    # calibrated (profiles/r3_fetch_calibration.json): FETCH_SIZE as tallied (64 B per request) plus
    # half the streamed bytes (streamed requests move 128 B)
    assert mp["fetch_size_bytes_per_read"] == 7.0 * 1024  # (1 + 2 + 4) kB per read
    assert mp["fetch_bytes_per_read"] == 7.0 * 1024 + 225
    assert mp["write_bytes_per_read"] == 7.0 / 8 * 1024
    assert mp["hbm_bytes_per_read"] == 7.0 * 1024 + 225 + 7.0 / 8 * 1024
    # the per-launch figure: the median over the full-size dispatches (no streamed bytes given)
    assert k["k_map1"]["fetch_bytes_per_read"] == 2.0 * 1024
    assert "k_bin_sum" in k


def test_traffic_one_k_map_has_no_pass_entry(tmp_path):
    rows = [(1, ONE, 500, 1000.0), (2, ONE, 500, 1100.0), (3, ONE, 500, 900.0)]
    _write(str(tmp_path / "F"), "FETCH_SIZE", rows)
    _write(str(tmp_path / "W"), "WRITE_SIZE", rows)
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), "cfg3", str(tmp_path / "F"),
                    str(tmp_path / "W"), str(out), "k_map1=150"], check=True, capture_output=True)
    t = json.load(open(out))
    k = t["kernels"]
    assert list(k) == ["k_map1"]
    assert k["k_map1"]["hbm_bytes_per_read"] == 2 * 2.0 * 1024 + 75
    assert "r3_fetch_calibration" in t["calibration"]
