"""bench.py attaches a PMC `traffic` figure only from a profile of the SAME libyms.so build it runs
(a round-4 profile was reported for round-5 kernels): profiles carry the sha256 of the
library they profiled (tools/rocprof_summary.py), and the lookup skips every other build."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _profile(d, name, sha, workload, nbytes):
    os.makedirs(os.path.join(d, "profiles"), exist_ok=True)
    j = {"train": {"bench_config": {"workload": workload}, "conv_hbm_bytes_per_call": nbytes,
                   "conv_mfma_busy_frac": 0.2}}
    if sha is not None:
        j["libyms_sha256"] = sha
    with open(os.path.join(d, "profiles", name), "w") as f:
        json.dump(j, f)


def test_traffic_only_from_the_loaded_build(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "_LIB_SHA", "a" * 64)
    wl = "configs[2]: test workload"
    _profile(tmp_path, "r09_pmc_traffic.json", "b" * 64, wl, 111.0)      # newest: another build
    _profile(tmp_path, "r08_pmc_traffic.json", None, wl, 222.0)          # no sha recorded
    assert bench.pmc_traffic("train", wl) == (None, None, None)
    roof = {}
    bench.add_traffic(roof, "train", wl)
    assert "traffic" not in roof and roof["traffic_source"].startswith("none")
    assert roof["traffic_libyms_sha256"] == "a" * 64
    _profile(tmp_path, "r07_pmc_traffic.json", "a" * 64, wl, 333.0)      # older file, same build
    t, src, busy = bench.pmc_traffic("train", wl)
    assert (t, src, busy) == (333.0, os.path.join("profiles", "r07_pmc_traffic.json"), 0.2)
    assert bench.pmc_traffic("train", "another workload") == (None, None, None)
    roof = {}
    bench.add_traffic(roof, "train", wl)
    assert roof["traffic"] == 333 and roof["traffic_source"].endswith("r07_pmc_traffic.json")
