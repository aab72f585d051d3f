"""bench.py's roofline only uses a rocprofv3 profile taken on this very build and workload
(profiles/pmc_<code>[_<batch>].json stamped with qec_build_id(), tools/gpu/pmc_summary.py), and the
committed profiles of the shipped workloads carry the current build's id (no GPU needed)."""
import json
import os
import sys

import qec_ldpc_amd as q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_committed_profiles_match_this_build():
    for name, batch in (("pmc_p61.json", 1 << 20), ("pmc_p7.json", 1 << 20), ("pmc_p7_65536.json", 65536)):
        with open(os.path.join(ROOT, "profiles", name)) as f:
            pm = json.load(f)
        assert pm["build_id"] == q.build_id(), name
        assert pm["batch"] == batch and pm["stop"] == "fixed"
        assert pm["valu_insts_per_syndrome"] > 0 and pm["valu_weighted_slots_per_syndrome"] > 0


def test_load_pmc_checks_workload_batch_and_build(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"iters": 50, "stop": "fixed", "p": 0.01, "batch": 4096, "build_id": q.build_id(),
            "valu_insts_per_syndrome": 100.0}
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    (prof / "pmc_p61.json").write_text(json.dumps(base))
    pm, path = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
    assert pm is not None and path.endswith("pmc_p61.json")
    for change, why in (({"build_id": "0000000000000000"}, "another build"), ({"batch": 8192}, "batch 8192"),
                        ({"p": 0.02}, "other workload"), ({"iters": 20}, "other workload")):
        (prof / "pmc_p61.json").write_text(json.dumps(dict(base, **change)))
        pm, note = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
        assert pm is None and why in note, (change, note)
    # a batch-specific profile wins over the generic one
    (prof / "pmc_p61.json").write_text(json.dumps(dict(base, batch=65536)))
    (prof / "pmc_p61_4096.json").write_text(json.dumps(base))
    pm, path = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
    assert pm is not None and path.endswith("pmc_p61_4096.json")


def test_valu_roofline_weighted_and_null():
    pm = {"valu_insts_per_syndrome": 1000.0, "valu_weighted_slots_per_syndrome": 1300.0, "batch": 1000,
          "valu_trans_per_launch": 100000, "hbm_bytes_per_syndrome": 500.0}
    r = bench.valu_roofline(pm, os.path.join(ROOT, "profiles", "x.json"), 1000, 1.0, 1)
    peak = 1024 * 2.4e9 / 2 / 1e12
    assert abs(r["frac"] - 1300.0 * 1000 / 1e-3 / 1e12 / peak) < 1e-3
    assert abs(r["frac_unweighted"] - 1000.0 * 1000 / 1e-3 / 1e12 / peak) < 1e-3
    assert r["traffic"] == 500000
    r = bench.valu_roofline(None, "no profile", 1000, 1.0, 1)
    assert r["frac"] is None and "no PMC profile" in r["note"]
