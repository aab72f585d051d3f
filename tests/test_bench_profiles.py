"""bench.py's roofline only uses a rocprofv3 profile taken on this very build and workload
(profiles/pmc_<code>[_<batch>].json stamped with qec_build_id(), tools/gpu/pmc_summary.py)."""
import json
import os
import sys

import qec_ldpc_amd as q

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_committed_profiles_are_well_formed():
    """Every committed profile names its workload and build; whether its build is this tree's is
    bench.py's call at run time (a stale profile gives frac null with the reason), not a unit test's:
    any source edit changes the build id until the next GPU profiling pass."""
    import glob
    names = sorted(os.path.basename(f) for f in glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    assert "pmc_p61.json" in names
    for name in names:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            pm = json.load(f)
        assert len(pm["build_id"]) == 16 and pm["batch"] > 0 and pm["stop"] in ("fixed", "ref", "syndrome"), name
        if name.startswith("pmc_mc_"):  # config-5 kernel profiles (tools/gpu/mc_pmc_summary.py)
            assert pm["dominant"] in pm["kernels"] and pm["samples"] > 0, name
            assert all(k["avg_ns"] > 0 and k.get("valu_issue_frac") is not None for k in pm["kernels"].values()), name
        else:  # decode-launch profiles (tools/gpu/pmc_summary.py)
            assert pm["valu_insts_per_syndrome"] > 0 and pm["valu_weighted_slots_per_syndrome"] > 0, name


def test_load_pmc_checks_workload_batch_and_build(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"iters": 50, "stop": "fixed", "p": 0.01, "batch": 4096, "build_id": q.build_id(),
            "valu_insts_per_syndrome": 100.0, "input": "bits", "hard_paths": 1}
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    (prof / "pmc_p61.json").write_text(json.dumps(base))
    pm, path = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
    assert pm is not None and path.endswith("pmc_p61.json")
    for change, why in (({"build_id": "0000000000000000"}, "another build"), ({"batch": 8192}, "batch 8192"),
                        ({"p": 0.02}, "other workload"), ({"iters": 20}, "other workload"),
                        ({"input": "bytes"}, "other workload"), ({"hard_paths": 0}, "other workload")):
        (prof / "pmc_p61.json").write_text(json.dumps(dict(base, **change)))
        pm, note = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
        assert pm is None and why in note, (change, note)
    # a batch-specific profile wins over the generic one
    (prof / "pmc_p61.json").write_text(json.dumps(dict(base, batch=65536)))
    (prof / "pmc_p61_4096.json").write_text(json.dumps(base))
    pm, path = bench.load_pmc("p61", 50, "fixed", 0.01, 4096)
    assert pm is not None and path.endswith("pmc_p61_4096.json")
    # the full-arithmetic launch (hard paths off) has profiles of its own
    pm, note = bench.load_pmc("p61", 50, "fixed", 0.01, 4096, hard_paths=0)
    assert pm is None and "_hp0" in note
    (prof / "pmc_p61_4096_hp0.json").write_text(json.dumps(dict(base, hard_paths=0)))
    pm, path = bench.load_pmc("p61", 50, "fixed", 0.01, 4096, hard_paths=0)
    assert pm is not None and path.endswith("pmc_p61_4096_hp0.json")


def test_valu_roofline_counter_exact_and_weighted():
    """frac is the counter-exact SQ_INSTS_VALU issue; the cost-weighted figures (each transcendental at 4
    and at 2 issue slots) sit beside it."""
    pm = {"valu_insts_per_syndrome": 1000.0, "valu_weighted_slots_per_syndrome": 1300.0, "batch": 1000,
          "valu_trans_per_launch": 100000, "hbm_bytes_per_syndrome": 500.0, "lds_bank_conflict_share": 0.23}
    r = bench.valu_roofline(pm, os.path.join(ROOT, "profiles", "x.json"), 1000, 1.0)
    peak = 1024 * 2.4e9 / 2 / 1e12
    assert abs(r["frac"] - 1000.0 * 1000 / 1e-3 / 1e12 / peak) < 1e-3
    assert abs(r["frac_weighted_probe4x"] - 1300.0 * 1000 / 1e-3 / 1e12 / peak) < 1e-3
    assert abs(r["frac_weighted_guide2x"] - 1100.0 * 1000 / 1e-3 / 1e12 / peak) < 1e-3
    assert r["traffic"] == 500000 and r["lds_bank_conflict_share"] == 0.23
    r = bench.valu_roofline(None, "no profile", 1000, 1.0)
    assert r["frac"] is None and "no PMC profile" in r["note"]


def test_host_threads_reports_its_source(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n, src = bench.host_threads()
    assert n == 3 and src["source"] == "OMP_NUM_THREADS" and src["os_cpu_count"] == os.cpu_count()
    monkeypatch.delenv("OMP_NUM_THREADS")
    n, src = bench.host_threads()
    assert 1 <= n <= os.cpu_count() and src["source"] in ("CPU affinity set", "cgroup cpu.max quota")
