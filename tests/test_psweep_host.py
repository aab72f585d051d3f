"""Host logic of tools/psweep.py (config 5's sweep; no GPU): a sweep line's roofline is taken only from
a profile of the same workload on the same library build, its frac is the issue fraction of the bound
it names, and the rates follow from the summed counters."""
import json
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import psweep  # noqa: E402

CODE = "J_4_K_5_L_10_P_61_s_9_t_49"


def _profile(tmp_path, monkeypatch, build_id, valu, lds, **over):
    import qec_ldpc_amd as q
    monkeypatch.setattr(psweep, "ROOT", str(tmp_path))
    monkeypatch.setattr(q, "build_id", lambda: "b1")
    os.makedirs(tmp_path / "profiles", exist_ok=True)
    pm = {"p": 0.005, "samples": 1 << 20, "batch": 1 << 20, "stop": "syndrome", "iters": 50, "build_id": build_id,
          "dominant": "bp_decode_kernel[mode 2]",
          "kernels": {"bp_decode_kernel[mode 2]": {"avg_ns": 530000, "valu_issue_frac": valu, "lds_issue_frac": lds,
                                                   "wait_over_issue": 0.54},
                      "mc_fused_kernel": {"avg_ns": 120000, "valu_issue_frac": 0.49, "lds_issue_frac": 0.28}}}
    pm.update(over)
    with open(tmp_path / "profiles" / "pmc_mc_p61_p0.005.json", "w") as f:
        json.dump(pm, f)


def test_roofline_frac_is_the_bound_fraction(tmp_path, monkeypatch):
    _profile(tmp_path, monkeypatch, "b1", 0.39, 0.42)
    r = psweep.mc_roofline(0.005, 1 << 20, "syndrome", 50, 1 << 20, CODE)
    assert r["bound"] == "lds" and r["frac"] == pytest.approx(0.42)
    assert r["valu_issue_frac"] == pytest.approx(0.39) and r["lds_issue_frac"] == pytest.approx(0.42)
    assert r["kernels_us"] == {"bp_decode_kernel[mode 2]": 530.0, "mc_fused_kernel": 120.0}
    _profile(tmp_path, monkeypatch, "b1", 0.62, 0.51)
    r = psweep.mc_roofline(0.005, 1 << 20, "syndrome", 50, 1 << 20, CODE)
    assert r["bound"] == "valu" and r["frac"] == pytest.approx(0.62)


@pytest.mark.parametrize("case", ["other_build", "other_workload", "other_stop", "missing"])
def test_roofline_refuses_foreign_profiles(tmp_path, monkeypatch, case):
    _profile(tmp_path, monkeypatch, "b0" if case == "other_build" else "b1", 0.39, 0.42,
             **({"samples": 4096} if case == "other_workload" else {}))
    stop = "fixed" if case == "other_stop" else "syndrome"  # reads pmc_mc_p61_fixed_p0.005.json: absent
    p = 0.01 if case == "missing" else 0.005
    r = psweep.mc_roofline(p, 1 << 20, stop, 50, 1 << 20, CODE)
    assert r["frac"] is None and r["note"]


def test_summarize_rates():
    c = dict.fromkeys(psweep.FIELDS, 0)
    c.update(tested=1000, corrected=990, logical=4, synX=3, synZ=3, iterationsX=1500, iterationsZ=1200)
    line = psweep.summarize(0.01, c, 0.5, 2)
    assert line["syndromes_per_s"] == 2000.0 and line["n_gpus"] == 2
    assert line["decoder_failure_rate"] == pytest.approx(0.01) and line["logical_error_rate"] == pytest.approx(0.004)
    assert line["mean_iterations_x"] == pytest.approx(1.5) and line["mean_iterations_z"] == pytest.approx(1.2)
