"""The HBM-traffic summary bench.py builds from its own rocprofv3 --pmc passes
(tools/pmc_summary.py): the headline is the FIRST headline-kernel dispatch of the pass, later
XCD-kernel dispatches are the 8-utterance line, the many-row kernel's RAW instantiations are not
config 3's, and bytes = 1024 · (2 · FETCH_SIZE + WRITE_SIZE) (gfx950 read correction)."""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import pmc_summary  # noqa: E402

FIELDS = ["Dispatch_Id", "Kernel_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def _write(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for i, (name, kib, dur) in enumerate(rows):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": name, "Counter_Value": kib, "Start_Timestamp": 1000,
                        "End_Timestamp": 1000 + dur})


def test_summary_picks_the_headline_dispatch_and_sums_the_configs(tmp_path):
    xcd = "void wrnn::fatchord_xcd_kernel<false>(wrnn::XcdArgs)"
    for counter, scale in (("FETCH_SIZE", 1.0), ("WRITE_SIZE", 0.5)):
        _write(str(tmp_path / f"pmc_{counter}" / "pmc_counter_collection.csv"), [
            ("Cijk_gemm", 5.0 * scale, 10),
            (xcd, 100.0 * scale, 400),                                       # the headline (first)
            ("void wrnn::fatchord_xcdm_kernel<1, false, false>(wrnn::XcdmArgs)", 3.0 * scale, 60),   # fold-batched
            (xcd, 900.0 * scale, 500),                                       # 8 utterances: longer, later
            ("void wrnn::fatchord_xcdm_kernel<1, false, true>(wrnn::XcdmArgs)", 7.0 * scale, 100),   # RAW
            ("void wrnn::fatchord_xcdm_kernel<4, false, false>(wrnn::XcdmArgs)", 40.0 * scale, 50),
            ("void wrnn::fatchord_xcdm_kernel<4, false, false>(wrnn::XcdmArgs)", 60.0 * scale, 50),
            ("void wrnn::fatchord_xcdm_kernel<1, false, false>(wrnn::XcdmArgs)", 20.0 * scale, 70),  # 32 streams
            ("void wrnn::fatchord_xcds_kernel<false>(wrnn::XcdsArgs)", 11.0 * scale, 50),
            ("void wrnn::deepmind_xcd_kernel<false>(wrnn::DxArgs)", 13.0 * scale, 50),
        ])
    out = pmc_summary.summarise(str(tmp_path))
    assert out["counters"]["FETCH_SIZE"]["value_kib"] == 100.0
    assert out["bytes"] == 1024.0 * (2 * 100.0 + 50.0)
    cfg = out["other_configs"]
    assert cfg["config2_8_streams"]["bytes_per_step"] == 1024.0 * (2 * 900.0 + 450.0) / 110275
    assert cfg["config3_mol_fold_60s"]["bytes_per_step"] == 1024.0 * (2 * 100.0 + 50.0) / 12100
    assert cfg["config2_32_streams"]["bytes_per_step"] == 1024.0 * (2 * 20.0 + 10.0) / 110275
    assert cfg["fold_batched"]["bytes_per_step"] == 1024.0 * (2 * 3.0 + 1.5) / 12100
    assert cfg["config3_mol_fold_60s"]["kernel"] == "fatchord_xcdm_kernel"
    assert cfg["config4_sparse896_8utt"]["fetch_kib"] == 11.0
    assert cfg["config5_deepmind_32utt"]["write_kib"] == 6.5


def test_bench_traffic_never_falls_back_to_an_unnamed_profile(tmp_path, monkeypatch):
    """when the live passes fail, the headline's traffic is null with the reason
    (no older kernel's profile presented as this one's); a profile named by WRNN_PMC_PROFILE is used
    and labelled; the fold-batched line carries its own traffic_per_step."""
    sys.path.insert(0, REPO)
    import json
    import bench
    tr, src = bench.resolve_traffic(None, None)
    assert tr is None and src.startswith("unavailable")
    tr, src = bench.resolve_traffic(None, str(tmp_path / "missing.json"))
    assert tr is None and src.startswith("unavailable")
    prof = tmp_path / "named.json"
    prof.write_text(json.dumps({"bytes": 123.0, "other_configs": {"fold_batched": {"bytes_per_step": 9.0}}}))
    tr, src = bench.resolve_traffic(None, str(prof))
    assert tr["bytes"] == 123.0 and "WRNN_PMC_PROFILE" in src
    live = {"bytes": 1.0, "other_configs": {}}
    assert bench.resolve_traffic(live, str(prof)) == (live, "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this run")
    rec = {"fold_batched": {"roofline": {}}, "other_configs": {"config3_mol_fold_60s": {"roofline": {}}, "x": {}}}
    bench.attach_traffic(rec, tr, src)
    assert rec["fold_batched"]["roofline"]["traffic_per_step"] == 9.0
    assert rec["other_configs"]["config3_mol_fold_60s"]["roofline"]["traffic_per_step"] is None
    assert rec["other_configs"]["config3_mol_fold_60s"]["roofline"]["traffic_from"] == src
    assert bench.PMC_PROFILE == os.environ.get("WRNN_PMC_PROFILE")
