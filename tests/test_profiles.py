"""The committed PMC evidence is reproducible (CPU only): every
profiles/traffic_<config>.json that lists its counter CSVs is recomputed from
those CSVs with tools/pmc_frac.py (the dominant kernel's VALU issue fraction
and HBM bytes, and the step totals over the scoring kernels), and every
bench line of the latest round that quotes a traffic or VALU figure quotes
that file's."""
import glob
import json
import math
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import pmc_frac  # noqa: E402


def _traffic_files():
    out = []
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_*.json"))):
        with open(f) as fh:
            tj = json.load(fh)
        csvs = (tj.get("sources") or {}).get("pmc_csvs") or []
        if csvs and all(c.endswith(".gz") for c in csvs) and \
                all(os.path.exists(os.path.join(REPO, c)) for c in csvs):
            out.append(f)
    return out


def _close(a, b):
    if a is None or b is None:
        return a is None and b is None
    return math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-6)


@pytest.mark.parametrize("path", _traffic_files(), ids=os.path.basename)
def test_traffic_json_recomputes_from_its_csvs(path):
    with open(path) as fh:
        tj = json.load(fh)
    csvs = [os.path.join(REPO, c) for c in tj["sources"]["pmc_csvs"]]
    dom = pmc_frac.summarize(tj["dominant"]["kernel_substring"], csvs)
    assert dom["dispatches"] > 0
    assert _close(dom.get("valu_issue_frac"), tj["valu"]["valu_issue_frac"])
    assert _close(dom.get("hbm_bytes_per_dispatch"), tj["hbm_bytes_per_launch"])
    # the step totals over the scoring kernels (tools/collect_profile.py)
    agg = tj["scoring"]
    runs = agg.get("step_runs_in_pmc_pass", 1)
    tot = {}
    for sub in agg["kernels"]:
        s = pmc_frac.summarize(sub, csvs)
        if not s.get("dispatches"):
            continue
        for c, v in s["per_dispatch"].items():
            n = s["counter_dispatches"][c]
            t = tot.setdefault(c, [0.0, 0.0])
            t[0] += v * n / runs
            t[1] += s["mean_duration_ns_by_pass"][c] * n / runs
    if "valu_issue_frac" in agg:
        v, dur = tot["SQ_INSTS_VALU"]
        assert _close(2.0 * v / (pmc_frac.SIMDS * dur * 1e-9 * pmc_frac.CLK),
                      agg["valu_issue_frac"])
    if "hbm_bytes_per_step" in agg:
        assert _close((2.0 * tot.get("FETCH_SIZE", [0.0])[0] +
                       tot.get("WRITE_SIZE", [0.0])[0]) * 1024.0, agg["hbm_bytes_per_step"])


def _latest_round_lines():
    rounds = sorted({os.path.basename(f)[:3] for f in
                     glob.glob(os.path.join(REPO, "profiles", "r??_bench_*.json"))})
    assert rounds, "no bench lines under profiles/"
    r = rounds[-1]
    return r, sorted(glob.glob(os.path.join(REPO, "profiles", f"{r}_bench_*.json")))


def test_bench_lines_quote_the_traffic_files():
    rnd, lines = _latest_round_lines()
    checked = 0
    for f in lines:
        with open(f) as fh:
            d = json.load(fh)
        for k in ("metric", "value", "unit", "roofline", "cpu_baseline", "parity"):
            assert k in d, (f, k)
        cfg = os.path.basename(f)[len(f"{rnd}_bench_"):-len(".json")]
        tf = os.path.join(REPO, "profiles", f"traffic_{cfg}.json")
        r = d["roofline"]
        if not os.path.exists(tf) or r.get("valu", {}).get("valu_issue_frac") is None:
            continue
        with open(tf) as fh:
            tj = json.load(fh)
        assert _close(r["valu"]["valu_issue_frac"], tj["valu"]["valu_issue_frac"]), f
        if r.get("traffic") is not None:
            want = (tj.get("scoring") or {}).get("hbm_bytes_per_step", tj["hbm_bytes_per_launch"])
            assert _close(r["traffic"], want), f
        checked += 1
    assert checked >= 8
