"""Turn a config's rocprofv3 runs (tools/gpu_task.sh trace TAG + pmc TAG mem /
valu / wait, same bench arguments) into the committed evidence under
profiles/ and the profiles/traffic_CONFIG.json that bench.py reads.

Usage: python tools/collect_profile.py [--runs R] CONFIG TAG DOMINANT [SCORING ...]

DOMINANT selects the kernel the bench line's roofline prices (every dispatch
whose name contains it); SCORING (default: DOMINANT) the substrings of every
candidate-scoring launch of one step (e.g. k_small_prep1 k_small_one
k_small_finalize for the small pipeline).  The PMC passes ran `bench.py
--steps 1 --warmup 0`; R (default 1) is how many times that run executes
the step: 2 for the grouped greedy configs (bench.py's timed() runs the step
once without and once with the scoring timers), 1 for the importance and PLN
lines.  Step totals are the PMC run's totals divided by R.

Fractions are computed over each dispatch's own duration (End - Start of its
counter_collection.csv row), tools/pmc_frac.py:
  valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 SIMDs * duration * 2.4e9);
  hbm bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE x2).
Everything in traffic_CONFIG.json can be recomputed from the CSVs it lists.
"""
import glob
import gzip
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import pmc_frac  # noqa: E402

PASSES = ("fetch", "write", "valu", "wait")


def one(pattern):
    f = sorted(glob.glob(pattern, recursive=True))
    return f[0] if f else None


def main():
    argv = sys.argv[1:]
    runs = 1
    if argv[0] == "--runs":
        runs, argv = int(argv[1]), argv[2:]
    config, tag, dom = argv[0], argv[1], argv[2]
    scoring = argv[3:] or [dom]
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    files = {}
    for what, pat in (("kernel_stats", f"prof_{tag}_trace/**/*kernel_stats.csv"),
                      ("kernel_trace", f"prof_{tag}_trace/**/*kernel_trace.csv")):
        f = one(os.path.join(src, pat))
        if f:
            files[what] = os.path.join("profiles", f"{tag}_{what}.csv")
            if what == "kernel_trace":  # one row per dispatch: kept gzipped
                files[what] += ".gz"
                with open(f, "rb") as fi, gzip.open(os.path.join(ROOT, files[what]), "wb") as fo:
                    shutil.copyfileobj(fi, fo)
            else:
                shutil.copy(f, os.path.join(ROOT, files[what]))
    csvs = []
    for p in PASSES:
        f = one(os.path.join(src, f"prof_{tag}_{p}/**/*counter_collection.csv"))
        if not f:
            continue
        rel = os.path.join("profiles", f"{tag}_pmc_{p}.csv.gz")  # gzipped (pmc_frac reads it)
        with open(f, "rb") as fi, gzip.open(os.path.join(ROOT, rel), "wb") as fo:
            shutil.copyfileobj(fi, fo)
        csvs.append(rel)
    absf = [os.path.join(ROOT, c) for c in csvs]
    d = pmc_frac.summarize(dom, absf)
    # every scoring dispatch of the step: totals per pass, then the fractions
    tot = {}
    for sub in scoring:
        s = pmc_frac.summarize(sub, absf)
        if not s.get("dispatches"):
            continue
        for c, v in s["per_dispatch"].items():
            n = s["counter_dispatches"][c]
            tot.setdefault(c, [0.0, 0.0])
            tot[c][0] += v * n / runs
            tot[c][1] += s["mean_duration_ns_by_pass"][c] * n / runs
    agg = {"kernels": scoring, "step_runs_in_pmc_pass": runs}
    if "SQ_INSTS_VALU" in tot:
        v, dur = tot["SQ_INSTS_VALU"]
        agg["valu_instructions_per_step"] = v
        agg["duration_ns_per_step"] = dur
        agg["valu_issue_frac"] = 2.0 * v / (pmc_frac.SIMDS * dur * 1e-9 * pmc_frac.CLK)
    if "FETCH_SIZE" in tot or "WRITE_SIZE" in tot:
        agg["hbm_bytes_per_step"] = (2.0 * tot.get("FETCH_SIZE", [0.0])[0] +
                                     tot.get("WRITE_SIZE", [0.0])[0]) * 1024.0
    line = None
    lf = os.path.join(src, f"prof_{tag}_trace.log")
    if os.path.exists(lf):
        for ln in open(lf):
            if ln.startswith('{"metric"'):
                line = json.loads(ln)
    cfg = (line or {}).get("config", {})
    out = {"config": config, "tag": tag,
           "blocks": cfg.get("blocks_per_gpu", cfg.get("groups_per_step")),
           "dominant": d, "scoring": agg,
           "hbm_bytes_per_launch": d.get("hbm_bytes_per_dispatch"),
           "valu": {"valu_issue_frac": d.get("valu_issue_frac"),
                    "formula": d.get("valu_issue_formula")},
           "sources": {"pmc_csvs": csvs, **files},
           "method": "rocprofv3 --pmc passes (FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU "
                     "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE | SQ_WAVE_CYCLES "
                     "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES) of `python3 "
                     "bench.py --steps 1 --warmup 0 --no-cpu --no-e2e`, one pass each "
                     "(tools/gpu_task.sh pmc); tools/collect_profile.py + tools/pmc_frac.py"}
    with open(os.path.join(dst, f"traffic_{config}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("config", "blocks", "hbm_bytes_per_launch", "valu",
                                          "scoring")}, indent=1))


if __name__ == "__main__":
    main()
