"""Per-kernel PMC summary over the dispatches' own durations (rocprofv3
--pmc counter_collection.csv files; every row carries its dispatch's
Start/End timestamps).

  python tools/pmc_frac.py SUBSTR file.csv [file.csv ...] [--json out.json]

For the dispatches whose kernel name contains SUBSTR (every dispatch of the
profiled run; pass several CSVs of separate --pmc passes of the same
command), prints and optionally writes:
  dispatches, mean dispatch duration (End - Start, ns);
  counters summed and per dispatch;
  valu_issue_frac = 2 * SQ_INSTS_VALU / (1024 SIMDs * duration * 2.4 GHz):
      VALU wave-instructions issued against the chip's issue capacity of one
      wave-instruction per 2 cycles per SIMD (MI355X_MICROARCH.md, v_fma_f32
      2 cyc SIMD-32) at the nominal clock, over the dispatch's own duration;
  hbm_bytes_per_dispatch = 2 * FETCH_SIZE + WRITE_SIZE (kB units * 1024):
      FETCH_SIZE doubled for gfx950 (MI355X_MICROARCH.md, HBM section).
"""
import csv
import gzip
import json
import sys

CLK = 2.4e9
SIMDS = 1024


def summarize(sub, files):
    disp = {}  # (file, dispatch id) -> {counter: value, "_dur": ns}
    for f in files:
        for row in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            if sub not in row["Kernel_Name"]:
                continue
            d = disp.setdefault((f, row["Dispatch_Id"]), {"_dur": 0.0, "_name": row["Kernel_Name"]})
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            d["_dur"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    out = {"kernel_substring": sub, "files": files, "dispatches": 0}
    if not disp:
        return out
    names = sorted({d["_name"] for d in disp.values()})
    counters = sorted({k for d in disp.values() for k in d if not k.startswith("_")})
    per = {}
    for c in counters:  # mean over the dispatches of the pass that collected c
        vals = [d[c] for d in disp.values() if c in d]
        per[c] = sum(vals) / len(vals)
        out.setdefault("counter_dispatches", {})[c] = len(vals)
    durs = {c: [d["_dur"] for d in disp.values() if c in d] for c in counters}
    out.update({"kernel_names": names, "dispatches": len(disp),
                "mean_duration_ns_by_pass": {c: sum(v) / len(v) for c, v in durs.items()},
                "per_dispatch": per, "clock_hz": CLK, "simds": SIMDS})
    if "SQ_INSTS_VALU" in per:
        dur = sum(durs["SQ_INSTS_VALU"]) / len(durs["SQ_INSTS_VALU"]) * 1e-9
        out["valu_issue_frac"] = 2.0 * per["SQ_INSTS_VALU"] / (SIMDS * dur * CLK)
        out["valu_issue_formula"] = ("2 * SQ_INSTS_VALU / (1024 * (End_Timestamp - "
                                     "Start_Timestamp) * 2.4e9), mean over the dispatches")
        if "GRBM_GUI_ACTIVE" in per:
            out["effective_clock_hz"] = per["GRBM_GUI_ACTIVE"] / 8.0 / dur
    if "SQ_WAVE_CYCLES" in per:
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in per:
                out[k.lower() + "_per_wave_cycle"] = per[k] / per["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in per or "WRITE_SIZE" in per:
        out["hbm_bytes_per_dispatch"] = (2.0 * per.get("FETCH_SIZE", 0.0) +
                                         per.get("WRITE_SIZE", 0.0)) * 1024.0
        out["hbm_formula"] = "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (gfx950: FETCH_SIZE x2)"
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    jpath = None
    if "--json" in args:
        i = args.index("--json")
        jpath = args[i + 1]
        args = args[:i] + args[i + 2:]
    r = summarize(args[0], args[1:])
    print(json.dumps(r, indent=1))
    if jpath:
        with open(jpath, "w") as f:
            json.dump(r, f, indent=1)
