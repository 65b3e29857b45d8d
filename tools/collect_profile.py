"""Turn tools/profile.sh output into the committed evidence under profiles/.
Usage: python tools/collect_profile.py TAG CONFIG KERNEL_SUBSTR [BLOCKS ALG_BYTES]
KERNEL_SUBSTR selects the priced kernels (every dispatch whose name contains
it, counters summed: "k_small_" takes prep + screen + survivors).  BLOCKS (the
blocks or groups of one launch) and ALG_BYTES default to the bench line of the
trace run (config.blocks_per_gpu / groups_per_step, roofline's algorithmic
bytes)."""
import csv, glob, json, os, shutil, sys

tag, config, ksub = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(root, "gpurun_out", "prof_" + tag)
dst = os.path.join(root, "profiles")
if len(sys.argv) > 5:
    blocks, alg = int(sys.argv[4]), int(sys.argv[5])
else:
    line = [ln for ln in open(os.path.join(src, "trace.log")) if ln.startswith('{"metric"')][-1]
    bl = json.loads(line)
    blocks = bl["config"].get("blocks_per_gpu", bl["config"].get("groups_per_step"))
    alg = bl["roofline"]["algorithmic_bytes_per_launch"]


def one(pattern):
    f = sorted(glob.glob(os.path.join(src, pattern), recursive=True))
    assert f, pattern
    return f[0]


shutil.copy(one("trace/**/*kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
shutil.copy(one("trace/**/*kernel_trace.csv"), os.path.join(dst, f"{tag}_kernel_trace.csv"))
vals = {}
for pas in ("fetch", "write", "valu"):
    f = one(f"{pas}/**/*counter_collection.csv")
    shutil.copy(f, os.path.join(dst, f"{tag}_pmc_{pas}.csv"))
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if ksub in row["Kernel_Name"]:
                vals.setdefault(row["Counter_Name"], 0.0)
                vals[row["Counter_Name"]] += float(row["Counter_Value"])
fetch_kb, write_kb = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
hbm = int((2 * fetch_kb + write_kb) * 1024)
out = {"config": config, "blocks": blocks, "kernel": ksub, "FETCH_SIZE_kB": fetch_kb,
       "WRITE_SIZE_kB": write_kb, "hbm_bytes_per_launch": hbm,
       "algorithmic_bytes_per_launch": alg,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of "
                 "`python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e` (one eval launch "
                 "each); bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per MI355X_MICROARCH.md",
       "valu": {k: vals.get(k) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU",
                                         "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE")}}
v = out["valu"]
if v.get("SQ_INSTS_VALU") and v.get("GRBM_GUI_ACTIVE"):
    # a wave64 VALU instruction occupies its SIMD32 for 2 cycles (MI355X_MICROARCH.md);
    # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
    cycles = v["GRBM_GUI_ACTIVE"] / 8.0
    v["kernel_cycles"] = cycles
    v["valu_issue_frac"] = 2.0 * v["SQ_INSTS_VALU"] / (1024.0 * cycles)
with open(os.path.join(dst, f"traffic_{config}.json"), "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(out, indent=1))
