"""Sum rocprofv3 counter_collection.csv values per counter for kernels whose
name contains SUBSTR.  Usage: python tools/pmc_sum.py SUBSTR file.csv [...]"""
import csv, sys
sub = sys.argv[1]
vals, disp = {}, set()
for f in sys.argv[2:]:
    for row in csv.DictReader(open(f)):
        if sub in row["Kernel_Name"]:
            vals[row["Counter_Name"]] = vals.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            disp.add((f, row.get("Dispatch_Id")))
print(f"{len(disp)} dispatches")
for k, v in sorted(vals.items()):
    print(f"  {k:24s} {v:.4e}")
if "SQ_INSTS_VALU" in vals and "GRBM_GUI_ACTIVE" in vals:
    cyc = vals["GRBM_GUI_ACTIVE"] / 8.0
    print(f"  kernel cycles {cyc:.4e}; valu issue frac {2.0 * vals['SQ_INSTS_VALU'] / (1024.0 * cyc):.3f}")
if "SQ_WAIT_INST_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
    print(f"  wait_inst_any / wave_cycles {vals['SQ_WAIT_INST_ANY'] / vals['SQ_WAVE_CYCLES']:.3f}; "
          f"active_valu / wave_cycles {vals['SQ_ACTIVE_INST_VALU'] / vals['SQ_WAVE_CYCLES']:.3f}; "
          f"wait_any / wave_cycles {vals['SQ_WAIT_ANY'] / vals['SQ_WAVE_CYCLES']:.3f}")
