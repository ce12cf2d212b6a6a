"""Per-kernel PMC summary of tools/pmc_lean.sh passes: counter totals per dispatch of the named
kernel (last dispatch of each pass), derived per-tile instruction counts and wait fractions.

    python tools/pmc_summary.py <tiles> <pass dir> [<pass dir> ...] [--kernel SUBSTR]"""
import csv
import json
import os
import sys

args = [a for a in sys.argv[1:]]
kern = "lloyd_t1"
if "--kernel" in args:
    i = args.index("--kernel")
    kern = args[i + 1]
    del args[i:i + 2]
tiles = float(args[0])
vals = {}
for d in args[1:]:
    path = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    if not rows:
        continue
    last = max(int(r["Dispatch_Id"]) for r in rows)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            vals["_vgpr"] = int(r["VGPR_Count"])
out = {"kernel": kern, "counters": vals}
wc = vals.get("SQ_WAVE_CYCLES")
if wc:
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in vals:
            out[c + "_frac_of_wave_cycles"] = round(vals[c] / wc, 4)
for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM",
          "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_MFMA"):
    if c in vals:
        out[c + "_per_tile"] = round(vals[c] / tiles, 2)
if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
    # busy cycles summed over SIMDs (1024) against the GPU-active clock
    busy = vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (vals["GRBM_GUI_ACTIVE"] * 1024)
    out["mfma_busy_frac"] = round(busy, 4)
print(json.dumps(out, indent=1))
