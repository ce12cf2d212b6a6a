"""Per-kernel PMC summary of rocprofv3 counter passes (tools/gpu.sh pmc:<probe>:<pass> steps):
counter totals of the named kernel's last dispatch in each pass, per-tile instruction counts,
and busy fractions normalised by THAT dispatch's own duration (its Start/End_Timestamp in the
counter CSV) — not by GRBM_GUI_ACTIVE alone, which the profiler accumulates over more than the
kernel.  The effective clock is GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md, DVFS
give-back); when a pass lacks GRBM_GUI_ACTIVE, --clock-ghz (default 2.1) is used.

    python tools/pmc_summary.py <tiles> <pass dir> [<pass dir> ...] [--kernel SUBSTR]
                                [--simds 1024] [--clock-ghz 2.1] [--dispatch last|longest|N]

--dispatch picks which dispatch of the kernel each pass reports: the last (default), the longest,
or the N-th (0-based, in dispatch order).  Memory passes add the L2 (TCC) hit ratio and, with
FETCH_SIZE (KiB), the bytes fetched from HBM and their rate over the dispatch.

Units: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES
counts cycles summed over SIMDs."""
import csv
import json
import os
import sys


def main(argv):
    args = list(argv)
    opts = {"--kernel": "lloyd_t1", "--simds": "1024", "--clock-ghz": "2.1", "--dispatch": "last"}
    for key in list(opts):
        if key in args:
            i = args.index(key)
            opts[key] = args[i + 1]
            del args[i:i + 2]
    kern, simds, clk_default = opts["--kernel"], float(opts["--simds"]), float(opts["--clock-ghz"])
    tiles = float(args[0])
    vals, durations, clocks = {}, [], []
    for d in args[1:]:
        path = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
        if not rows:
            continue
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        pick = opts["--dispatch"]
        if pick == "last":
            last = ids[-1]
        elif pick == "longest":
            span = {int(r["Dispatch_Id"]): float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                    for r in rows}
            last = max(ids, key=lambda i: span[i])
        else:
            last = ids[min(int(pick), len(ids) - 1)]
        mine = [r for r in rows if int(r["Dispatch_Id"]) == last]
        dur_ns = float(mine[0]["End_Timestamp"]) - float(mine[0]["Start_Timestamp"])
        durations.append(dur_ns)
        pv = {}
        for r in mine:
            pv[r["Counter_Name"]] = pv.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            vals["_vgpr"] = int(r["VGPR_Count"])
        if "GRBM_GUI_ACTIVE" in pv and dur_ns > 0:
            clocks.append(pv["GRBM_GUI_ACTIVE"] / 8.0 / dur_ns)
        for c, v in pv.items():
            if c != "GRBM_GUI_ACTIVE":
                vals[c] = v
    out = {"kernel": kern, "counters": vals}
    if not durations:
        print(json.dumps(out, indent=1))
        return 0
    dur = sum(durations) / len(durations)
    ghz = sum(clocks) / len(clocks) if clocks else clk_default
    cyc = dur * ghz  # kernel cycles (per SIMD)
    out.update({"dispatch_ms_mean": round(dur * 1e-6, 4), "clock_ghz_effective": round(ghz, 3),
                "clock_source": "GRBM_GUI_ACTIVE/8/duration" if clocks else "assumed",
                "kernel_cycles": round(cyc)})
    wc = vals.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in vals:
                out[c + "_frac_of_wave_cycles"] = round(vals[c] / wc, 4)
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM",
              "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_MOPS_F16"):
        if c in vals:
            out[c + "_per_tile"] = round(vals[c] / tiles, 2)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals:
        out["mfma_busy_frac_per_simd"] = round(vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (simds * cyc), 4)
        if "SQ_INSTS_MFMA" in vals and vals["SQ_INSTS_MFMA"] > 0:
            out["mfma_busy_cycles_per_mfma"] = round(
                vals["SQ_VALU_MFMA_BUSY_CYCLES"] / vals["SQ_INSTS_MFMA"], 2)
    for c, name in (("SQ_ACTIVE_INST_VALU", "valu"), ("SQ_ACTIVE_INST_LDS", "lds"),
                    ("SQ_ACTIVE_INST_VMEM", "vmem"), ("SQ_ACTIVE_INST_SCA", "salu")):
        if c in vals:  # quad-cycles summed over waves, per SIMD-cycle of the dispatch
            out[name + "_active_frac_per_simd"] = round(4.0 * vals[c] / (simds * cyc), 4)
    if "SQ_INST_LEVEL_VMEM" in vals and vals.get("SQ_INSTS_VMEM"):
        # (level accumulates in-flight VMEM instructions per quad-cycle: mean latency in cycles)
        out["vmem_mean_latency_cycles"] = round(4.0 * vals["SQ_INST_LEVEL_VMEM"] /
                                                vals["SQ_INSTS_VMEM"], 1)
    if "TCC_HIT_sum" in vals and "TCC_MISS_sum" in vals:
        tot = vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"]
        out["tcc_hit_ratio"] = round(vals["TCC_HIT_sum"] / tot, 4) if tot else None
    if "FETCH_SIZE" in vals:
        out["hbm_fetch_gb"] = round(vals["FETCH_SIZE"] * 1024 / 1e9, 3)
        out["hbm_fetch_tb_per_s"] = round(vals["FETCH_SIZE"] * 1024 / (dur * 1e-9) / 1e12, 3)
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main(sys.argv[1:]))
