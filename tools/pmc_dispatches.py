"""Per-dispatch PMC table of the last fit in rocprofv3 counter passes (tools/gpu.sh pmc steps):
kernel, duration, effective clock, wait/issue fractions, MFMA busy, instruction mix per pass.

    python tools/pmc_dispatches.py <pass dir> [<pass dir> ...]"""
import csv, sys, re, collections
# per-dispatch table of the last fit: kernel short name, ms, counters (merged over passes)
rows = collections.OrderedDict()
for p in sys.argv[1:]:
    for r in csv.DictReader(open(p + "/run_counter_collection.csv")):
        m = re.search(r"(oap_\w+)(<[^>(]*>)?", r["Kernel_Name"]); name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:30]
        key = (p, int(r["Dispatch_Id"]))
        d = rows.setdefault(key, {"name": name, "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "grid": r["Grid_Size"], "wg": r["Workgroup_Size"], "vgpr": r["VGPR_Count"], "lds": r["LDS_Block_Size"]})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
# group per pass; take the last fit: dispatches after the last init (take last ~60 per pass)
bypass = collections.defaultdict(list)
for (p, i), d in rows.items(): bypass[p].append((i, d))
for p, lst in bypass.items():
    lst.sort()
    sel = [d for i, d in lst if ("lean_img" in d["name"] or "lloyd_t1" in d["name"] or "exact_cand" in d["name"] or "exact_rows" in d["name"])]
    sel = sel[-42:]
    print("==", p)
    for d in sel:
        ms = d["ms"]; clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e9
        wc = d.get("SQ_WAVE_CYCLES", 0)
        out = "%-28s %7.3f clk%.2f" % (d["name"][:28], ms, clk)
        if wc:
            out += " wait%.2f inst%.2f act%.2f" % (d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc, d["SQ_ACTIVE_INST_ANY"] / wc)
            out += " mfma%.2f" % (d["SQ_VALU_MFMA_BUSY_CYCLES"] / (ms * 1e-3 * clk * 1e9 * 1024)) if clk else ""
        if "SQ_INSTS_VALU" in d:
            cyc = ms * 1e-3 * clk * 1e9
            out += " valu%.2fG lds%.2fG vmem%.3fG mfma%.3fG salu%.2fG valuact%.2f ldsact%.2f" % (d["SQ_INSTS_VALU"]/1e9, d["SQ_INSTS_LDS"]/1e9, d["SQ_INSTS_VMEM"]/1e9, d["SQ_INSTS_MFMA"]/1e9, d["SQ_INSTS_SALU"]/1e9, d["SQ_ACTIVE_INST_VALU"]*4/(cyc*1024), d["SQ_ACTIVE_INST_LDS"]*4/(cyc*1024))
        if "SQ_LDS_BANK_CONFLICT" in d:
            cyc = ms * 1e-3 * clk * 1e9
            out += " bankconf%.3f waitlds%.3f lvl_vmem%.1f" % (d["SQ_LDS_BANK_CONFLICT"]/(cyc*256), d["SQ_WAIT_INST_LDS"]/wc, d["SQ_INST_LEVEL_VMEM"]/max(d["SQ_INSTS_VMEM"],1))
        print(out)
