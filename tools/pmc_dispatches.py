"""Per-dispatch PMC table of the last fit in rocprofv3 counter passes (tools/gpu.sh pmc steps):
kernel, duration, effective clock, wait / issue fractions, MFMA busy and the instruction mix.

    python tools/pmc_dispatches.py <pass dir> [<pass dir> ...]"""
import collections
import csv
import re
import sys

KERNELS = ("lean_img", "lloyd_t1", "exact_cand", "exact_rows")


def load(pass_dir):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(pass_dir + "/run_counter_collection.csv")):
        m = re.search(r"(oap_\w+)(<[^>(]*>)?", r["Kernel_Name"])
        name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:30]
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        d = rows.setdefault(int(r["Dispatch_Id"]), {"name": name, "ms": ms})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    return [d for _, d in sorted(rows.items())]


def line(d):
    ms = d["ms"]
    clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (ms * 1e-3) / 1e9
    cyc = ms * 1e-3 * clk * 1e9
    out = "%-28s %7.3f clk%.2f" % (d["name"][:28], ms, clk)
    wc = d.get("SQ_WAVE_CYCLES", 0)
    if wc and "SQ_WAIT_ANY" in d:
        out += " wait%.2f inst%.2f act%.2f" % (d["SQ_WAIT_ANY"] / wc, d["SQ_WAIT_INST_ANY"] / wc,
                                               d["SQ_ACTIVE_INST_ANY"] / wc)
        if clk:
            out += " mfma%.2f" % (d["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024))
    if "SQ_INSTS_VALU" in d and cyc:
        out += " valu%.2fG lds%.2fG vmem%.3fG mfma%.3fG salu%.2fG" % tuple(
            d[k] / 1e9 for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_MFMA",
                                 "SQ_INSTS_SALU"))
        out += " valuact%.2f ldsact%.2f" % (d["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024),
                                            d["SQ_ACTIVE_INST_LDS"] * 4 / (cyc * 1024))
    return out


def main(argv):
    for p in argv:
        sel = [d for d in load(p) if any(k in d["name"] for k in KERNELS)][-42:]
        print("==", p)
        for d in sel:
            print(line(d))


if __name__ == "__main__":
    main(sys.argv[1:])
