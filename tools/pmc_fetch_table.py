"""Per-dispatch HBM read rate of one kernel from a FETCH_SIZE pass (tools/gpu.sh pmc:...:fetch).
On gfx950 FETCH_SIZE tallies each 128-B memory-side read request at 64 B
(/opt/skills/guides/MI355X_MICROARCH.md, 'FETCH_SIZE reports exactly 1/2 ...'), so the bytes are
doubled here; durations are the dispatches' own (under the profiler, slightly longer than in a
plain run).

    python tools/pmc_fetch_table.py <pass dir> --kernel SUBSTR [--min-ms 0.5]"""
import csv
import re
import json
import os
import sys


def main(argv):
    args = list(argv)
    kern, min_ms = None, 0.5
    if "--kernel" in args:
        i = args.index("--kernel")
        kern = args[i + 1]
        del args[i:i + 2]
    if "--min-ms" in args:
        i = args.index("--min-ms")
        min_ms = float(args[i + 1])
        del args[i:i + 2]
    path = os.path.join(args[0], "run_counter_collection.csv")
    by = {}
    for r in csv.DictReader(open(path)):
        if kern and kern not in r["Kernel_Name"]:
            continue
        d = by.setdefault(int(r["Dispatch_Id"]), {
            "kernel": (re.search(r"oap_\w+(<[^>]*>)?", r["Kernel_Name"]) or
                       re.search(r".*", r["Kernel_Name"])).group(0)[:60],
            "ms": (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e6})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = []
    for k in sorted(by):
        d = by[k]
        if d["ms"] < min_ms:
            continue
        gb = 2.0 * d.get("FETCH_SIZE", 0.0) * 1024 / 1e9
        out.append({"dispatch": k, "kernel": d["kernel"], "ms": round(d["ms"], 4),
                    "fetch_size_gb_raw": round(gb / 2, 3), "hbm_read_gb": round(gb, 3),
                    "hbm_read_tb_per_s": round(gb / d["ms"], 3)})
    print(json.dumps({"source": path, "note": "hbm_read = 2 x FETCH_SIZE (128-B requests tallied "
                      "at 64 B on gfx950)", "dispatches": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
