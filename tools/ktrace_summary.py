"""Per-kernel totals of a rocprofv3 --kernel-trace CSV: total ms (divided by --reps), dispatch
count and the first few dispatch times, largest first.

    python tools/ktrace_summary.py <run_kernel_trace.csv> [--reps N] [--top K]"""
import collections
import csv
import re
import sys


def main(argv):
    args = list(argv)
    reps, top = 1, 12
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    if "--top" in args:
        i = args.index("--top")
        top = int(args[i + 1])
        del args[i:i + 2]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(args[0])):
        m = re.search(r"(oap_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        agg[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
        head = " ".join("%.2f" % x for x in v[:5])
        print("%9.3f ms/rep  n=%-4d %s  [%s]" % (sum(v) / reps, len(v), k, head))


if __name__ == "__main__":
    main(sys.argv[1:])
