"""Summarise a rocprofv3 kernel_stats.csv (average ms per launch, launches) and, given the redo probe's log, the
re-anchoring kernels' time per re-anchored row.  usage: python tools/kstats.py <kernel_stats.csv> [probe.log]"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    redo = 0
    if len(sys.argv) > 2:
        for line in open(sys.argv[2]):
            m = re.match(r"it\s+(\d+): redo\s+(\d+)", line)
            if m and int(m.group(1)) > 1:
                redo += int(m.group(2))
    for r in rows:
        name = r["Name"].split("(")[0].replace("void ", "").replace("pcd::", "")
        if "at::" in name or "__amd" in name:
            continue
        calls = int(r["Calls"])
        avg = float(r["AverageNs"]) / 1e6
        tot = float(r["TotalDurationNs"]) / 1e6
        extra = ""
        if redo and ("requery<64, false>" in name or "redo_wave<64, false>" in name):
            extra = f"  {tot / redo * 1e6:.2f} ns/redo-row (non-dense launches incl. the first)"
        print(f"{name:40s} calls={calls:4d} avg={avg:8.3f} ms total={tot:9.2f} ms{extra}")


if __name__ == "__main__":
    main()
