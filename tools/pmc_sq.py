"""Per-kernel SQ counter summary from one rocprofv3 --pmc pass (csv): averages per launch, plus the fractions
WAIT_ANY / WAVE_CYCLES, WAIT_INST_ANY / WAVE_CYCLES, ACTIVE_INST_ANY / WAVE_CYCLES and VALU instructions per wave.

usage: python tools/pmc_sq.py <counter_collection.csv>
"""
import csv
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    with open(sys.argv[1], newline="") as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("pcd::", "").strip()
            if "rocprim" in name or "at::" in name or "__amd" in name:
                continue
            vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in sorted(vals.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        waves = avg.get("SQ_WAVES", 0.0) or 1.0
        parts = [f"{name:34s} launches={len(next(iter(cs.values())))}"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in avg:
                parts.append(f"{c[3:].lower()}={avg[c] / wc:.2f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if c in avg:
                parts.append(f"{c[3:].lower()}/wave={avg[c] / waves:.0f}")
        for c in sorted(avg):
            if not c.startswith("SQ_"):
                parts.append(f"{c}={avg[c]:.4g}")
        parts.append(f"waves={waves:.0f}")
        print(" ".join(parts))


if __name__ == "__main__":
    main()
