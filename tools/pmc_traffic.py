"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; csv output) into profiles/traffic.json.

HBM bytes per launch of each kernel = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: the counters are in KiB, and on gfx950
FETCH_SIZE tallies half the bytes of 16-B-per-lane reads (MI355X_MICROARCH.md, HBM / rocprofv3 section).  The raw
values are kept next to the corrected ones.

Calibrated per access width on the box (tools/calib_traffic.hip -> profiles/r3/calib_traffic.json): the x2 holds for
coalesced 4-, 8- and 16-B/lane reads alike, and a random 16-B row gather counts 128 B (the missed line) after it;
WRITE_SIZE is exact for coalesced stores and counts a 32-B sector per partial store.  So one factor serves every
kernel here -- but FETCH_SIZE counts the L2's memory-side requests INCLUDING Infinity-Cache hits: a kernel whose
gathered rows sit in the 256 MiB cache (k_edge_len's 160 MB of positions) can read "more than HBM bandwidth".  The
bytes are L2-miss traffic, an upper bound on HBM traffic.

usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <points> <k> [out.json]
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path, newline="") as fh:
        for row in csv.DictReader(fh):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            vals[name].append(float(row["Counter_Value"]))
    return vals


def short(name):
    base = name.split("(")[0]
    return base.replace("void ", "").replace("pcd::", "").strip()


def main():
    fetch_csv, write_csv = sys.argv[1], sys.argv[2]
    points, k = int(sys.argv[3]), int(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        if "pcd::" not in name:
            continue
        f = fetch.get(name, [])
        w = write.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        entry = {"launches_fetch": len(f), "launches_write": len(w),
                 "fetch_size_kib_raw": fk, "write_size_kib_raw": wk}
        if fk is not None and wk is not None:
            entry["hbm_bytes_per_launch"] = (2.0 * fk + wk) * 1024.0
        kernels.setdefault(short(name), []).append(dict(entry, symbol=name))
    # bytes of one seeded iteration: every per-iteration kernel's average bytes x its launches, over the number of
    # iterations (= NVT2 launches); one-time kernels (grid build, load/store, the dense first re-anchoring) excluded
    one_time = ("k_bbox", "k_sample", "k_keys", "k_gather_sorted", "k_count_starts", "k_brick_flags", "k_insert",
                "k_load", "k_store", "k_edge_len", "k_knn<", "k_nn1", "k_radius", "k_dense_radius", "k_knn_dense_q")
    dense = re.compile(r"k_knn_(redo_wave|requery|nvt1)<\d+, true")   # the dense first re-anchoring / unseeded K1
    n_iter = sum(e["launches_fetch"] for kn, v in kernels.items() if kn.startswith("k_nvt2<32") for e in v) or None
    per_iter = None
    if n_iter:
        per_iter = 0.0
        for kname, v in kernels.items():
            if any(t in kname for t in one_time) or dense.search(kname):
                continue
            for e in v:
                if e.get("hbm_bytes_per_launch") is not None:
                    per_iter += e["hbm_bytes_per_launch"] * e["launches_fetch"] / n_iter
    # the build the counters measured (the in-tree libpcd.so, or PCD_LIB): the bench reads the file only when its own
    # library has the same build id
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                    "normal-guided-pointcloud-denoiser_amd"))
    import pcd_native
    res = {"build_id": pcd_native.build_id(), "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes, csv; "
                     "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch (gfx950 FETCH_SIZE counts half; x2 "
                     "calibrated for 4/8/16-B reads and 16-B gathers, profiles/r3/calib_traffic.json); L2-miss bytes "
                     "including Infinity-Cache hits (an upper bound on HBM bytes)",
           "points": points, "k": k, "iterations": n_iter, "per_iteration_bytes": per_iter,
           "source": os.path.relpath(fetch_csv), "kernels": kernels}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for kname, v in kernels.items():
        for e in v:
            print(kname, e.get("hbm_bytes_per_launch"), e["launches_fetch"], e["launches_write"])


if __name__ == "__main__":
    main()
