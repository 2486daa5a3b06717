"""Average per-dispatch PMC values per kernel from rocprofv3 --pmc csv passes.

    python scripts/pmc_summary.py <pmc dir> [--json out.json]

With --json, writes {kernel: {counter: avg, ..., "hbm_read_bytes", "hbm_write_bytes", "hbm_bytes"}} where
the HBM bytes follow MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE
reports half of a coalesced streaming read, so it is doubled.
"""
import collections
import csv
import glob
import json
import sys


def short(name: str) -> str:
    for k in ("k_stage_multi", "k_propagate_weigh_multi", "k_resample_final_multi", "k_resample_multi",
              "k_weigh_pk_multi", "k_group_top_multi", "k_group_multi", "k_top_wide_multi", "k_top_multi",
              "k_weigh_pk", "k_weigh_stream", "k_group_top", "k_group", "k_top_wide", "k_top", "k_propagate_weigh",
              "k_resample_final", "k_resample_owners", "k_resample", "k_frame2", "k_frame", "k_regen", "k_import", "k_export",
              "k_weights_export"):
        if k in name:
            return k
    return name[:60]


def main():
    d = sys.argv[1]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "rocclr" in name or "__amd" in name:
                continue
            acc[short(name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in sorted(acc.items()):
        print(k)
        row = {}
        for c, v in sorted(cs.items()):
            row[c] = sum(v) / len(v)
            print(f"   {c:28s} {row[c]:16.1f}  (n={len(v)})")
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            row["hbm_read_bytes"] = 2.0 * row["FETCH_SIZE"] * 1024.0
            row["hbm_write_bytes"] = row["WRITE_SIZE"] * 1024.0
            row["hbm_bytes"] = row["hbm_read_bytes"] + row["hbm_write_bytes"]
            print(f"   {'=> HBM bytes/launch':28s} {row['hbm_bytes']:16.0f}")
        res[k] = row
    if out:
        json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
