"""Summarise a rocprofv3 kernel trace: per-kernel stats + the last frames' timeline."""
import csv, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
for r in rows:
    print(r["Name"][:80].ljust(82), r["Calls"], "avg_us=%.2f" % (float(r["AverageNs"]) / 1e3), "pct=%s" % r["Percentage"])
tr = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda t: int(t["Start_Timestamp"]))
last = tr[-int(sys.argv[2]) if len(sys.argv) > 2 else -8:]
t0 = int(last[0]["Start_Timestamp"])
prev_end = None
for t in last:
    s, e = int(t["Start_Timestamp"]), int(t["End_Timestamp"])
    gap = (s - prev_end) / 1e3 if prev_end else 0.0
    print(t["Kernel_Name"][:50].ljust(52), "start=%.2f dur=%.2f gap=%.2f vgpr=%s sgpr=%s lds=%s scratch=%s" % (
        (s - t0) / 1e3, (e - s) / 1e3, gap, t["VGPR_Count"], t["SGPR_Count"], t["LDS_Block_Size"], t["Scratch_Size"]))
    prev_end = e
