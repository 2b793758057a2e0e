"""Per-kernel HBM traffic from the two rocprofv3 PMC passes (scripts/pmc_traffic.sh).

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM):
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is doubled;
WRITE_SIZE is taken as is.  Output: CSV kernel,calls,avg_read_MB,avg_write_MB,avg_total_MB
usage: python scripts/pmc_summary.py gpurun_out/TAG > profiles/rN_pmc_traffic.csv
"""
import csv
import sys
from collections import defaultdict

base = sys.argv[1]
acc = defaultdict(lambda: {"calls": 0, "FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0})
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    seen = defaultdict(int)
    for r in csv.DictReader(open(f"{base}.{ctr}/run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0]
        acc[name][ctr] += float(r["Counter_Value"])
        seen[name] += 1
    for k, v in seen.items():
        acc[k]["calls"] = max(acc[k]["calls"], v)
w = csv.writer(sys.stdout)
w.writerow(["kernel", "calls", "avg_read_MB", "avg_write_MB", "avg_total_MB"])
rows = []
for k, v in acc.items():
    c = max(v["calls"], 1)
    rd = 2.0 * v["FETCH_SIZE"] * 1024 / c / 1e6
    wr = v["WRITE_SIZE"] * 1024 / c / 1e6
    rows.append((rd + wr, k, c, rd, wr))
for tot, k, c, rd, wr in sorted(rows, reverse=True):
    w.writerow([k, c, f"{rd:.2f}", f"{wr:.2f}", f"{tot:.2f}"])
