"""Per-kernel averages of the SQ counter passes written by scripts/sq_pmc.sh, merged.
usage: python scripts/sq_summary.py gpurun_out/TAG.p1 gpurun_out/TAG.p2 ... > profiles/x.csv
Adds VALU_per_MFMA = SQ_INSTS_VALU / SQ_INSTS_MFMA and MFMA_busy = SQ_VALU_MFMA_BUSY_CYCLES /
(4 SIMDs x SQ_BUSY_CYCLES-normalised GRBM cycles are not collected: busy is reported per wave
as SQ_VALU_MFMA_BUSY_CYCLES / (SQ_WAVE_CYCLES x 4) where both passes hold them)."""
import csv
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"].split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for v in vals.values() for c in v})
w = csv.writer(sys.stdout)
w.writerow(["kernel"] + cols + ["VALU_per_MFMA"])
for k, v in vals.items():
    avg = {c: sum(v[c]) / len(v[c]) for c in v}
    ratio = avg["SQ_INSTS_VALU"] / avg["SQ_INSTS_MFMA"] if avg.get("SQ_INSTS_MFMA") else ""
    w.writerow([k] + [f"{avg[c]:.4g}" if c in avg else "" for c in cols] +
               [f"{ratio:.3f}" if ratio != "" else ""])
