"""Which launches precede each __amd_rocclr_copyBuffer in a rocprofv3 kernel trace (dev tool)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = collections.Counter()
for i, r in enumerate(rows):
    if "copyBuffer" in r["Kernel_Name"]:
        prev[rows[i - 1]["Kernel_Name"][:60] if i else "-"] += 1
print("copyBuffer total", sum(prev.values()))
for k, v in prev.most_common(20):
    print(f"{v:6d}  after {k}")
