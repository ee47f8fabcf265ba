"""Dev tool: the end of one training step from a rocprofv3 --kernel-trace CSV -- when each queue
finishes, how long the main queue waits for the weight-gradient queue, and the kernels of the last
`tail_ms` per queue.  The step = the kernels between the last two `pack_weight_batched` launches.
    python tools/step_tail.py run_kernel_trace.csv [tail_ms]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tail = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "pack_weight_batched" in r["Kernel_Name"]]
lo, hi = (marks[-2], marks[-1]) if len(marks) >= 2 else (0, len(rows))
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])


def fam(n):
    n = re.sub(r"<.*", "", n)
    n = re.sub(r"^void ", "", n).replace("yms::", "")
    return n.split("(")[0][:44]


q = collections.defaultdict(list)
for r in step:
    q[r["Queue_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, fam(r["Kernel_Name"])))
t1 = max(e for v in q.values() for _, e, _ in v)
print(f"step {t1 / 1e6:.3f} ms, {len(step)} kernels")
for qid, ks in sorted(q.items(), key=lambda kv: -len(kv[1])):
    busy = sum(e - s for s, e, _ in ks)
    print(f"queue {qid}: {len(ks)} kernels, busy {busy / 1e6:.3f} ms, first start {ks[0][0] / 1e6:.3f}, "
          f"last end {max(e for _, e, _ in ks) / 1e6:.3f} ms")
for qid, ks in sorted(q.items(), key=lambda kv: -len(kv[1])):
    print(f"-- queue {qid}, kernels ending in the last {tail} ms")
    for s, e, n in ks:
        if e >= t1 - tail * 1e6:
            print(f"   {s / 1e6:8.3f} - {e / 1e6:8.3f}  {(e - s) / 1e3:7.1f} us  {n}")

# the largest idle gaps of the busiest queue (what ran before / after)
qid, ks = max(q.items(), key=lambda kv: len(kv[1]))
gaps = sorted(((ks[i + 1][0] - ks[i][1], i) for i in range(len(ks) - 1)), reverse=True)[:15]
print(f"-- queue {qid}: idle {sum(max(0, ks[i + 1][0] - ks[i][1]) for i in range(len(ks) - 1)) / 1e6:.3f} ms in gaps; largest:")
for g, i in gaps:
    print(f"   {g / 1e3:7.1f} us at {ks[i][1] / 1e6:8.3f} ms  after {ks[i][2]}  before {ks[i + 1][2]}")

# every kernel of the busiest queue in a window [a, b] ms (argv 3, 4)
if len(sys.argv) > 4:
    a, b = float(sys.argv[3]) * 1e6, float(sys.argv[4]) * 1e6
    print(f"-- queue {qid}, kernels in [{sys.argv[3]}, {sys.argv[4]}] ms")
    for s, e, n in ks:
        if e >= a and s <= b:
            print(f"   {s / 1e6:8.3f} - {e / 1e6:8.3f}  {(e - s) / 1e3:7.1f} us  {n}")
