"""Critical-path view of one training step from a rocprofv3 --kernel-trace CSV (dev tool).

Picks the last complete step (between the last two `pack_weight_batched` launches), then per
queue: busy time, idle gaps, and per kernel family the time it occupies on that queue.
    python tools/step_timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "pack_weight_batched" in r["Kernel_Name"]]
if len(marks) >= 2:
    lo, hi = marks[-2], marks[-1]
else:
    lo, hi = 0, len(rows)
step = rows[lo:hi]
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
print(f"step window {(t1 - t0) / 1e6:.3f} ms, {len(step)} kernels")


def fam(n):
    n = re.sub(r"<.*", "", n)
    n = re.sub(r"^void ", "", n)
    n = n.replace("yms::", "")
    return n.split("(")[0][:40]


byq = collections.defaultdict(list)
for r in step:
    byq[r["Queue_Id"]].append(r)
for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    busy = 0
    end = int(rs[0]["Start_Timestamp"])
    gaps = []
    fams = collections.Counter()
    for r in rs:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > end:
            gaps.append(s - end)
        busy += max(0, e - max(s, end))
        end = max(end, e)
        fams[fam(r["Kernel_Name"])] += e - s
    print(f"queue {q}: {len(rs)} kernels, busy {busy / 1e6:.3f} ms, idle gaps {sum(gaps) / 1e6:.3f} ms "
          f"(n={len(gaps)}, >20us: {sum(g for g in gaps if g > 20000) / 1e6:.3f} ms)")
    for k, v in fams.most_common(14):
        print(f"   {v / 1e6:8.3f} ms  {k}")

# tail of the step: the last kernels per queue (relative ms) -- is the side stream backlogged
# when the main stream's backward ends?
print("last 24 kernels of the step (queue, start..end ms, name):")
for r in step[-24:]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"  q{r['Queue_Id']:>3} {s:8.3f}..{e:8.3f}  {fam(r['Kernel_Name'])}")

# the largest idle gaps of the busiest queue, with the kernels around them
q1 = sorted(byq.items(), key=lambda kv: -len(kv[1]))[0][1]
gl = []
end, prev = int(q1[0]["Start_Timestamp"]), None
for r in q1:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > end:
        gl.append((s - end, (end - t0) / 1e6, fam(prev["Kernel_Name"]) if prev else "", fam(r["Kernel_Name"])))
    if e > end:
        end, prev = e, r
print("largest idle gaps on the main queue (us, at ms, after -> before):")
for g, at, a, b in sorted(gl, reverse=True)[:25]:
    print(f"  {g / 1e3:7.1f} us @ {at:7.3f}  {a} -> {b}")
