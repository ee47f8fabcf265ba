"""Dev tool: per-call kernel breakdown from a rocprofv3 rocpd database (.db): dispatches are cut
into calls at every launch of the kernel named by --start (default nms_prep), calls are grouped
in runs of --per (default 23 = nms_bench's 3 warmups + 20 timed), and the mean duration per
kernel per group is printed in microseconds."""
import argparse, collections, re, sqlite3
ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--start", default="nms_prep_kernel")
ap.add_argument("--per", type=int, default=23)
ap.add_argument("--labels", default="")
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute("select name, duration from kernels order by start").fetchall()
calls, cur = [], None
for name, dur in rows:
    short = re.sub(r"\(.*", "", name).split("::")[-1]
    if a.start in short:
        cur = collections.defaultdict(float)
        calls.append(cur)
    if cur is not None:
        cur[short] += dur / 1e3
labels = a.labels.split(",") if a.labels else []
for g in range(0, len(calls), a.per):
    grp = calls[g:g + a.per]
    keys = sorted({k for cl in grp for k in cl})
    lab = labels[g // a.per] if g // a.per < len(labels) else f"group {g // a.per}"
    tot = sum(sum(cl.values()) for cl in grp) / len(grp)
    print(f"{lab}: total {tot:.1f} us; " + ", ".join(f"{k} {sum(cl.get(k, 0) for cl in grp) / len(grp):.1f}" for k in keys))
