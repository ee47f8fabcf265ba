"""Dev tool: mean duration per NMS / decode kernel from a rocprofv3 rocpd database (.db)."""
import collections, re, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
agg = collections.defaultdict(list)
for n, d in c.execute("select name, duration from kernels"):
    k = re.sub(r"\(.*", "", n)
    if "nms" in k or "decode" in k:
        agg[k].append(d)
tot = 0.0
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    us = sum(v) / len(v) / 1e3
    tot += us if "nms" in k else 0.0
    print(f"{k[:60]:60s} n={len(v):4d} avg={us:8.2f} us")
print(f"nms kernels per call: {tot:.1f} us")
