"""Condense rocprofv3 --pmc passes (p1/p2/p3 under a dir) into one row per (kernel, grid) (dev tool)."""
import collections, csv, glob, os, sys

d = sys.argv[1]
rows = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
order = []
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "conv" not in name and "wgrad" not in name and "dwconv" not in name:
            continue
        short = name.split("<")[0].replace("void ", "").replace("yms::", "")[:24]
        tmpl = name[name.find("<"):name.find(">") + 1][:40] if "<" in name else ""
        key = (short + tmpl, r.get("Grid_Size", r.get("Grid_Size_X", "")))
        if key not in rows:
            order.append(key)
        cn = r["Counter_Name"]
        rows[key][cn] += float(r["Counter_Value"])
        cnt[key][cn] += 1
cols = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
        "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "TCC_HIT_sum", "TCC_MISS_sum",
        "FETCH_SIZE"]
for key in order:
    v = {c: rows[key][c] / max(cnt[key][c], 1) for c in cols if cnt[key][c]}
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    out = [f"{key[0]} grid={key[1]}"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in v:
            out.append(f"{c[3:]}={v[c] / wc:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "GRBM_GUI_ACTIVE" in v:
        # MFMA busy summed over SIMDs (1024) vs GUI-active summed over 8 XCDs
        out.append(f"mfma_busy={v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
        out.append(f"gui_us={v['GRBM_GUI_ACTIVE'] / 8 / 2.1e3:.1f}")
    if "SQ_LDS_IDX_ACTIVE" in v:
        out.append(f"lds_conf={v.get('SQ_LDS_BANK_CONFLICT', 0) / max(v['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
    if "TCC_HIT_sum" in v:
        out.append(f"l2hit={v['TCC_HIT_sum'] / max(v['TCC_HIT_sum'] + v['TCC_MISS_sum'], 1):.3f}")
    if "FETCH_SIZE" in v:
        out.append(f"fetchMB={2 * v['FETCH_SIZE'] / 1024:.1f}")
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_WAIT_INST_LDS"):
        if c in v:
            out.append(f"{c[9:]}={v[c]:.3g}")
    print("  ".join(out))
