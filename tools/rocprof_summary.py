#!/usr/bin/env python3
"""Condense rocprofv3 output of `bench.py` into the per-family summaries kept under profiles/.

    python tools/rocprof_summary.py stats  <kernel_stats.csv>            > profiles/rNN_..._stats.txt
    python tools/rocprof_summary.py pmc    <counter_collection.csv> ...  > profiles/rNN_..._traffic.json

`stats`: the rocprofv3 --kernel-trace --stats table regrouped by kernel family.  The conv
families are the ones bench.py's roofline aggregates (yms_conv_fwd / _dgrad / _wgrad calls):
  conv_nt MODE 0  -> yms_conv_fwd   (one launch per call)
  conv_nt MODE 1/2-> yms_conv_dgrad (one launch per call; MODE 2 = stride-2 parity classes)
  conv_wgrad + wgrad_reduce -> yms_conv_wgrad (one or two launches per call)
so "avg us per conv call" here is directly comparable with bench.py's roofline.avg_launch_us.

`pmc`: per-dispatch FETCH_SIZE / WRITE_SIZE (KB; collected in separate passes since they
do not fit one TCC pass on gfx950) and SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE, averaged
per family.  HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950
FETCH_SIZE tallies 128-B requests of 16-B/lane streaming loads at 64 B
(MI355X_MICROARCH.md "HBM [CDNA4]").  Infinity-Cache (256 MiB) hits are counted by the
fabric-side counters, i.e. this is "bytes below L2", an upper bound on HBM bytes.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def family(name):
    # conv_nt_kernel<T, KS, MODE, EPI, BM, BN, WGM, WGN>: EPI 0 (affine) / 1 (BN stats) are
    # forward launches, 2 (store) / 3 (accumulate) are dgrad launches
    m = re.search(r"conv_ntp?_kernelI(DF16b|DF16_|f)Li(\d+)ELi(\d+)ELi(\d+)E", name)
    if m:
        return "conv_fwd" if int(m.group(4)) <= 1 else "conv_dgrad"
    m = re.search(r"conv_ntp?_kernel<(.*)>", name)
    if m:   # demangled (rocprof garbles T/KS): MODE and EPI are the first two numeric arguments
        nums = [a.strip() for a in m.group(1).split(",") if a.strip().isdigit()]
        epi = int(nums[1])
        return "conv_fwd" if epi <= 1 else "conv_dgrad"
    # every weight-gradient kernel behind yms_conv_wgrad: the im2col TT kernel, the LDS-DMA ring
    # (wgrad_ring.hip), the halo-tiled 3x3 kernel (wgrad_halo.hip) and their split-K reducer
    if ("conv_wgrad_kernel" in name or "conv_wgrad_ring_kernel" in name or "conv_wgrad_halo_kernel" in name
            or "wgrad_reduce_kernel" in name) and "stem" not in name and "dwconv" not in name:
        return "conv_wgrad"
    m = re.search(r"yms::(\w+?)(?:_kernel)?[(<]", name) or re.search(r"_ZN3yms\d+(\w+?)(?:_kernel)?I", name) \
        or re.search(r"N3yms\d+(\w+)E", name)
    if m:
        return m.group(1)
    return name[:48]


def is_call_head(name):
    """Kernels that start one yms_conv_* call (the wgrad reducer does not)."""
    return ("conv_nt_kernel" in name or "conv_ntp_kernel" in name or "conv_wgrad_kernel" in name
            or "conv_wgrad_ring_kernel" in name or "conv_wgrad_halo_kernel" in name)


def stats(path):
    fam = defaultdict(lambda: [0, 0.0, 0])   # launches, total ns, call heads
    for r in csv.DictReader(open(path)):
        f = family(r["Name"])
        fam[f][0] += int(r["Calls"])
        fam[f][1] += float(r["TotalDurationNs"])
        if is_call_head(r["Name"]):
            fam[f][2] += int(r["Calls"])
    tot = sum(v[1] for v in fam.values())
    print(f"# rocprofv3 --kernel-trace --stats, regrouped by family ({path})")
    print(f"{'family':28s} {'launches':>9s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
    for f, (n, ns, _) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{f:28s} {n:9d} {ns / 1e6:10.3f} {ns / n / 1e3:9.2f} {100 * ns / tot:6.2f}")
    conv = [fam[k] for k in ("conv_fwd", "conv_dgrad", "conv_wgrad") if k in fam]
    calls = sum(v[2] for v in conv)
    ns = sum(v[1] for v in conv)
    if calls:
        print(f"\nconv calls (fwd+dgrad+wgrad): {calls}, {ns / 1e6:.3f} ms, avg {ns / calls / 1e3:.2f} us per call")
        for k in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
            if k in fam and fam[k][2]:
                print(f"  {k:12s} calls {fam[k][2]:6d}  avg {fam[k][1] / fam[k][2] / 1e3:8.2f} us per call")


def pmc(paths):
    json.dump(pmc_families(paths), sys.stdout, indent=1, sort_keys=True)
    print()


def traffic(out_dir):
    """profile_round.sh output dir -> {mode: {families, conv_hbm_bytes_per_call, ...}}."""
    import os
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.environ.get("YMS_LIB") or os.path.join(root, "yolo-ms_amd", "yms", "libyms.so")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE "
                     "SQ_BUSY_CYCLES, separate passes of `bench.py --mode M --steps 2 --warmup 1`; "
                     "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 half-counted 128-B reads)",
           # the library the passes ran: bench.py attaches this profile's traffic only to runs of
           # the same build (a stale profile must not be reported as current)
           "libyms_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest()}
    for mode in ("train", "infer"):
        paths = [os.path.join(out_dir, f"pmc_{mode}_{c}", "run_counter_collection.csv")
                 for c in ("fetch_size", "write_size", "sq_valu_mfma_busy_cycles")]
        paths = [p for p in paths if os.path.exists(p)]
        if not paths:
            continue
        fam = pmc_families(paths)
        d = {"families": fam}
        if "_conv_all" in fam:
            d["conv_hbm_bytes_per_call"] = fam["_conv_all"]["hbm_bytes_per_call"]
        busy = sum(fam[f].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) * fam[f]["dispatches"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
                   for f in ("conv_fwd", "conv_dgrad", "conv_wgrad") if f in fam)
        act = sum(fam[f].get("GRBM_GUI_ACTIVE", 0) * fam[f]["dispatches"].get("GRBM_GUI_ACTIVE", 0)
                  for f in ("conv_fwd", "conv_dgrad", "conv_wgrad") if f in fam)
        if act:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy sums 1024 SIMDs (32 per 32x32x16 MFMA)
            d["conv_mfma_busy_frac"] = busy / (act / 8.0 * 1024.0)
        jf = os.path.join(out_dir, f"pmc_{mode}_fetch_size.json")
        try:
            line = json.loads(open(jf).read().strip().splitlines()[-1])
            cfg = line.get("config", {})
            d["bench_config"] = {"workload": cfg.get("workload"), "dtype": line.get("dtype")}
        except Exception:
            pass
        res[mode] = d
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


def pmc_families(paths):
    # per dispatch: counter -> value (rocprofv3 may emit one row per counter per dispatch)
    per = defaultdict(dict)
    names = {}
    for p in paths:
        tag = p
        for r in csv.DictReader(open(p)):
            did = (tag, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            names[did] = r["Kernel_Name"]
            per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    fam = defaultdict(lambda: defaultdict(list))
    for did, cv in per.items():
        f = family(names[did])
        for c, v in cv.items():
            fam[f][c].append(v)
    out = {}
    for f, cs in fam.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = {c: len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        out[f] = d
    conv = [f for f in ("conv_fwd", "conv_dgrad", "conv_wgrad") if f in out and "hbm_bytes_per_launch" in out[f]]
    if conv:
        # per conv *call*: wgrad calls launch kernel + reducer; weight by head launches
        tot_b = sum(out[f]["hbm_bytes_per_launch"] * out[f]["dispatches"]["FETCH_SIZE"] for f in conv)
        heads = 0
        for did, nm in names.items():
            if is_call_head(nm) and "FETCH_SIZE" in per[did]:
                heads += 1
        out["_conv_all"] = {"calls": heads, "hbm_bytes_per_call": tot_b / max(heads, 1)}
    return out


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2])
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2])
    else:
        pmc(sys.argv[2:])
