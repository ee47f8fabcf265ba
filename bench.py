#!/usr/bin/env python3
"""YOLO-MS-S (reference graph = YOLOv8-s) 640x640 bf16 on MI355X.

Headline `value`: whole-job TRAINING images/sec (BASELINE.json configs[2]: B=64 per GPU,
data-parallel over N GPUs with bucketed RCCL all-reduce overlapped with backward; fwd +
loss + bwd + all-reduce + SGD-nesterov step).  The same line carries the single-GPU
INFERENCE images/sec of configs[1] (B=32: forward + decode + class-wise NMS), the conv
roofline of the dominant kernel family and the CPU-oracle baseline.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yolo-ms_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense bf16, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64, help="training images per GPU (configs[2])")
    ap.add_argument("--infer-batch", type=int, default=32, help="inference batch (configs[1])")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--version", default="s")
    ap.add_argument("--nc", type=int, default=80)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "f32"])
    ap.add_argument("--no-infer", action="store_true")
    ap.add_argument("--loss", default="compute", choices=["compute", "surrogate"],
                    help="compute: the reference's ComputeLoss semantics on the GPU (loss.py:94-677) with "
                         "synthetic targets; surrogate: sum of mean(o^2) over the head maps")
    ap.add_argument("--gts", type=int, default=8, help="synthetic ground-truth boxes per image (--loss compute)")
    ap.add_argument("--ms-version", default="ms-s",
                    help="also time this YOLO-MS (MS-Block / HKS) graph at 1 GPU ('none': skip)")
    ap.add_argument("--nms-overlap", type=int, default=1,
                    help="inference: class-wise NMS of batch k on a second stream, overlapping the "
                         "forward of batch k+1 (0: one stream)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--mode", default="both", choices=["both", "train", "infer"])
    ap.add_argument("--priority", type=int, default=1,
                    help="run the step on a high-priority stream (the weight-gradient side stream keeps "
                         "normal priority, so the critical path wins CU arbitration)")
    ap.add_argument("--graph", type=int, default=0,
                    help="replay each step as one captured HIP graph (1 GPU; the plans are static)")
    return ap.parse_args()


def timed(fn, steps, warmup, world):
    """W untimed warmups, then exactly K steps bracketed by barrier + synchronize on both sides
    (max over ranks).  Also returns the median per-step GPU time from events recorded between
    steps on the compute stream (no host sync inside the timed loop)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    per = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
    med = per[len(per) // 2] if per else 0.0
    if world > 1:
        t = torch.tensor([dt, med], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, med = t[0].item(), t[1].item()
    return dt, med


def graphed(step, warmup):
    """Capture `step` (static inputs, static plan) as one HIP graph and return its replay.  The
    warmup runs eagerly on a side stream first (optimizer state, packed-weight tables, plan caches
    are created outside the capture)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(max(warmup, 2)):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    return g.replay


def add_traffic(roof, mode, workload):
    t, src, busy = pmc_traffic(mode, workload)
    roof["traffic_libyms_sha256"] = loaded_lib_sha256()
    if t is not None:
        roof["traffic"] = round(t)
        roof["traffic_unit"] = "bytes below L2 per conv launch (PMC)"
        roof["traffic_source"] = src
        if busy is not None:
            roof["mfma_busy_frac_pmc"] = round(busy, 4)
    else:
        roof["traffic_source"] = "none: no PMC profile of this workload with the loaded libyms.so build"


def conv_roofline(prof, label):
    rows = [v for k, v in prof.items() if k.startswith("yms_conv_") and v[2]]
    calls = sum(v[0] for v in rows)
    ms = sum(v[1] for v in rows)
    fl = sum(v[2] for v in rows)
    nb = sum(v[3] for v in rows)
    t_roof = sum(v[4] for v in rows)
    ach = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": None, "kernel": label,
            "launches": calls, "avg_launch_us": round(ms * 1e3 / max(calls, 1), 2),
            "algorithmic_gflop_per_launch": round(fl / max(calls, 1) / 1e9, 3),
            # per-launch roofline of each layer's own arithmetic intensity, min(MFMA peak,
            # AI x HBM peak): sum over launches of max(flops / 2.5 PF, bytes / 8 TB/s) against the
            # measured time; bytes = input + output + weights once per launch (algorithmic)
            "by_entry_point": {k.replace("yms_conv_", ""): {
                "launches": v[0], "ms": round(v[1], 4), "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1) if v[1] else 0.0,
                "per_layer_roofline_frac": round(v[4] / v[1], 4) if v[1] else 0.0}
                for k, v in prof.items() if k.startswith("yms_conv_") and v[2]},
            "per_layer_roofline": {
                "t_attainable_ms": round(t_roof, 4), "t_measured_ms": round(ms, 4),
                "frac": round(t_roof / ms, 4) if ms > 0 else 0.0,
                "hbm_bound_launches": sum(v[5] for v in rows),
                "algorithmic_mb_per_launch": round(nb / max(calls, 1) / 1e6, 2),
                "achieved_hbm_gb_s": round(nb / (ms * 1e-3) / 1e9, 1) if ms > 0 else 0.0,
                "peak_hbm_gb_s": HBM_PEAK_GBS}}


VALU_F32_PEAK_TFLOPS = 157.3    # fp32 vector FMA rate, MI355X_MICROARCH.md chip table
DW_NAMES = ("yms_dwconv_fwd", "yms_dwconv_dgrad", "yms_dwconv_wgrad")
BN_NAMES = ("yms_bn_act_bwd_reduce", "yms_bn_act_bwd_apply", "yms_affine_act", "yms_add_views", "yms_add_grad2")


def family_roofline(prof, names, label):
    """Roofline of a non-MFMA kernel family from one profiled step: algorithmic bytes (each operand
    once) and FLOPs per launch against the summed HIP-event durations on the launch streams;
    per launch the attainable time is max(bytes / 8 TB/s, FLOPs / VALU peak)."""
    rows = {k: v for k, v in prof.items() if k in names}
    calls = sum(v[0] for v in rows.values())
    ms = sum(v[1] for v in rows.values())
    if not calls or ms <= 0:
        return None
    fl = sum(v[2] for v in rows.values())
    nb = sum(v[3] for v in rows.values())
    t_roof = sum(v[4] for v in rows.values())
    gbs = nb / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "kernel": label, "launches": calls,
            "ms_per_step": round(ms, 4), "algorithmic_mb_per_launch": round(nb / calls / 1e6, 2),
            "valu_tflops": round(fl / (ms * 1e-3) / 1e12, 2) if fl else None,
            "per_launch_roofline_frac": round(t_roof / ms, 4),
            "by_entry_point": {k.replace("yms_", ""): {
                "launches": v[0], "ms": round(v[1], 4),
                "gb_s": round(v[3] / (v[1] * 1e-3) / 1e9, 1) if v[1] else 0.0,
                "roofline_frac": round(v[4] / v[1], 4) if v[1] else 0.0} for k, v in rows.items()}}


def step_rooflines(prof, dtype_name, what):
    """conv (MFMA) roofline + the depthwise and BN/elementwise families' HBM rooflines of one
    profiled step."""
    roof = conv_roofline(prof, f"conv implicit-GEMM {what} ({dtype_name} MFMA), one step")
    dw = family_roofline(prof, DW_NAMES, "depthwise k x k (VALU, fp32 accumulate)")
    if dw is not None:
        roof["depthwise"] = dw
    bn = family_roofline(prof, BN_NAMES, "BN+SiLU affine / BN backward reduce+apply / branch sums")
    if bn is not None:
        roof["bn_elementwise"] = bn
    return roof


def train_workload(version, a, world):
    tcfg = {"s": "configs[2]: YOLO-MS-S", "l": "configs[3]: YOLO-MS-L",
            "ms-l": "configs[3]: YOLO-MS-L (MS-Block / HKS 3-5-7-9 depthwise graph)",
            "ms-s": "YOLO-MS-S (MS-Block / HKS graph)"}.get(version, f"custom: YOLO-MS-{version.upper()}")
    graph = "" if version.startswith("ms-") else f" (reference YOLOv8-'{version}' graph)"
    allreduce = "bucketed RCCL allreduce+" if world > 1 else ""
    return (f"{tcfg}{graph} {a.size}x{a.size} {a.dtype} training, B={a.batch}/GPU, fwd+loss+bwd+"
            f"{allreduce}SGD-nesterov step")


def infer_workload(version, a):
    icfg = {(640, "bf16"): "configs[1]", (1280, "f16"): "configs[4]"}.get((a.size, a.dtype), "custom")
    if version.startswith("ms-"):
        icfg += f" (YOLO-MS-{version[3:].upper()} MS-Block / HKS graph)"
    elif version != "s":
        icfg += f" (YOLO-MS-{version.upper()} graph)"
    return f"{icfg}: {a.size}x{a.size} {a.dtype} inference B={a.infer_batch} on 1 GPU (forward + decode + class-wise NMS)"


class MeanSquare(torch.autograd.Function):
    """mean(o^2) of a head map: forward is one fp32-accumulating norm reduction (no fp32 copy of
    o), backward writes d/do = 2*o/numel in one elementwise pass (autograd's vector_norm backward
    takes three: a divide by the norm, a masked fill for norm == 0 and a multiply)."""

    @staticmethod
    def forward(ctx, o):
        ctx.save_for_backward(o)
        return torch.linalg.vector_norm(o, dtype=torch.float32).square() / o.numel()

    @staticmethod
    def backward(ctx, g):
        (o,) = ctx.saved_tensors
        return o * (g * (2.0 / o.numel())).to(o.dtype)


_LIB_SHA = None


def loaded_lib_sha256():
    """sha256 of the libyms.so this process runs (yms._lib.LIB_PATH)."""
    global _LIB_SHA
    if _LIB_SHA is None:
        import hashlib
        from yms import _lib
        _LIB_SHA = hashlib.sha256(open(_lib.LIB_PATH, "rb").read()).hexdigest()
    return _LIB_SHA


def pmc_traffic(mode, workload):
    """HBM bytes per conv call from the newest committed PMC profile of the same workload AND the
    same library build (profiles/*_pmc_traffic.json, written by tools/profile_round.sh +
    tools/rocprof_summary.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
    script, with the sha256 of the libyms.so they profiled).  PMC counters cannot be read from
    inside the timed run, so this is the profiled value of the same command on the same kernels;
    None when no profile of this workload was taken with the loaded library (a profile of an
    older build is never attached: its kernels are not the ones timed)."""
    import glob
    sha = loaded_lib_sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_traffic.json")), reverse=True):
        try:
            j = json.load(open(f))
        except Exception:
            continue
        if j.get("libyms_sha256") != sha:
            continue
        d = j.get(mode, {})
        if d.get("bench_config", {}).get("workload") == workload and "conv_hbm_bytes_per_call" in d:
            return d["conv_hbm_bytes_per_call"], os.path.relpath(f, ROOT), d.get("conv_mfma_busy_frac")
    return None, None, None


def cpu_threads():
    """Host threads for the CPU baseline: the box's CPU share for one GPU (OMP_NUM_THREADS, which
    the GPU pool sets to 16 -- os.cpu_count() there reports the whole machine), else all cores."""
    n = int(os.environ.get("OMP_NUM_THREADS") or 0) or os.cpu_count() or 1
    torch.set_num_threads(n)
    return n


def _oracle(version):
    if version.startswith("ms-"):
        from oracle import ms_ref as M
    else:
        from oracle import model_ref as M
    return M


def synth_targets(batch, nc, per_img, seed, device="cpu"):
    """[batch*per_img, 6] collated targets (image, class, cx, cy, w, h normalised), boxes 5-45% of
    the image side, fully inside it (the dataloader's format, dataset.py:235-267)."""
    g = torch.Generator().manual_seed(seed)
    n = batch * per_img
    wh = torch.rand(n, 2, generator=g) * 0.4 + 0.05
    c = torch.rand(n, 2, generator=g) * (1 - wh) + wh / 2
    img = torch.arange(batch).repeat_interleave(per_img).float()
    cls = torch.randint(0, nc, (n,), generator=g).float()
    return torch.cat([img[:, None], cls[:, None], c, wh], 1).to(device)


def cpu_baseline_train(version, nc, size, batch=8, steps=8, loss="compute", gts=8):
    """Oracle (fp32 torch-CPU restatement of the reference graph and loss) train step on host cores."""
    M = _oracle(version)
    from oracle import loss_ref
    threads = cpu_threads()
    sd = M.init_params(version, nc)
    p = {k: (t.clone().requires_grad_(True) if t.is_floating_point() and "running" not in k
             and k != "head.dfl.conv.weight" else t.clone()) for k, t in sd.items()}
    params = [t for k, t in p.items() if t.requires_grad]
    opt = torch.optim.SGD(params, lr=0.01, momentum=0.937, nesterov=True, weight_decay=5e-4)
    x = torch.randn(batch, 3, size, size, generator=torch.Generator().manual_seed(0))
    tg = synth_targets(batch, nc, gts, 0)

    def step():
        opt.zero_grad()
        outs = M.forward(p, version, nc, x, True)
        if loss == "compute":
            loss_ref.compute_loss(list(outs), tg, nc, (size, size))[0].backward()
        else:
            sum((o ** 2).mean() for o in outs).backward()
        opt.step()

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "images/sec", "cores": threads,
            "kind": "port", "sample": f"oracle/{'ms_ref' if version.startswith('ms-') else 'model_ref'}.py train step (fwd+{'loss_ref ComputeLoss' if loss == 'compute' else 'surrogate loss'}+bwd+SGD), fp32, B={batch}, "
            f"{size}x{size}, {steps} timed steps after 1 warmup ({dt:.1f} s), torch threads={threads} "
            f"(OMP_NUM_THREADS share of a host reporting {os.cpu_count()} cpus)"}


def cpu_baseline_infer(version, nc, size, batch=8, steps=12):
    from oracle import nms as onms
    M = _oracle(version)
    sd = M.init_params(version, nc)
    x = torch.randn(batch, 3, size, size, generator=torch.Generator().manual_seed(0))
    threads = cpu_threads()

    def step():
        with torch.no_grad():
            y = M.forward(dict(sd), version, nc, x, False).numpy()
        for b in range(batch):
            onms.postprocess(y[b], 0.25, 0.45)

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "images/sec", "cores": threads,
            "kind": "port", "sample": f"oracle/{'ms_ref' if version.startswith('ms-') else 'model_ref'}.py eval forward + C NMS (1 core), fp32, B={batch}, {steps} timed steps "
            f"({dt:.1f} s), torch threads={threads}"}


def make_sgd(params):
    """The reference's SGD-nesterov step (train.py optimizer settings); one fused multi-tensor
    kernel where torch has it for this device, else the foreach kernels."""
    kw = dict(lr=0.01, momentum=0.937, nesterov=True, weight_decay=5e-4)
    params = list(params)
    try:
        return torch.optim.SGD(params, fused=True, **kw)
    except (RuntimeError, TypeError, ValueError):
        pass
    return torch.optim.SGD(params, foreach=True, **kw)


def measure_ms_family(a, dev, dtype):
    """The MS-Block / HKS graph of the same size class (the reference holds it only as
    a diagram, so these lines are not oracle-pinned like configs[2]): training step with the GPU
    ComputeLoss at the same per-GPU batch, and inference + NMS at the configs[1] batch."""
    from yms import set_compute_dtype
    from yms import ops as yops
    from yolov8.tools.loss import ComputeLoss
    from yolov8.yolov8 import YOLOv8

    steps, warmup = min(a.steps, 40), min(a.warmup, 10)
    out = {"version": a.ms_version, "steps": steps, "warmup": warmup}
    torch.manual_seed(0)
    m = YOLOv8(a.ms_version, a.nc).to(dev)
    m.head.stride = torch.tensor([8.0, 16.0, 32.0])
    set_compute_dtype(m, dtype)
    if a.mode in ("both", "train"):
        m.train()
        opt = make_sgd(m.parameters())
        x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=torch.Generator(device=dev).manual_seed(7))
        crit = ComputeLoss(m.head, a.nc, dev, (a.size, a.size))
        tg = synth_targets(a.batch, a.nc, a.gts, 4321, dev)

        def step():
            opt.zero_grad(set_to_none=True)
            crit.loss_tensor(m(x), tg)[0].backward()
            opt.step()

        dt, med = timed(step, steps, warmup, 1)
        out["train"] = {"value": round(a.batch * steps / dt, 2), "unit": "images/sec",
                        "ms_per_step": round(dt / steps * 1e3, 3), "ms_per_step_median": round(med, 3),
                        "workload": train_workload(a.ms_version, a, 1)}
        log(f"[rank 0] {a.ms_version} train: {out['train']['value']} img/s")
        if not a.no_profile:
            from yms import _lib
            _lib.profile_begin()
            step()
            out["train"]["roofline"] = step_rooflines(_lib.profile_end(), a.dtype, "fwd+dgrad+wgrad")
            add_traffic(out["train"]["roofline"], "train", out["train"]["workload"])
        del opt, x
    if a.mode in ("both", "infer") and not a.no_infer:
        torch.manual_seed(0)
        mi = YOLOv8(a.ms_version, a.nc).to(dev).eval()
        mi.head.stride = torch.tensor([8.0, 16.0, 32.0])
        set_compute_dtype(mi, dtype)
        xi = torch.randn(a.infer_batch, 3, a.size, a.size, device=dev,
                         generator=torch.Generator(device=dev).manual_seed(99))

        ns = torch.cuda.Stream(device=dev) if a.nms_overlap else None

        def istep():
            y = mi(xi)
            if ns is None:
                yops.batched_nms_indices(y, 0.25, 0.45)
                return
            ns.wait_stream(torch.cuda.current_stream(dev))       # as the configs[1] pipeline
            y.record_stream(ns)
            with torch.cuda.stream(ns):
                yops.batched_nms_indices(y, 0.25, 0.45)

        dti, medi = timed(istep, steps, warmup, 1)
        out["infer"] = {"value": round(a.infer_batch * steps / dti, 2), "unit": "images/sec",
                        "ms_per_batch": round(dti / steps * 1e3, 3), "ms_per_batch_median": round(medi, 3),
                        "workload": infer_workload(a.ms_version, a), "nms_overlap": bool(a.nms_overlap)}
        log(f"[rank 0] {a.ms_version} infer: {out['infer']['value']} img/s")
        if not a.no_profile:
            from yms import _lib
            if ns is not None:
                torch.cuda.current_stream(dev).wait_stream(ns)
            _lib.profile_begin()
            istep()
            out["infer"]["roofline"] = step_rooflines(_lib.profile_end(), a.dtype, "fwd")
            add_traffic(out["infer"]["roofline"], "infer", out["infer"]["workload"])
    torch.cuda.empty_cache()
    if not a.no_cpu_baseline:
        # the MS restatement on host cores (oracle/ms_ref.py: the same torch-CPU ops the reference
        # graph uses, with depthwise grouped convs): smaller sample, the graph is ~2x YOLOv8-s on CPU
        log(f"[rank 0] {a.ms_version} cpu baseline...")
        if "train" in out:
            out["train"]["cpu_baseline"] = cpu_baseline_train(a.ms_version, a.nc, a.size, batch=8, steps=3,
                                                              gts=a.gts)
        if "infer" in out:
            out["infer"]["cpu_baseline"] = cpu_baseline_infer(a.ms_version, a.nc, a.size, batch=8, steps=4)
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torchrun (even --nproc-per-node 1) the DP path runs: RCCL process group, bucketed
    # all-reduce hook inside the plan backward, side-stream joins
    distributed = world > 1 or "LOCAL_RANK" in os.environ
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if a.priority:
        # the critical path (forward, BN/dgrad backward chain) on a high-priority stream: it gets its
        # own hardware queue and wins CU arbitration against the side-stream weight gradients
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    dtype = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[a.dtype]

    from yms import _lib, set_compute_dtype
    from yms import ops as yops
    from yolov8.yolov8 import YOLOv8

    torch.manual_seed(0)
    model = YOLOv8(a.version, a.nc).to(dev)
    model.head.stride = torch.tensor([8.0, 16.0, 32.0])
    set_compute_dtype(model, dtype)
    net = model
    if distributed:
        from yms.dist import DataParallel
        net = DataParallel(model)
    result = {}

    # ---------------- training (configs[2]) ----------------
    if a.mode in ("both", "train"):
        model.train()
        opt = make_sgd(model.parameters())
        g = torch.Generator(device=dev).manual_seed(1234 + rank)
        x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=g)
        if a.loss == "compute":
            from yolov8.tools.loss import ComputeLoss
            crit = ComputeLoss(model.head, a.nc, dev, (a.size, a.size))
            tg = synth_targets(a.batch, a.nc, a.gts, 4321 + rank, dev)

        def train_step():
            opt.zero_grad(set_to_none=True)
            outs = net(x)
            if a.loss == "compute":
                loss = crit.loss_tensor(outs, tg)[0]      # device tensor: no host sync in the step
            else:
                # surrogate sum_i mean(o_i^2)
                loss = sum(MeanSquare.apply(o) for o in outs)
            loss.backward()
            opt.step()

        run_train = train_step
        use_graph = bool(a.graph) and not distributed
        if use_graph:
            run_train = graphed(train_step, a.warmup)
        log(f"[rank {rank}] train warmup {a.warmup} + {a.steps} steps, B={a.batch}/GPU, graph={use_graph}")
        dt, med = timed(run_train, a.steps, a.warmup, world)
        result["train"] = {"dt": dt, "med_ms": med, "graph": use_graph, "img_s": world * a.batch * a.steps / dt,
                           "peak_gb": torch.cuda.max_memory_allocated() / 2**30}
        log(f"[rank {rank}] train: {result['train']['img_s']:.1f} img/s ({dt / a.steps * 1e3:.1f} ms/step)")
        if rank == 0 and not a.no_profile:
            _lib.profile_begin()
            train_step()
            prof = _lib.profile_end()
            result["train_prof"] = prof
        del opt, x
        torch.cuda.empty_cache()

    # ---------------- inference (configs[1]) ----------------
    if rank == 0 and a.mode in ("both", "infer") and not a.no_infer:
        # a fresh random-init model (SURVEY 8d input set 1: ~8400 candidates/image, ~105/class);
        # the surrogate-trained weights above collapse every logit to ~0 (all classes tie).
        torch.manual_seed(0)
        imodel = YOLOv8(a.version, a.nc).to(dev).eval()
        imodel.head.stride = torch.tensor([8.0, 16.0, 32.0])
        set_compute_dtype(imodel, dtype)
        xi = torch.randn(a.infer_batch, 3, a.size, a.size, device=dev,
                         generator=torch.Generator(device=dev).manual_seed(99))

        nms_stream = torch.cuda.Stream(device=dev) if a.nms_overlap else None

        def infer_step():
            y = imodel(xi)
            if nms_stream is None:
                yops.batched_nms_indices(y, 0.25, 0.45)
                return
            # serving pipeline: batch k's decode output goes to class-wise NMS on a second stream
            # while batch k+1's forward runs (the greedy NMS of a big segment holds one CU)
            nms_stream.wait_stream(torch.cuda.current_stream(dev))
            y.record_stream(nms_stream)
            with torch.cuda.stream(nms_stream):
                yops.batched_nms_indices(y, 0.25, 0.45)

        run_infer = graphed(infer_step, a.warmup) if a.graph else infer_step
        dti, medi = timed(run_infer, a.steps, a.warmup, 1)
        if nms_stream is not None:
            torch.cuda.current_stream(dev).wait_stream(nms_stream)
        result["infer"] = {"dt": dti, "med_ms": medi, "graph": bool(a.graph),
                           "img_s": a.infer_batch * a.steps / dti}
        log(f"[rank 0] infer: {result['infer']['img_s']:.1f} img/s ({dti / a.steps * 1e3:.2f} ms/batch)")
        if not a.no_profile:
            _lib.profile_begin()
            infer_step()
            result["infer_prof"] = _lib.profile_end()

    if rank == 0 and world == 1 and a.ms_version != "none" and not a.version.startswith("ms-"):
        result["ms"] = measure_ms_family(a, dev, dtype)

    if rank == 0:
        from oracle import model_ref as M
        if a.version.startswith("ms-"):
            # YOLO-MS family: dense conv FLOPs from the plan (the depthwise k x k FLOPs are VALU work
            # and are reported separately, outside the MFMA conv roofline)
            from yms import runner as _r
            _m = YOLOv8(a.version, a.nc).train()
            _p = _r.get_plan(_m, [torch.empty(1, 3, a.size, a.size, device="meta")], dtype, True)
            flops_img = _p.flops
            dw_flops_img = sum(getattr(op, "dw_flops", 0) for op in _p.ops)
        else:
            flops_img = M.count_conv_flops(a.version, a.nc, a.size, a.size)
            dw_flops_img = 0
        line = {"metric": "images/sec (train+infer) YOLO-MS-S 640x640 bf16 at 1/2/4/8 MI355X; mAP parity",
                "unit": "images/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
                "data": f"synthetic (randn images, torch-default random-init weights of the "
                        f"{'YOLO-MS ' + a.version if a.version.startswith('ms-') else 'YOLOv8-' + a.version} graph)"}
        if "train" in result:
            tr = result["train"]
            line["value"] = round(tr["img_s"], 2)
            line["ms_per_step"] = round(tr["dt"] / a.steps * 1e3, 3)
            line["ms_per_step_median"] = round(tr["med_ms"], 3)
            line["config"] = {"workload": train_workload(a.version, a, world),
                              "global_batch": a.batch * world, "per_gpu_batch": a.batch, "img": a.size,
                              "parallelism": f"dp{world}",
                              "loss": (f"ComputeLoss semantics (tools/loss.py:94-677) on the GPU, {a.gts} synthetic "
                                       "GT boxes per image" if a.loss == "compute" else
                                       "surrogate sum(mean(o^2)) over the 3 head maps"),
                              "conv_gflop_per_img_fwd": round(flops_img / 1e9, 3),
                              "depthwise_gflop_per_img_fwd": round(dw_flops_img / 1e9, 3),
                              "peak_hbm_gib": round(tr["peak_gb"], 2),
                              "hip_graph": tr["graph"]}
            if "train_prof" in result:
                line["roofline"] = step_rooflines(result["train_prof"], a.dtype, "fwd+dgrad+wgrad")
                add_traffic(line["roofline"], "train", line["config"]["workload"])
        if "infer" in result:
            inf = {"value": round(result["infer"]["img_s"], 2), "unit": "images/sec",
                   "ms_per_batch": round(result["infer"]["dt"] / a.steps * 1e3, 3),
                   "ms_per_batch_median": round(result["infer"]["med_ms"], 3),
                   "workload": infer_workload(a.version, a), "hip_graph": result["infer"]["graph"],
                   "nms_overlap": bool(a.nms_overlap)}
            if "infer_prof" in result:
                inf["roofline"] = step_rooflines(result["infer_prof"], a.dtype, "fwd")
                add_traffic(inf["roofline"], "infer", inf["workload"])
            line["infer"] = inf
            if "value" not in line:
                line["value"] = inf["value"]
                line["ms_per_step"] = inf["ms_per_batch"]
                line["config"] = {"workload": inf["workload"], "global_batch": a.infer_batch, "img": a.size,
                                  "parallelism": "replica"}
        if "ms" in result:
            line["ms_family"] = result["ms"]
        if world == 1 and not a.no_cpu_baseline:
            log("[rank 0] cpu baseline (oracle on host cores)...")
            if "train" in result:
                line["cpu_baseline"] = cpu_baseline_train(a.version, a.nc, a.size, loss=a.loss, gts=a.gts)
            if "infer" in result:
                cb = cpu_baseline_infer(a.version, a.nc, a.size)
                if "cpu_baseline" in line:
                    line["infer"]["cpu_baseline"] = cb
                else:
                    line["cpu_baseline"] = cb
        for key in ("train_prof", "infer_prof"):
            if key in result:
                log(f"--- {key} (calls, ms, GFLOP) ---")
                for k, v in sorted(result[key].items(), key=lambda kv: -kv[1][1]):
                    log(f"  {k:28s} {v[0]:5d} {v[1]:9.3f} ms {v[2] / 1e9:9.1f}")
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
