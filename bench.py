#!/usr/bin/env python
"""RecBLR training-step benchmark on MI355X (BASELINE.json metric).

One step = RecBLR.calculate_loss (CE over all items) + backward + Adam step at
B=2048 sequences per GPU, L=200, d=128 (H=256), 2 layers, n_items=10,544
(amazon-beauty), train mode (dropout 0.2) — SURVEY.md §8(d).  Inputs are
synthetic RecBole-shaped batches already resident in HBM; weights are the
reference init.  Multi-GPU: one process per GPU (torchrun), batch-DP with
DDP gradient all-reduce over RCCL, weak scaling (2048 per GPU).

Prints ONE JSON line on rank 0 with the throughput, the HBM roofline of the
dominant HIP kernel (HIP-event timed inside the timed region) and the CPU
oracle baseline (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_plan(gpus: int, environ: dict, argv: list, visible_gpus: int | None,
                dry_run: bool = False):
    """What `bench.py --gpus N` must do before anything touches a GPU.

    Returns ("run", None) when this process is a rank of the right world (N = 1
    and no WORLD_SIZE, or WORLD_SIZE == N from torchrun / the self-launch);
    ("launch", cmd) when N > 1 and no WORLD_SIZE is set: cmd starts N rank
    processes (torch.distributed.run, one per GPU, rendezvous on 127.0.0.1)
    as a child of this process; ("error", message) for a world size that
    disagrees with --gpus or more ranks than visible GPUs (never warn and
    run a different world)."""
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", f"--gpus {gpus} but WORLD_SIZE={ws}: the launch disagrees with the request"
        return "run", None
    if gpus < 1:
        return "error", f"--gpus must be >= 1, got {gpus}"
    if gpus == 1:
        return "run", None
    if not dry_run and (visible_gpus or 0) < gpus:
        return "error", f"--gpus {gpus} but only {visible_gpus or 0} GPU(s) visible"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    return "launch", cmd


def _gpus_arg(argv) -> tuple[int, bool]:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true")
    ns, _ = ap.parse_known_args(argv)
    return ns.gpus, ns.dry_run


def _launch_or_check() -> None:
    """Run before any GPU call: self-launch N ranks when --gpus N > 1 came
    without torchrun's env, exit non-zero on a world-size mismatch."""
    gpus, dry = _gpus_arg(sys.argv[1:])
    visible = None
    if "WORLD_SIZE" not in os.environ and gpus > 1 and not dry:
        import torch   # device_count() does not initialise the GPU on this image
        visible = torch.cuda.device_count()
    what, detail = launch_plan(gpus, os.environ, sys.argv[1:], visible, dry)
    if what == "error":
        print(f"bench.py: {detail}", file=sys.stderr, flush=True)
        sys.exit(2)
    if what == "launch":
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get(
            "HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        sys.exit(subprocess.call(detail, env=env))


if __name__ == "__main__":
    _launch_or_check()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from datamining_recblr_amd import kernels  # noqa: E402
from datamining_recblr_amd.distributed import (barrier, init_from_env, max_over_ranks,  # noqa: E402
                                               synthetic_interaction, wrap_ddp)
from datamining_recblr_amd.gemm_tuning import tuned_gemms_active  # noqa: E402
from datamining_recblr_amd.linear import split_gemm_enabled  # noqa: E402
from datamining_recblr_amd.model import RecBLR  # noqa: E402
from datamining_recblr_amd.recbole_compat import Interaction, SyntheticDataset  # noqa: E402

METRIC = "sequences/sec fwd+bwd at B=2048 L=200 d=128; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFS = 157.3     # MI355X dense fp32 MFMA spec (MI355X_MICROARCH.md)
F16_MFMA_PEAK_TFS = 2516.6     # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md)
F16X3_PEAK_TFS = F16_MFMA_PEAK_TFS / 3   # fp32-equivalent: 3 f16 products per fp32 product
DOMINANT = "rb_gate_scan_bwd"  # the HIP kernel moving the most bytes per step


def make_cfg(args):
    return dict(hidden_size=args.hidden, loss_type="CE", num_layers=args.layers,
                dropout_prob=args.dropout, expand=2, d_conv=4, bd_lru_only=False,
                disable_conv1d=False, disable_ffn=False, MAX_ITEM_LIST_LENGTH=args.seq_len)


def _cpu_threads():
    """(threads to use, physical cores visible, logical CPUs visible): the
    physical cores of this process's CPU affinity set (lscpu -p), capped by
    OMP_NUM_THREADS when set (the GPU box allots each one-GPU job a share of
    the host and sets it)."""
    import subprocess

    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    phys = None
    try:
        txt = subprocess.run(["lscpu", "-p=CPU,CORE,SOCKET"], capture_output=True, text=True,
                             timeout=10).stdout
        core_of = {}
        for line in txt.splitlines():
            if line and not line.startswith("#"):
                c, core, sock = line.split(",")[:3]
                core_of[int(c)] = (sock, core)
        phys = len({core_of[c] for c in cpus if c in core_of}) or None
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    n = phys or len(cpus) or (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, phys, len(cpus) or os.cpu_count()


def cpu_baseline(args, state_dict):
    """The CPU oracle (serial-scan restatement of the reference) on a bounded
    sample of the same workload: one fwd+bwd+Adam train step (dropout as the
    GPU step) over `cpu_sample` sequences, median of 3 after 1 warm-up; and
    the scan-only leg (SURVEY.md §8(d) CPU baseline (i)): the serial forward
    scan at [B, C, T] = [2048, 256, 256], median of 3."""
    from oracle import recblr_oracle as orc

    threads, phys, logical = _cpu_threads()
    torch.set_num_threads(threads)
    cfg = make_cfg(args)
    params = {k: v.detach().cpu().clone().requires_grad_(v.dtype.is_floating_point)
              for k, v in state_dict.items()}
    leaves = [p for p in params.values() if p.requires_grad]
    opt = torch.optim.Adam(leaves, lr=1e-3)
    inter = synthetic_interaction(args.cpu_sample, args.seq_len, args.n_items, "cpu", seed=0)
    times = []
    for _ in range(4):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = orc.calculate_loss(params, cfg, inter["item_id_list"], inter["item_length"],
                                  inter["item_id"], p_drop=args.dropout)
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
    med = sorted(times[1:])[1]
    B, C, T = 2048, 2 * args.hidden, 256
    g = torch.Generator().manual_seed(0)
    gates = torch.rand(B, C, T, generator=g) * 0.1 + 0.9
    tokens = torch.randn(B, C, T, generator=g)
    st = []
    for _ in range(3):
        t0 = time.perf_counter()
        orc.serial_scan(gates, tokens)
        st.append(time.perf_counter() - t0)
    smed = sorted(st)[1]
    # BASELINE.md's CPU plan (ii): the whole C1 train step (configs[0]: B=128,
    # L=50, d=64; ml-1m's 3,706 items + padding, synthetic ids)
    cfg1 = dict(cfg, hidden_size=64, MAX_ITEM_LIST_LENGTH=50)
    torch.manual_seed(2020)
    m1 = RecBLR(cfg1, SyntheticDataset(3707))
    p1 = {k: v.detach().clone().requires_grad_(v.dtype.is_floating_point)
          for k, v in m1.state_dict().items()}
    opt1 = torch.optim.Adam([p for p in p1.values() if p.requires_grad], lr=1e-3)
    i1 = synthetic_interaction(128, 50, 3707, "cpu", seed=0)
    t1s = []
    for _ in range(4):
        t0 = time.perf_counter()
        opt1.zero_grad(set_to_none=True)
        orc.calculate_loss(p1, cfg1, i1["item_id_list"], i1["item_length"], i1["item_id"],
                           p_drop=args.dropout).backward()
        opt1.step()
        t1s.append(time.perf_counter() - t0)
    c1med = sorted(t1s[1:])[1]
    cap = os.environ.get("OMP_NUM_THREADS")
    where = (f"{threads} threads ({phys} physical cores / {logical} logical CPUs in this "
             f"process's affinity set; OMP_NUM_THREADS={cap}"
             + (": the box's CPU share for a one-GPU job, which caps the thread count"
                if cap and phys and int(cap) < phys else "") + ")")
    return {"value": round(args.cpu_sample / med, 3), "unit": "sequences/sec", "cores": threads,
            "kind": "port",
            "sample": (f"oracle (serial-scan CPU restatement of RecBLR.py + parallel_scan.py) "
                       f"CE fwd+bwd+Adam train step on {args.cpu_sample} of the {args.batch} "
                       f"sequences, L={args.seq_len}, d={args.hidden}, n_items={args.n_items}, "
                       f"dropout {args.dropout} as the GPU step; median of 3 after 1 warm-up; "
                       f"{med:.2f} s/step on {where}"),
            "c1_train_step": {"config": "configs[0] shape: B=128, L=50, d=64, n_items=3707 "
                                        "(synthetic ids), CE, dropout as the GPU step",
                              "s_per_step": round(c1med, 3),
                              "sequences_per_sec": round(128 / c1med, 1),
                              "note": "the whole oracle train step (fwd+bwd+Adam), median of 3 "
                                      "after 1 warm-up, same threads"},
            "scan_fwd_only": {"shape_BCT": [B, C, T], "s": round(smed, 3),
                              "sequences_per_sec": round(B / smed, 1),
                              "note": "serial_scan (parallel_scan.py:44-60 order, no FMA), "
                                      "median of 3"}}


def _newest_profiles(suffix):
    """profiles/*<suffix>, oldest first by run tag (the name before the
    suffix): r05_final < r05_final2 < r06_v0."""
    files = glob.glob(os.path.join(ROOT, "profiles", "*" + suffix))
    return sorted(files, key=lambda f: os.path.basename(f)[:-len(suffix)])


def pmc_traffic(args, kernel_prefix):
    """HBM bytes per launch of `kernel_prefix` from the newest committed PMC
    summary (profiles/*_pmc_traffic.json, tools/pmc_traffic.py: FETCH_SIZE and
    WRITE_SIZE passes of this bench at its default shape, gfx950 read
    correction applied).  None unless this run is that default shape."""
    if (args.batch, args.seq_len, args.hidden) != (2048, 200, 128):
        return None, None
    files = _newest_profiles("_pmc_traffic.json")
    if not files:
        return None, None
    data = json.load(open(files[-1]))
    for name, k in data.get("kernels", {}).items():
        if name.startswith(kernel_prefix) and k.get("traffic_bytes"):
            return int(k["traffic_bytes"]), os.path.relpath(files[-1], ROOT)
    return None, None


def pmc_mfma(args):
    """MFMA busy fraction of the projection GEMMs from the newest committed PMC
    summary (profiles/*_pmc_mfma.json, tools/pmc_mfma.py:
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x SIMDs)), per kernel family:
    the f16 split kernels (k_gemm_nt_h / k_gemm_tn_h: 3 f16 MFMA products per
    fp32 product), bf16 kernels (configs[4]) and hipBLASLt's fp32 kernels
    (>= 20 GFLOP per launch).  Busy is the fraction of the MFMA pipe's
    cycles, whatever the dtype."""
    if (args.batch, args.seq_len, args.hidden) != (2048, 200, 128):
        return None
    files = _newest_profiles("_pmc_mfma.json")
    if not files:
        return None
    data = json.load(open(files[-1]))
    fam = {"f16x3": [], "bf16": [], "hipblaslt_f32": []}
    for name, k in data.get("kernels", {}).items():
        if not k.get("mfma_util"):
            continue
        if "k_gemm_nt_h" in name or "k_gemm_tn_h" in name:
            fam["f16x3"].append(k["mfma_util"])
        elif k.get("mfma_flops_bf16_per_dispatch", 0) >= 2e10:
            fam["bf16"].append(k["mfma_util"])
        elif k.get("mfma_flops_f32_per_dispatch", 0) >= 2e10:
            fam["hipblaslt_f32"].append(k["mfma_util"])
    out = {f: {"min": min(u), "max": max(u)} for f, u in fam.items() if u}
    if not out:
        return None
    out["source"] = os.path.relpath(files[-1], ROOT)
    return out


def gemm_bytes(by_shape):
    """Algorithmic HBM bytes per step of the projection GEMMs from the
    per-shape labels: fwd / dX (mm_nt, mm_nn) read A [M, K] and write
    out [M, N]; a weight gradient (wgrad) reads dY [M, N] and X [M, K]
    (weights, partials and row-group maxima are negligible)."""
    import re
    total = 0.0
    for label, v in by_shape.items():
        m = re.match(r"(mm_nt|mm_nn)\[(\d+)x(\d+)->(\d+)\]", label)
        if m:
            M, K, N = int(m.group(2)), int(m.group(3)), int(m.group(4))
            total += v["per_step"] * 4.0 * M * (K + N)
            continue
        m = re.match(r"wgrad\[(\d+):(\d+)x(\d+)\]", label)
        if m:
            M, N, K = int(m.group(1)), int(m.group(2)), int(m.group(3))
            total += v["per_step"] * 4.0 * M * (N + K)
    return total


def kernel_report(summ, steps, ntok_step=None, H=None, layers=None):
    """Per-kernel report from a KernelTimer summary: MFMA kernels (FLOP_KERNELS:
    their launches count algorithmic FLOPs) against the f16x3 or fp32 MFMA
    peak, every other kernel's algorithmic bytes against 8 TB/s; the fused
    scan + conv + gate path both by its kernels' own byte counts and against
    SURVEY §8(d)'s fixed model, 20 * ntok * H * 4 B per layer and step
    (ntok = the packed tokens per step).  An HBM fraction above 1 means a
    byte count is wrong: listed under "anomalies" (tests keep it empty)."""
    rep, anomalies = {}, []
    for name, d in summ.items():
        if name in kernels.FLOP_KERNELS:
            tf = d["avg_bytes"] / (d["avg_ms"] * 1e-3) / 1e12
            pk = F16X3_PEAK_TFS if kernels.f16_split_kernel(name) else FP32_MFMA_PEAK_TFS
            rep[name] = {"launches_per_step": d["launches"] / steps,
                         "avg_us": round(d["avg_ms"] * 1e3, 2),
                         "algo_flops": int(d["avg_bytes"]),
                         "achieved_tflops": round(tf, 1),
                         "peak_tflops": round(pk, 1),
                         "frac": round(tf / pk, 4)}
            continue
        gbs = d["avg_bytes"] / (d["avg_ms"] * 1e-3) / 1e9
        rep[name] = {"launches_per_step": d["launches"] / steps,
                     "avg_us": round(d["avg_ms"] * 1e3, 2),
                     "algo_bytes": int(d["avg_bytes"]),
                     "achieved_gbs": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4)}
        if gbs > HBM_PEAK_GBS:
            anomalies.append(name)
    hbm = [d for n, d in summ.items() if n not in kernels.FLOP_KERNELS]
    tot_b = sum(d["bytes"] for d in hbm)
    tot_ms = sum(d["ms"] for d in hbm)
    core = [summ[n] for n in ("rb_conv_silu_fwd", "rb_gate_scan_fwd", "rb_gate_scan_bwd",
                              "rb_conv_silu_bwd", "rb_grl_fwd", "rb_grl_bwd") if n in summ]
    if core:   # BASELINE's target: the fused scan + conv + gate path
        cb = sum(d["bytes"] for d in core)
        cms = sum(d["ms"] for d in core)
        path = {"ms_per_step": round(cms / steps, 4),
                "achieved_gbs": round(cb / (cms * 1e-3) / 1e9, 1),
                "frac": round(cb / (cms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if ntok_step and H and layers:
            mb = 20.0 * ntok_step * H * 4 * layers
            path["model_bytes_per_step"] = int(mb)
            path["model_frac"] = round(mb / (cms / steps * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            path["model"] = ("SURVEY §8(d): 20 * ntok * H * 4 B per layer (fwd 7N + bwd 13N), "
                             "ntok = packed tokens per step, against the path kernels' time")
        rep["scan_conv_gate_path"] = path
    if tot_ms:
        rep["fused_path_total"] = {
            "ms_per_step": round(tot_ms / steps, 4),
            "achieved_gbs": round(tot_b / (tot_ms * 1e-3) / 1e9, 1),
            "frac": round(tot_b / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "every HIP kernel counted in bytes (FLOP_KERNELS excluded)"}
    if anomalies:
        rep["anomalies"] = anomalies
    return rep



def scan_microbench(args, dev, reps=20):
    """BASELINE configs[1]: forward-only parallel_scan at B=2048, C=H=256,
    T=L=200 on the reference layout [B, C, T] (the reference pads T to 256;
    rb_scan_fwd does not need to).  Algorithmic bytes 3*N*4 (R gates, tokens;
    W states)."""
    B, C, T = args.batch, 2 * args.hidden, args.seq_len
    g = torch.rand(B, C, T, device=dev) * 0.1 + 0.9
    x = torch.randn(B, C, T, device=dev)
    kernels.scan_fwd(g, x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        kernels.scan_fwd(g, x)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    gbs = 3 * g.numel() * 4 / (ms * 1e-3) / 1e9
    return {"shape_BCT": [B, C, T], "us": round(ms * 1e3, 1), "achieved_gbs": round(gbs, 1),
            "frac": round(gbs / HBM_PEAK_GBS, 4),
            "sequences_per_sec": round(B / (ms * 1e-3), 1)}


def long_seq_c5(args, env, dev, steps=3, warmup=2):
    """BASELINE configs[4]: long-sequence stress, L = 2048, d = 256, B = 1024
    per GPU, bf16 activations (fp32 recurrence arithmetic, bf16 MFMA GEMMs
    with fp32 accumulation, fp32 parameters and gradients).  One step = one
    GatedRecurrentLayer (the fused conv + gate + scan path with its in/gate/out
    projections) forward + backward on synthetic input; sequences/s over all
    ranks (weak scaling, max-over-ranks time).  The HBM fraction is that of
    the bf16 conv + gate-scan kernels (algorithmic bytes 20*N*2 per step,
    N = B*L*H).  The projections run per shape on our bf16 kernels
    (rb_gemm_nt_bf16; weight gradients on hipBLASLt's split-K) or torch's bf16 GEMMs (hipBLASLt):
    RECBLR_BF16_GEMM=auto (default: ours where faster), 1 (ours on the six NT
    shapes), 0 (hipBLASLt on all nine); projection_gemms_ab times the three."""
    from datamining_recblr_amd.model import GatedRecurrentLayer

    B, L, d = args.c5_batch, 2048, 256
    torch.manual_seed(2020)
    layer = GatedRecurrentLayer(d_model=d).to(dev)
    g = torch.Generator(device=dev).manual_seed(env.rank)
    x = torch.randn(B, L, d, device=dev, generator=g).to(torch.bfloat16).requires_grad_()
    gy = torch.randn(B, L, d, device=dev, generator=g).to(torch.bfloat16)

    def one():
        layer.zero_grad(set_to_none=True)
        x.grad = None
        layer(x).backward(gy)

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    barrier(env)
    # the headline steps untimed per launch (HIP events around every launch
    # cost ~0.5 ms of this step), then a second pass for the kernel summary
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    barrier(env)
    el = max_over_ranks(time.perf_counter() - t0, env, dev)
    with kernels.kernel_timing() as t:
        for _ in range(steps):
            one()
        torch.cuda.synchronize()
    summ = t.summary()
    # the projections on our bf16 kernel (rb_gemm_nt_bf16)
    # vs torch's bf16 GEMMs (hipBLASLt), alternated, best of 2 per variant
    from datamining_recblr_amd import linear as _lin
    saved_g = _lin.set_bf16_gemm(_lin._bf16_gemm)
    arms = (("per_shape_auto", "auto"), ("own_bf16_kernels", "1"), ("torch_hipblaslt", "0"))
    runs = {name: [] for name, _ in arms}
    for _ in range(2):
        for name, on in arms:
            _lin.set_bf16_gemm(on)
            one()
            torch.cuda.synchronize()
            barrier(env)
            t1 = time.perf_counter()
            for _ in range(steps):
                one()
            torch.cuda.synchronize()
            barrier(env)
            runs[name].append(round(1000.0 * max_over_ranks(time.perf_counter() - t1, env, dev)
                                    / steps, 3))
    _lin.set_bf16_gemm(saved_g)
    gemm_ab = {k: {"ms_per_step": min(v), "all": v} for k, v in runs.items()}
    gemm_ab["headline"] = {m: n for n, m in arms}[saved_g]
    path = [summ[n] for n in ("rb_conv_silu_fwd_bf16", "rb_conv_silu_bwd_bf16",
                              "rb_gate_scan_fwd_bf16", "rb_gate_scan_bwd_bf16") if n in summ]
    pb, pms = sum(p["bytes"] for p in path), sum(p["ms"] for p in path)
    gbs = pb / (pms * 1e-3) / 1e9 if pms else None
    kern = {n: {"avg_us": round(summ[n]["avg_ms"] * 1e3, 1),
                "frac": round(summ[n]["avg_bytes"] / (summ[n]["avg_ms"] * 1e-3) / 1e9
                              / HBM_PEAK_GBS, 4)}
            for n in ("rb_conv_silu_fwd_bf16", "rb_conv_silu_bwd_bf16",
                      "rb_gate_scan_fwd_bf16", "rb_gate_scan_bwd_bf16") if n in summ}
    return {"workload": "GatedRecurrentLayer fwd+bwd (BASELINE configs[4])",
            "batch_per_gpu": B, "seq_len": L, "hidden_size": d, "inner_H": 2 * d,
            "dtype": "bf16 storage, fp32 recurrence math", "steps": steps,
            "value": round(env.world_size * B * steps / el, 1), "unit": "sequences/sec",
            "ms_per_step": round(1000.0 * el / steps, 3),
            "projection_gemms_ab": gemm_ab,
            "scan_conv_gate_path": {"ms_per_step": round(pms / steps, 3),
                                    "achieved_gbs": round(gbs, 1) if gbs else None,
                                    "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                                    "kernels": kern}}


def gemm_pattern(args, batch, dev, rounds=7):
    """Each projection GEMM shape beside its streaming floor: the f16x3 NT
    GEMM (linear.mm_nt at the batch's packed row count) alternated on this
    lease with rb_probe_gemm_pattern, which reads the same A rows once and
    writes the same outputs with trivial arithmetic (16-B accesses, the
    epilogue's nontemporal stores).  Median per launch; kernel_over_pattern
    is the GEMM's time in units of that floor."""
    from datamining_recblr_amd import _lib, linear
    from datamining_recblr_amd.kernels import _stream
    d, H = args.hidden, 2 * args.hidden
    M = int(batch["item_length"].sum())
    shapes = {"in.fwd": (d, 2 * H), "in.dX": (2 * H, d), "gates.fwd": (H, 2 * H),
              "gates.dX": (2 * H, H), "out.fwd": (H, d), "out.dX": (d, H),
              "w2.fwd": (4 * d, d), "w2.dX": (d, 4 * d)}
    g = torch.Generator(device=dev).manual_seed(6)
    rmax_r = max(r for r, _ in shapes.values())
    rmax_c = max(c for _, c in shapes.values())
    a_all = torch.randn(M, rmax_r, device=dev, generator=g)
    out = torch.empty(M, rmax_c, device=dev)
    res, tot_k, tot_p = {}, 0.0, 0.0
    for name, (R, C) in shapes.items():
        a = a_all[:, :R].contiguous()
        w = torch.randn(C, R, device=dev, generator=g) * R ** -0.5
        o = out[:, :C]
        st = _stream(a)

        def real():
            linear.mm_nt(a, w)

        def pattern():
            _lib.call_probe("rb_probe_gemm_pattern", a.data_ptr(), M, R, o.data_ptr(), C, st)

        real(), pattern()
        torch.cuda.synchronize()
        ts = {"kernel": [], "pattern": []}
        for _ in range(rounds):
            for key, fn in (("kernel", real), ("pattern", pattern)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                ts[key].append(e0.elapsed_time(e1) * 1e3)
        ku = sorted(ts["kernel"])[rounds // 2]
        pu = sorted(ts["pattern"])[rounds // 2]
        tot_k, tot_p = tot_k + ku, tot_p + pu
        gbs = M * (R + C) * 4 / (pu * 1e-6) / 1e9
        res[name] = {"R": R, "C": C, "kernel_us": round(ku, 1), "pattern_us": round(pu, 1),
                     "pattern_frac": round(gbs / HBM_PEAK_GBS, 4),
                     "kernel_over_pattern": round(ku / pu, 3)}
        del a, w
    return {"rows": M, "shapes": res, "kernel_us": round(tot_k, 1), "pattern_us": round(tot_p, 1),
            "kernel_over_pattern": round(tot_k / tot_p, 3),
            "note": "linear.mm_nt (rb_gemm_nt_h) vs rb_probe_gemm_pattern (the same A reads and "
                    "output writes, trivial math), alternated on this lease; a ratio of 1 would "
                    "be a GEMM at the streaming floor of its own bytes"}


def gate_bwd_pattern(args, batch, dev, rounds=15):
    """The dominant kernel beside a trivial-math kernel with its exact memory
    access pattern (rb_probe_gate_bwd_pattern: the same 5 reads + 4 writes
    per step and channel, strides, wave/lane layout, sequence pairing and
    reverse tile order), alternated on this lease over the bench's packed
    layout (the batch's lengths, longest first, as the model packs them):
    the pattern's rate is the ceiling the memory system grants this
    read/write mix, here and now.  Median per-launch of each."""
    from datamining_recblr_amd import _lib
    from datamining_recblr_amd.kernels import _stream
    H = 2 * args.hidden
    lens = batch["item_length"].to("cpu").sort(descending=True).values
    B = lens.numel()
    offs_h = torch.zeros(B + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=offs_h[1:])
    ntok = int(offs_h[-1])
    offs = offs_h.to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    rg = torch.randn(ntok, 2 * H, device=dev, generator=g)
    xz = torch.randn(ntok, 2 * H, device=dev, generator=g)
    xc = torch.randn(ntok, H, device=dev, generator=g)
    dy = torch.randn(ntok, H, device=dev, generator=g)
    lam = torch.full((H,), -3.0, device=dev)
    carries = torch.zeros(B, kernels.num_tiles(args.seq_len), H, device=dev)
    drg = torch.empty(ntok, 2 * H, device=dev)
    dxc = torch.empty(ntok, H, device=dev)
    dxz = torch.empty(ntok, 2 * H, device=dev)
    part = torch.empty(4, B, H, device=dev)
    z, dz = xz[:, H:], dxz[:, H:]
    st = _stream(xc)

    def real():
        _lib.call("rb_gate_scan_bwd", rg.data_ptr(), 2 * H, xc.data_ptr(), H, z.data_ptr(), 2 * H,
                  lam.data_ptr(), 0, carries.data_ptr(), dy.data_ptr(), drg.data_ptr(), 2 * H,
                  dxc.data_ptr(), H, dz.data_ptr(), 2 * H, part.data_ptr(), part[3].data_ptr(),
                  B, args.seq_len, H, offs.data_ptr(), st)

    def pattern():
        _lib.call_probe("rb_probe_gate_bwd_pattern", rg.data_ptr(), 2 * H, xc.data_ptr(), H,
                  z.data_ptr(), 2 * H, dy.data_ptr(), drg.data_ptr(), 2 * H, dxc.data_ptr(), H,
                  dz.data_ptr(), 2 * H, B, args.seq_len, H, offs.data_ptr(), st)

    ts = {"kernel": [], "pattern": []}
    for fn in (real, pattern):
        fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for name, fn in (("kernel", real), ("pattern", pattern)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts[name].append(e0.elapsed_time(e1) * 1e3)
    nbytes = 9 * ntok * H * 4
    out = {}
    for name, v in ts.items():
        us = sorted(v)[len(v) // 2]
        out[name + "_frac"] = round(nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        out[name + "_us"] = round(us, 2)
    out["kernel_over_pattern"] = round(out["kernel_frac"] / out["pattern_frac"], 4)
    out["note"] = ("rb_gate_scan_bwd vs rb_probe_gate_bwd_pattern (its access pattern, trivial "
                   "math) alternated on this lease over a packed batch of the bench's lengths, "
                   "9 streams x ntok x H x 4 B; the pattern's rate on these boxes moves between "
                   "~0.63 and ~0.75 of 8 TB/s (profiles/r02_kbench_gate_bwd_pattern.log)")
    return out


def ddp_overhead(args, model, batches, dev, rounds=3):
    """What DistributedDataParallel (bucketed gradient all-reduce over RCCL)
    costs one GPU: the same train step on a copy of the model, plain and
    wrapped in DDP inside a one-rank nccl (RCCL) group, alternated `rounds`
    times on this lease, best of each.  At world size 1 the all-reduce moves
    nothing between GPUs, so this is the per-step DDP tax (reducer hooks,
    bucket copies, the RCCL launch) the N-GPU scaling pays on top of xGMI."""
    import copy

    from datamining_recblr_amd.distributed import LossModule, single_rank_group

    twin = copy.deepcopy(model)
    opt = torch.optim.Adam(twin.parameters(), lr=1e-3, fused=True)
    plain = LossModule(twin)
    env1 = single_rank_group("nccl")
    try:
        ddp = wrap_ddp(twin, env1)

        def run(mod, n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                opt.zero_grad(set_to_none=True)
                mod(batches[i % len(batches)]).backward()
                opt.step()
            torch.cuda.synchronize()
            return 1000.0 * (time.perf_counter() - t0) / n

        run(plain, 3)
        run(ddp, 3)
        p_ms, d_ms = [], []
        for _ in range(rounds):
            p_ms.append(run(plain, args.steps))
            d_ms.append(run(ddp, args.steps))
    finally:
        dist.destroy_process_group()
    p, d = min(p_ms), min(d_ms)
    return {"plain_ms_per_step": round(p, 3), "ddp_ms_per_step": round(d, 3),
            "overhead_frac": round(d / p - 1.0, 4), "backend": "nccl (RCCL), world size 1",
            "note": "same lease, same step on a copy of the model, alternated plain/DDP "
                    f"{rounds}x{args.steps} steps, best of each"}


def dry_run_ranks(args):
    """--dry-run: the launch plumbing without a GPU.  Every rank joins a gloo
    group from the env torchrun (or the self-launch) set, all-gathers what it
    sees, and rank 0 prints one JSON line; the world must equal --gpus."""
    env = init_from_env(backend="gloo")
    mine = torch.tensor([env.rank, env.local_rank, env.world_size], dtype=torch.int64)
    if env.distributed:
        got = [torch.empty_like(mine) for _ in range(env.world_size)]
        dist.all_gather(got, mine)
    else:
        got = [mine]
    ranks = [dict(zip(("rank", "local_rank", "world_size"), t.tolist())) for t in got]
    ok = env.world_size == args.gpus and sorted(r["rank"] for r in ranks) == list(range(args.gpus))
    if env.rank == 0:
        print(json.dumps({"dry_run": True, "gpus": args.gpus, "world_size": env.world_size,
                          "ranks": ranks, "ok": ok}), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        raise SystemExit(3)


def allreduce_probe(model, env, dev, reps=20):
    """The gradient exchange alone: one all-reduce (RCCL) of a flat fp32
    buffer the size of all parameters, median of `reps` after 3 warm-ups,
    max over ranks; bus bandwidth as nccl-tests defines it for all-reduce
    (2 (N-1)/N x bytes / time)."""
    n = sum(p.numel() for p in model.parameters())
    buf = torch.ones(n, device=dev)
    for _ in range(3):
        dist.all_reduce(buf)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        barrier(env)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_reduce(buf)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    us = max_over_ranks(sorted(ts)[reps // 2], env, dev) * 1e6
    nbytes = 4 * n
    busbw = 2 * (env.world_size - 1) / env.world_size * nbytes / (us * 1e-6) / 1e9
    return {"bytes": nbytes, "us": round(us, 1), "busbw_gbs": round(busbw, 1),
            "note": "one dist.all_reduce of a flat fp32 buffer of every parameter (RCCL), median "
                    "of 20, max over ranks; in the step DDP buckets it and overlaps it with the "
                    "backward"}


def per_rank_ms(ms: float, env, dev) -> list:
    t = torch.tensor([ms], dtype=torch.float64, device=dev)
    if not env.distributed:
        return [round(ms, 3)]
    got = [torch.empty_like(t) for _ in range(env.world_size)]
    dist.all_gather(got, t)
    return [round(float(x.item()), 3) for x in got]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-seconds", type=float, default=15.0,
                    help="after the warmup, keep running untimed steps for about this long "
                         "so the device clocks reach their sustained state (0: off); a fresh "
                         "box runs the GEMMs ~15%% slower for its first seconds under load")
    ap.add_argument("--batch", type=int, default=2048, help="sequences per GPU")
    ap.add_argument("--seq-len", type=int, default=200)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--n-items", type=int, default=10544)
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--cpu-sample", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--c5-batch", type=int, default=1024,
                    help="sequences per GPU of the long-sequence bf16 run (configs[4])")
    ap.add_argument("--no-c5", action="store_true", help="skip the configs[4] run")
    ap.add_argument("--no-ddp-ab", action="store_true",
                    help="skip the single-GPU DDP overhead A/B (N=1 only)")
    ap.add_argument("--no-full-tail", action="store_true",
                    help="skip the comparison run that evaluates the last layer's "
                         "position-wise tail at every position")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch and rendezvous only: every rank joins a gloo group and rank 0 "
                         "prints the ranks' (rank, local_rank, world_size); no GPU is touched")
    args = ap.parse_args()

    if args.dry_run:
        dry_run_ranks(args)
        return
    env = init_from_env()
    if env.world_size != args.gpus:   # _launch_or_check() exits first; belt and braces
        raise SystemExit(f"bench.py: --gpus {args.gpus} but world size {env.world_size}")
    if env.world_size > 1 and torch.cuda.device_count() < env.world_size:
        raise SystemExit(f"bench.py: world size {env.world_size} but "
                         f"{torch.cuda.device_count()} GPU(s) visible")
    dev = torch.device("cuda", env.local_rank)
    torch.cuda.set_device(dev)

    torch.manual_seed(2020)  # the reference run's seed (LOG51:6); same on every rank
    model = RecBLR(make_cfg(args), SyntheticDataset(args.n_items)).to(dev).train()
    step_mod = wrap_ddp(model, env)
    # the optimizer update: rb_adam_step over every parameter in one launch
    # (datamining_recblr_amd.optim.Adam; 6.112 vs 6.179 ms per step against
    # torch's fused Adam, profiles/r04_v0_bench.log), or RECBLR_ADAM=torch
    from datamining_recblr_amd.optim import Adam as NativeAdam

    def make_opt(kind):
        if kind == "native":
            return NativeAdam(model.parameters(), lr=1e-3)
        return torch.optim.Adam(model.parameters(), lr=1e-3, fused=True)

    adam_kind = os.environ.get("RECBLR_ADAM", "native")
    opt = make_opt(adam_kind)
    batches = [synthetic_interaction(args.batch, args.seq_len, args.n_items, dev,
                                     seed=1000 * env.rank + i) for i in range(4)]

    def step(i, opt_events=None):
        opt.zero_grad(set_to_none=True)
        b = batches[i % len(batches)]
        if isinstance(b, Interaction):   # a CPU batch, moved as RecBole's Trainer does
            b = b.to(dev)
        loss = step_mod(b)
        loss.backward()
        if opt_events is None:
            opt.step()
        else:   # breakdown pass: the optimizer step timed on its own
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            opt.step()
            e1.record()
            opt_events.append((e0, e1))
        return loss

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    # settle: untimed steps, sized from three timed ones (the same count on every rank)
    settle_steps = 0
    if args.settle_seconds > 0:
        t1 = time.perf_counter()
        for i in range(3):
            step(i)
        torch.cuda.synchronize()
        per = max_over_ranks((time.perf_counter() - t1) / 3, env, dev)
        settle_steps = int(args.settle_seconds / max(per, 1e-4))
        for i in range(settle_steps):
            step(i)
        settle_steps += 3
        torch.cuda.synchronize()
    barrier(env)
    torch.cuda.synchronize()

    # timed region: HIP events only around the dominant kernel's launches (the
    # roofline object); timing every launch costs ~5% of host time per step
    timing = kernels.kernel_timing(only={DOMINANT}) if not args.no_kernel_timing else None
    dom_timer = timing.__enter__() if timing else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    barrier(env)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if timing:
        timing.__exit__(None, None, None)
    rank_ms = per_rank_ms(1000.0 * elapsed / args.steps, env, dev)
    # host side of a step: the time to queue one step's launches from an idle
    # device (median of 5) — close to ms_per_step means the host paces the step
    host_ms = []
    for i in range(5):
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        step(i)
        host_ms.append(1000.0 * (time.perf_counter() - t5))
        torch.cuda.synchronize()
    host_enqueue_ms = sorted(host_ms)[2]
    elapsed = max_over_ranks(elapsed, env, dev)

    # N > 1: the exchange on its own, and the same step without DDP on every
    # rank at once (no collective: what each GPU does alone while its
    # neighbours run) — the in-job reference for the scaling efficiency
    multi = None
    if env.world_size > 1:
        from datamining_recblr_amd.distributed import LossModule
        plain = LossModule(model)
        for i in range(2):
            opt.zero_grad(set_to_none=True)
            plain(batches[i % len(batches)]).backward()
            opt.step()
        torch.cuda.synchronize()
        barrier(env)
        t3 = time.perf_counter()
        for i in range(args.steps):
            opt.zero_grad(set_to_none=True)
            plain(batches[i % len(batches)]).backward()
            opt.step()
        torch.cuda.synchronize()
        barrier(env)
        plain_el = max_over_ranks(time.perf_counter() - t3, env, dev)
        plain_value = env.world_size * args.batch * args.steps / plain_el
        value_n = env.world_size * args.batch * args.steps / elapsed
        multi = {"per_rank_ms_per_step": rank_ms,
                 "allreduce": allreduce_probe(model, env, dev),
                 "plain_local_ms_per_step": round(1000.0 * plain_el / args.steps, 3),
                 "efficiency_vs_local_plain": round(value_n / plain_value, 4),
                 "note": "efficiency_vs_local_plain = value / (the same step without DDP run "
                         "concurrently on every rank, summed over ranks): the exchange's and "
                         "DDP's cost at this N; value_N / (N value_1) across separate runs is "
                         "computed by the driver from its own 1-GPU line"}

    # per-kernel / per-GEMM breakdown: a second pass with every launch timed
    timer = breakdown_ms = None
    opt_events = []
    if not args.no_kernel_timing:
        with kernels.kernel_timing() as timer:
            t2 = time.perf_counter()
            for i in range(args.steps):
                step(i, opt_events)
            torch.cuda.synchronize()
            breakdown_ms = 1000.0 * (time.perf_counter() - t2) / args.steps
    optimizer = None
    if opt_events:
        optimizer = {"ms_per_step": round(sum(a.elapsed_time(b) for a, b in opt_events)
                                          / len(opt_events), 4),
                     "impl": type(opt).__module__ + "." + type(opt).__name__,
                     "note": "Adam over all parameters (rb_adam_step, one launch; "
                             "RECBLR_ADAM=torch: torch.optim.Adam(fused=True)); inside every timed "
                             "step, timed on its own in the breakdown pass"}
    ms = 1000.0 * elapsed / args.steps
    value = env.world_size * args.batch * args.steps / elapsed
    if not torch.isfinite(loss):
        raise RuntimeError(f"non-finite loss {loss}")

    # The same step in the reference's shapes, for comparison (results identical,
    # tests/test_gpu_eval.py): the dense [B, L] batch with the gathered tail,
    # and the dense batch with the last layer's tail at every position (the
    # reference's arithmetic position for position).
    def timed_variant(packed, gather):
        model.pack_sequences, model.gather_last_layer = packed, gather
        for i in range(2):
            step(i)
        torch.cuda.synchronize()
        barrier(env)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        barrier(env)
        torch.cuda.synchronize()
        el = max_over_ranks(time.perf_counter() - t1, env, dev)
        model.pack_sequences, model.gather_last_layer = True, True
        return {"value": round(env.world_size * args.batch * args.steps / el, 1),
                "ms_per_step": round(1000.0 * el / args.steps, 3)}

    fixed = None
    if not args.no_full_tail:
        full_len = [synthetic_interaction(args.batch, args.seq_len, args.n_items, dev,
                                          seed=1000 * env.rank + 50 + i, fixed_len=True)
                    for i in range(4)]
        saved, batches[:] = list(batches), full_len
        fixed = timed_variant(True, True)
        batches[:] = saved
        fixed["note"] = (f"every sequence of full length {args.seq_len} (packed == dense "
                         "rows), the same step otherwise: a length-independent companion to "
                         "the headline, whose lengths are ~U{1..L}")
    devlen = None
    if not args.no_full_tail:
        # run.py's path: RecBole hands item_length as a bare device tensor
        # (RecBLR.py:86, run.py:84) — no host copy attached, so the packed
        # forward reads the token count from the device (one sync per step)
        saved = list(batches)
        batches[:] = [dict(b, item_length=b["item_length"].clone()) for b in saved]
        devlen = timed_variant(True, True)
        batches[:] = saved
        devlen["note"] = ("the headline's batches with item_length as a bare device tensor "
                          "(no host lengths attached); the packed forward syncs once per "
                          "step for the token count")
        # run.py's path: CPU batches moved by Interaction.to(device) every step
        # (the hook keeps the host lengths: no sync; pageable H2D copies of
        # the batch inside the timed step, as RecBole's Trainer does)
        batches[:] = [Interaction({k: v.cpu() for k, v in b.items()}) for b in saved]
        recbole_path = timed_variant(True, True)
        batches[:] = saved
        recbole_path["note"] = ("CPU batches moved by Interaction.to(device) inside every step, "
                                "as RecBole's Trainer (run.py) does; the hook on Interaction.to "
                                "keeps the host lengths (recbole_compat.install_interaction_hook)")
        devlen["recbole_interaction_path"] = recbole_path
    fused_ab = None
    if not args.no_full_tail:
        # the fused GatedRecurrentLayer kernels (experimental/grl_fused.hip, opt-in):
        # A/B against the headline's three-launch path on the same batches
        from datamining_recblr_amd import recurrence
        saved_f = (recurrence._FUSED, recurrence._FUSED_BWD)
        fused_ab = {}
        for name, f, fb in (("fused_fwd", True, False), ("fused_fwd_and_bwd", True, True),
                            ("unfused", False, False)):
            if (f, fb) == saved_f:
                continue
            recurrence._FUSED, recurrence._FUSED_BWD = f, fb
            fused_ab[name] = timed_variant(True, True)
        recurrence._FUSED, recurrence._FUSED_BWD = saved_f
        fused_ab["headline"] = {"fused_fwd": saved_f[0], "fused_bwd": saved_f[1]}
        fused_ab["note"] = ("RECBLR_FUSED_GRL / RECBLR_FUSED_GRL_BWD A/B on the headline's "
                            "batches: rb_grl_fwd (conv + gates GEMM + scan in one launch) "
                            "alone and with rb_grl_bwd, against the three-launch path")
    ffn_act_ab = None
    if not args.no_full_tail:
        # the FeedForward's activation in w_1's GEMM epilogue (rb_gemm_nt_h_act)
        # against the GEMM + rb_silu_dropout_fwd, alternated 3x on the lease
        from datamining_recblr_amd import linear as _lin
        saved_a = _lin.set_ffn_act_fused(True)
        runs = {"fused": [], "two_launches": []}
        for _ in range(3):
            for name, on in (("fused", True), ("two_launches", False)):
                _lin.set_ffn_act_fused(on)
                runs[name].append(timed_variant(True, True)["ms_per_step"])
        _lin.set_ffn_act_fused(saved_a)
        ffn_act_ab = {k: {"ms_per_step": min(v), "all": v} for k, v in runs.items()}
        ffn_act_ab["headline"] = "fused" if saved_a else "two_launches"
        ffn_act_ab["note"] = ("RECBLR_FFN_ACT A/B on the headline's batches: w_1 with "
                              "dropout(silu(.)) in its epilogue vs the GEMM and "
                              "rb_silu_dropout_fwd, best of 3 alternated runs each")
    nt_ab = None
    if not args.no_full_tail:
        # rb_gemm_nt_h's kernel for the encoder's projections: the weight-
        # stationary kernel (round 6, csrc/gemm_ws.hip) against round 5's
        # persistent tiles, alternated 3x on the lease
        from datamining_recblr_amd import linear as _lin
        saved_w = _lin.set_nt_ws(True)
        runs = {"weight_stationary": [], "persistent_tiles": []}
        for _ in range(3):
            for name, on in (("weight_stationary", True), ("persistent_tiles", False)):
                _lin.set_nt_ws(on)
                runs[name].append(timed_variant(True, True)["ms_per_step"])
        _lin.set_nt_ws(saved_w)
        nt_ab = {k: {"ms_per_step": min(v), "all": v} for k, v in runs.items()}
        nt_ab["headline"] = "weight_stationary" if saved_w else "persistent_tiles"
        nt_ab["note"] = ("RECBLR_NT_WS A/B on the headline's batches: the projections' forward "
                         "/ input-gradient GEMMs from 16,384 rows on the weight-stationary "
                         "kernel vs the persistent 256-row tiles; best of 3 alternated runs")
    order_ab = None
    if not args.no_full_tail:
        # the gate backward's consumers: the conv backward right behind the
        # dX GEMM that wrote its second input (default) vs the weight gradient
        # first (round 3), alternated 3x on the lease
        from datamining_recblr_amd import recurrence as _rec
        saved_o = _rec.set_conv_first(True)
        runs = {"conv_first": [], "wgrad_first": []}
        for _ in range(3):
            for name, on in (("conv_first", True), ("wgrad_first", False)):
                _rec.set_conv_first(on)
                runs[name].append(timed_variant(True, True)["ms_per_step"])
        _rec.set_conv_first(saved_o)
        order_ab = {k: {"ms_per_step": min(v), "all": v} for k, v in runs.items()}
        order_ab["headline"] = "conv_first" if saved_o else "wgrad_first"
        order_ab["note"] = ("RECBLR_CONV_FIRST A/B on the headline's batches: in the "
                            "GatedRecurrentLayer backward, the conv backward before the gates "
                            "weight gradient (its inputs just written) or after it; best of 3")
    adam_ab = None
    if not args.no_full_tail:
        # the optimizer update: rb_adam_step (one launch over every parameter)
        # against torch's fused Adam, alternated 3x on the lease (each with its
        # own state; the step's other work is the same)
        saved_opt = opt
        arms = {adam_kind: saved_opt,
                ("torch" if adam_kind == "native" else "native"):
                    make_opt("torch" if adam_kind == "native" else "native")}
        runs = {k: [] for k in arms}
        for _ in range(3):
            for name, o in arms.items():
                opt = o
                runs[name].append(timed_variant(True, True)["ms_per_step"])
        opt = saved_opt
        adam_ab = {k: {"ms_per_step": min(v), "all": v} for k, v in runs.items()}
        adam_ab["headline"] = adam_kind
        adam_ab["note"] = ("RECBLR_ADAM A/B on the headline's batches: rb_adam_step (native, one "
                           "launch) vs torch.optim.Adam(fused=True), best of 3 alternated runs")
    dense = full_tail = None
    if not args.no_full_tail:
        dense = timed_variant(False, True)
        dense["note"] = ("dense [B, L] batch (right padding computed, RECBLR_PACKED=0), "
                         "last layer's tail at the gathered positions")
        full_tail = timed_variant(False, False)
        full_tail["note"] = ("dense [B, L] batch and the last layer's out-proj/LN/FFN at all "
                             "B*L positions: the reference's arithmetic")

    roofline = None
    kernels_report = None
    gemm = None
    if timer is not None:
        summ = timer.summary()
        g = summ.pop("gemm", None)
        if g is not None:
            tf = g["bytes"] / (g["ms"] * 1e-3) / 1e12
            from datamining_recblr_amd.linear import gemm_format
            fmt = gemm_format()
            peak = F16X3_PEAK_TFS if fmt == "f16x3" else FP32_MFMA_PEAK_TFS
            by_shape = timer.gemm_detail(args.steps)
            gb = gemm_bytes(by_shape)
            gms = g["ms"] / args.steps
            gemm = {"bound": "hbm", "dtype": "f32 (" + fmt + " split operands)" if fmt != "torch"
                    else "f32",
                    "achieved": round(tf, 1), "peak": round(peak, 1), "unit": "TFLOP/s",
                    "frac": round(tf / peak, 4),
                    "hbm": {"algo_bytes_per_step": int(gb),
                            "achieved_gbs": round(gb / (gms * 1e-3) / 1e9, 1),
                            "frac": round(gb / (gms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                            "note": "fp32 A read + fp32 output write per GEMM (dY, X reads "
                                    "for weight gradients): these tall-skinny GEMMs are "
                                    "bound by their row streams at f16x3"},
                    "ms_per_step": round(gms, 3),
                    "gemms_per_step": g["launches"] / args.steps,
                    "flops_per_step": int(g["bytes"] / args.steps),
                    "library": {"f16x3": "f16 two-part split MFMA kernels (csrc/gemm_half.hip): "
                                         "rb_gemm_nt_h forward/input-gradient, rb_gemm_tn_h "
                                         "weight gradients",
                                "torch": "hipBLASLt/rocBLAS via torch"}[fmt],
                    "tuned_table": tuned_gemms_active(),
                    "mfma_busy": pmc_mfma(args),
                    "by_shape": by_shape,
                    "breakdown_pass_ms_per_step": round(breakdown_ms, 3)}
        ntok_step = sum(int(batches[i % len(batches)]["item_length"].sum())
                        for i in range(args.steps)) / args.steps
        kernels_report = kernel_report(summ, args.steps, ntok_step, 2 * args.hidden, args.layers)
        dsumm = dom_timer.summary() if dom_timer is not None else {}
        if DOMINANT in dsumm:
            d = dsumm[DOMINANT]
            ach = d["avg_bytes"] / (d["avg_ms"] * 1e-3) / 1e9
            traffic, src = pmc_traffic(args, "k_gate_scan_bwd")
            roofline = {"kernel": DOMINANT, "bound": "hbm", "achieved": round(ach, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": src,
                        "algo_bytes_per_launch": int(d["avg_bytes"]),
                        "avg_launch_us": round(d["avg_ms"] * 1e3, 2),
                        "timed": "HIP events on the launch stream, inside the timed region"}
    if roofline is not None and env.rank == 0 and args.hidden * 2 % 4 == 0:
        roofline["pattern"] = gate_bwd_pattern(args, batches[0], dev)
    if gemm is not None and env.rank == 0 and fmt == "f16x3":
        gemm["pattern"] = gemm_pattern(args, batches[0], dev)
    ddp_ab = None
    if env.world_size == 1 and not args.no_ddp_ab:
        ddp_ab = ddp_overhead(args, model, batches, dev)
    scan = scan_microbench(args, dev) if env.rank == 0 else None
    c5 = None if args.no_c5 else long_seq_c5(args, env, dev)   # every rank (weak scaling)
    cpu = None
    if env.rank == 0 and env.world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, model.state_dict())

    from datamining_recblr_amd.linear import gemm_format
    gemm_format_name = gemm_format()
    if env.rank == 0:
        H = 2 * args.hidden
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sequences/sec",
            "n_gpus": env.world_size, "steps": args.steps, "warmup": args.warmup,
            "settle": {"seconds": args.settle_seconds, "steps": settle_steps},
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("f32 I/O, f16x3 split GEMM products" if gemm_format_name == "f16x3"
                      else "f32"),
            "lengths": {"headline": "packed, lengths ~U{1..L} (SURVEY §8(d))",
                        "fixed_length_value": fixed["value"] if fixed else None,
                        "fixed_length_ms_per_step": fixed["ms_per_step"] if fixed else None,
                        "device_lengths_ms_per_step": (devlen or {}).get("ms_per_step")},
            "data": "synthetic RecBole-shaped batches (ids ~U{1..n_items-1}, lengths ~U{1..L}, "
                    "right-padded), reference init (seed 2020), resident in HBM",
            "config": {"workload": "RecBLR train step: calculate_loss(CE)+backward+Adam",
                       "sequences": "packed: each sequence's first item_seq_len positions "
                                    "(right padding, which never reaches the output, dropped)",
                       "last_layer_tail": "gathered positions (gather_indexes rows only)",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * env.world_size,
                       "seq_len": args.seq_len, "hidden_size": args.hidden, "inner_H": H,
                       "num_layers": args.layers, "n_items": args.n_items,
                       "dropout": args.dropout, "parallelism": f"dp{env.world_size}"},
            "host_enqueue_ms_per_step": round(host_enqueue_ms, 3),
            "multi_gpu": multi,
            "roofline": roofline,
            "gemm": gemm,
            "optimizer": optimizer,
            "kernels": kernels_report,
            "fixed_length": fixed,
            "device_lengths": devlen,
            "fused_grl": fused_ab,
            "ffn_act": ffn_act_ab,
            "adam": adam_ab,
            "bwd_order": order_ab,
            "nt_kernel": nt_ab,
            "ddp_overhead": ddp_ab,
            "dense_batch": dense,
            "all_positions_tail": full_tail,
            "scan_fwd_only": scan,
            "long_seq_bf16": c5,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        barrier(env)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
