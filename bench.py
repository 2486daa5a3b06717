#!/usr/bin/env python3
"""Benchmark of the PF hot path (one "step" = one PF frame: propagate + weight + resample) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

N = 1 runs BASELINE.json configs[1] (C2: 5 LEDs, 100k particles, 50 blobs/frame, fp32 state).  For N > 1
the driver launches one process per GPU with torch.distributed.run; every rank runs an INDEPENDENT camera
stream (its own seed) on its own GPU — the path shards across streams with no data-path collective
(SURVEY.md §8e), so scaling is "weak".  gloo (CPU) carries only the barrier and the max-over-ranks time.

Inputs are resident in HBM before the timed region (pfmpe_stage_blob_bank); each step calls pfmpe_step,
which is blocking (its last act is the stream synchronize that brings the winner to the host), so the
timed region is bracketed by barrier + device sync on both sides.

Extra objects on the JSON line:
  roofline     — dominant kernel's algorithmic bytes per launch / its HIP-event-timed average duration
  cpu_baseline — the oracle (single-thread restatement of the reference loop, O(N^2) resample) timed on
                 this host on a bounded sample of the same workload (rank 0, N = 1 only)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=["C1", "C2", "C3", "C4"])
    ap.add_argument("--particles", type=int, default=0, help="override N")
    ap.add_argument("--force-iters", type=int, default=0)
    ap.add_argument("--rng", default="philox", choices=["philox", "reference"])
    ap.add_argument("--state", default="", choices=["", "f32", "f16", "f64"],
                    help="particle state storage (default: f16 for C4 per BASELINE.json configs[3], else f32)")
    ap.add_argument("--cpu-frames", type=int, default=3, help="oracle frames for cpu_baseline (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="do not bracket kernels with HIP events")
    ap.add_argument("--timing-period", type=int, default=25,
                    help="HIP events bracket the kernels of every P-th timed frame (they serialise the stream)")
    ap.add_argument("--diag", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--prune", type=int, default=1, choices=[0, 1], help="exact blob pruning (1) or brute force (0)")
    ap.add_argument("--pmc", default="", help="PMC summary json (scripts/pmc_summary.py --json) of this same "
                    "workload; default profiles/pmc_<config>_n<N>.json when present")
    ap.add_argument("--keep-prop", type=int, default=1, choices=[0, 1],
                    help="two-launch path: store the propagated set (1) or regenerate it in k_resample (0)")
    ap.add_argument("--python-loop", action="store_true", help="one FFI call per frame instead of pfmpe_step_batch")
    ap.add_argument("--fused", type=int, default=2, choices=[0, 1, 2],
                    help="frame shape: 2 flat one-launch (default), 1 tree one-launch, 0 two launches")
    return ap.parse_args()


def algorithmic_bytes(S: int, N: int) -> dict:
    """Compulsory HBM bytes per launch (DESIGN.md "Roofline")."""
    return {
        "k_propagate_weigh": N * (S + 4),      # read prior state, write weight
        "k_resample": N * (4 + S + S),          # read weight, read prior (regenerate), write new prior
        "k_frame": N * (S + 4 + S),             # one launch: read prior, write weight, write new prior
        "k_frame2": N * (S + 4 + S),
        "k_resample_final": 8 * -(-N // 256),   # read the block count partials
        "aux": 0,
    }


def pmc_traffic(path: str, kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC pass of the same workload (or None)."""
    if not path or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            rows = json.load(f)
        # PFMPE_K_FRAME times both one-launch shapes; the PMC pass names the kernel itself (k_frame2 by default)
        row = rows.get(kernel) or (rows.get("k_frame2") if kernel == "k_frame" else None) or {}
        return row.get("hbm_bytes")
    except (OSError, ValueError):
        return None


def combine_ranks(dist, elapsed: float, updates: float):
    """Whole-job figures: the slowest rank's time (max) and all ranks' particle-updates (sum), over gloo.
    No data-path collective exists: streams are independent, only these two scalars cross ranks."""
    if dist is None:
        return float(elapsed), float(updates)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    u = torch.tensor([updates], dtype=torch.float64)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def cpu_baseline(cfg, n_frames: int):
    from oracle import pforacle as orc
    from pf_monocular_pose_estimator_amd import synthetic as syn
    st = syn.make_stream(cfg, n_frames)
    prior = st.prior()
    times, iters = [], []
    for fr in st.frames:
        t0 = time.perf_counter()
        out, arr = orc.pf_step(st.markers, st.K, orc.make_params(), prior, fr.current_pose, fr.predicted_pose,
                               fr.prediction, fr.blobs, dt=fr.dt, seed=11 + fr.index, frame_idx=fr.index)
        times.append(time.perf_counter() - t0)
        iters.append(out["iters"])
        if out["resampled"]:
            prior = arr["resampled"]
    tm = statistics.median(times)
    k = statistics.median(iters)
    return {
        "value": cfg.N * k / tm, "unit": "particle-updates/s", "cores": 1, "kind": "port",
        "sample": f"{n_frames} frames of {cfg.name} (N={cfg.N}, M={cfg.M}, B={cfg.B}); oracle/pf_oracle.cpp "
                  f"fp64, median {tm:.3f} s/frame, k={k}; single thread like the reference's ros::spin",
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo on CPU: barrier + max only
        dist.init_process_group("gloo")

    import pf_monocular_pose_estimator_amd as pf
    from pf_monocular_pose_estimator_amd import synthetic as syn

    base = syn.CONFIGS[args.config]
    cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=args.particles or base.N, heavy=base.heavy, seed=rank)
    n_frames = args.warmup + args.steps
    st = syn.make_stream(cfg, n_frames)
    state = args.state or ("f16" if cfg.name == "C4" else "f32")
    state_dtype = {"f32": pf.STATE_F32, "f16": pf.STATE_F16, "f64": pf.STATE_F64}[state]
    # one GPU per rank; PFMPE_BENCH_DEVICE pins every rank to one device (rehearsing the multi-rank launch
    # on a one-GPU box: the ranks then share the card, so the figure is plumbing, not scaling)
    device = int(os.environ.get("PFMPE_BENCH_DEVICE", local_rank))
    eng = pf.Engine(device=device, max_particles=cfg.N, state_dtype=state_dtype)
    eng.set_model(st.markers, st.K)
    prm = pf.default_params()
    prm.rng_mode = pf.RNG_PHILOX if args.rng == "philox" else pf.RNG_REFERENCE
    eng.set_params(prm)
    eng.set_prior(st.prior())
    eng.set_option(pf.OPT_FUSED, args.fused)
    eng.set_option(pf.OPT_PRUNE, args.prune)
    eng.set_option(pf.OPT_KEEP_PROPAGATED, args.keep_prop)
    if args.diag:
        eng.set_option(99, args.diag)
    eng.stage_blob_bank([f.blobs for f in st.frames])
    frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                             dt=f.dt, seed=(rank << 32) + 17 + f.index, frame_idx=f.index,
                             force_iters=args.force_iters) for f in st.frames]

    for i in range(args.warmup):
        eng.step(frames[i])
    eng.reset_kernel_stats()
    if not args.no_timing:
        eng.set_option(pf.OPT_TIMING, args.timing_period)

    if dist:
        dist.barrier()
    timed = frames[args.warmup:n_frames]
    t0 = time.perf_counter()
    if args.python_loop:
        outs = [eng.step(f) for f in timed]  # one FFI call per frame
    else:
        outs = eng.step_batch(timed)  # the C loop a C++ tracker runs; every frame still blocks on its record
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    updates = sum(cfg.N * o.iters for o in outs)
    iters = [o.iters for o in outs]
    accepted = sum(o.accepted for o in outs)
    stats = eng.kernel_stats()
    eng.set_option(pf.OPT_TIMING, 0)

    elapsed, total_updates = combine_ranks(dist, elapsed, updates)

    if rank == 0:
        S = {"f32": 48, "f16": 24, "f64": 96}[state]  # SoA state bytes per particle
        ab = algorithmic_bytes(S, cfg.N)
        roof = None
        timed = {k: v for k, v in stats.items() if v[0] > 0}
        if timed:
            dom = max(timed, key=lambda k: timed[k][1])
            launches, ms = timed[dom]
            avg_s = ms / 1e3 / launches
            achieved = ab.get(dom, 0) / avg_s / 1e9 if avg_s > 0 else 0.0
            pmc = args.pmc or os.path.join(ROOT, "profiles", f"pmc_{cfg.name.lower()}_n{cfg.N}.json")
            traffic = pmc_traffic(pmc, dom)
            roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    "traffic": None if traffic is None else round(traffic),
                    "bytes_per_launch": ab.get(dom, 0), "avg_us": round(avg_s * 1e6, 3),
                    "per_kernel_avg_us": {k: round(v[1] * 1e3 / v[0], 3) for k, v in timed.items()}}
        cpu = None
        if world == 1 and args.cpu_frames > 0:
            cpu = cpu_baseline(cfg, args.cpu_frames)
        k_mean = float(np.mean(iters)) if iters else 0.0
        line = {
            "metric": "particle-updates/sec (propagate+weight+resample) per GPU; frames/sec at N_particles",
            "value": total_updates / elapsed,
            "unit": "particle-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if state != "f64" else "f64",
            "data": "synthetic",
            "config": {
                "workload": f"{cfg.name}: {cfg.M} LEDs, {cfg.N} particles, {cfg.B} blobs/frame"
                            f"{' (heavy outliers)' if cfg.heavy else ''}, {state} SoA state"
                            + (" (BASELINE.json configs[1])" if cfg.name == "C2" else ""),
                "state": state,
                "N_particles": cfg.N, "markers": cfg.M, "blobs": cfg.B,
                "frames_per_sec_per_gpu": args.steps / elapsed,
                "iters_per_frame": k_mean, "accept_rate": accepted / max(1, args.steps),
                "rng": args.rng, "parallelism": f"{world} independent camera streams (1 per GPU), no collectives",
            },
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
