#!/usr/bin/env python3
"""Benchmark of the PF hot path (one "step" = one PF frame: propagate + weight + resample) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]

N = 1 runs BASELINE.json configs[1] (C2: 5 LEDs, 100k particles, 50 blobs/frame, fp32 state).  For N > 1
the driver launches one process per GPU with torch.distributed.run and every rank runs configs[4] (C5): an
INDEPENDENT 1M-particle camera stream (its own seed) on its own GPU — the path shards across streams with no
data-path collective, so scaling is "weak".  gloo (CPU) carries only the barrier, the
max-over-ranks time and the sum of updates.

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
    ap.add_argument("--config", default="", choices=["", "C1", "C2", "C3", "C4", "C5"],
                    help="default: C2 (BASELINE.json configs[1]) at --gpus 1, C5 (configs[4]: one 1M-particle "
                         "stream per GPU) at --gpus > 1")
    ap.add_argument("--particles", type=int, default=0, help="override N")
    ap.add_argument("--force-iters", type=int, default=0)
    ap.add_argument("--rng", default="philox", choices=["philox", "reference"])
    ap.add_argument("--state", default="", choices=["", "f32", "f16", "f64"],
                    help="particle state storage (default: f16 for C4 per BASELINE.json configs[3], else f32)")
    ap.add_argument("--cpu-frames", type=int, default=3, help="oracle frames for cpu_baseline (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="no kernel pass (no HIP-event brackets at all)")
    ap.add_argument("--kernel-frames", type=int, default=0,
                    help="frames of the kernel pass after the timed region, every one HIP-event bracketed "
                         "(0 = max(20, steps))")
    ap.add_argument("--timing-period", type=int, default=0,
                    help="HIP events bracket the kernels of every P-th timed frame; default: two frames up to 40 "
                         "timed frames, four beyond (a bracketed C2 frame costs ~12 us more, DESIGN.md §7)")
    ap.add_argument("--occlude", type=int, default=0, choices=[0, 1],
                    help="time worst-case frames only: one LED hidden, so the reference's re-draw loop runs all "
                         "80 iterations (pose_estimator.cpp:535-616)")
    ap.add_argument("--worst-frames", type=int, default=10,
                    help="after the timed region, also time this many worst-case (one LED hidden) frames")
    ap.add_argument("--c1-frames", type=int, default=200, help="C1 oracle frames for the configs[0] CPU baseline")
    ap.add_argument("--stream-id", type=int, default=-1,
                    help="camera stream to run (seeds); default = this rank, so rank r runs stream r")
    ap.add_argument("--dump-records", default="", help=argparse.SUPPRESS)  # tests: per-rank records -> PATH.<rank>.json
    ap.add_argument("--diag", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--prune", type=int, default=1, choices=[0, 1], help="exact blob pruning (1) or brute force (0)")
    ap.add_argument("--pmc", default="", help="PMC summary json (scripts/pmc_summary.py --json) of this same "
                    "workload; default profiles/pmc_<config>_n<N>.json when present")
    ap.add_argument("--keep-prop", type=int, default=-1, choices=[-1, 0, 1],
                    help="two-launch path: store the propagated set (1) or regenerate it in k_resample (0); "
                         "-1 = the library's default for the state type")
    ap.add_argument("--python-loop", action="store_true", help="one FFI call per frame instead of pfmpe_step_batch")
    ap.add_argument("--multi-sweep", default="",
                    help="after the timed region, also run S independent streams of the config per GPU as one "
                         "batch (pfmpe_step_multi) for each S in this comma list; default 1,4,8,16,32 at C2 on one "
                         "GPU; 'none' skips the sweep")
    ap.add_argument("--multi-steps", type=int, default=50, help="timed batches per multi-stream point")
    ap.add_argument("--multi-groups", default="1,2",
                    help="batches per multi-stream point, each on its own host thread and HIP stream (comma list)")
    ap.add_argument("--exact-steps", type=int, default=100,
                    help="frames of the fp64 / reference-RNG (parity mode) C2 point beside the default line (0 = skip)")
    ap.add_argument("--scale-ref-steps", type=int, default=100,
                    help="frames of the one-GPU C5 reference beside the default C2 line (0 = skip)")
    ap.add_argument("--single-points", default="C3,C4",
                    help="configs timed as one stream beside the default C2 line, with their per-kernel HIP-event "
                         "averages (comma list; 'none' skips)")
    ap.add_argument("--single-steps", type=int, default=100, help="timed frames per --single-points config")
    ap.add_argument("--fused", type=int, default=2, choices=[0, 1, 2],
                    help="frame shape: 2 flat one-launch (default), 1 tree one-launch, 0 two launches")
    return ap.parse_args()


def info_or(pf, eng, key, default=-1):
    """pfmpe_get_info, or `default` for a key an older library (an A/B build) does not know."""
    try:
        return eng.info(key)
    except pf.PFError:
        return default


def kernel_pass(pf, eng, frames):
    """Per-kernel average durations over `frames`, every frame's kernels HIP-event bracketed (hipExtLaunchKernel
    dispatch timestamps, the same ones rocprofv3's kernel trace reads).  Run right after a timed region on the same
    stream, so the timed frames carry no bracket (a bracketed frame costs the host ~12 us at C2) and
    the averages cover every frame of the pass instead of a sample.  scripts/trace_check.py
    takes the same launches out of a rocprofv3 trace of the same command."""
    eng.reset_kernel_stats()
    eng.set_option(pf.OPT_TIMING, 1)  # every frame
    outs = eng.run_batch(eng.prepare_batch(frames))
    eng.set_option(pf.OPT_TIMING, 0)
    return eng.kernel_stats(), outs


def algorithmic_bytes(S: int, N: int, k: float = 1.0) -> dict:
    """Algorithmic HBM bytes per launch, SURVEY.md §8(d)'s canonical figure: 3*S + 8 bytes per particle-update
    for a k = 1 frame = read prior S + write weight 4 (propagate pass) + read weight 4 + gather-read the kept
    particle S + write the new prior S (resample pass); every further iteration adds S + 4."""
    return {
        "k_propagate_weigh": N * (S + 4),            # one weighing pass: read prior, write weight
        "k_resample": N * (4 + S + S),               # read weight, gather-read kept particle, write new prior
        "k_frame": int(N * (k * (S + 4) + 4 + 2 * S)),   # the whole frame in one launch
        "k_frame2": int(N * (k * (S + 4) + 4 + 2 * S)),
        "k_resample_final": 8 * -(-N // 256),        # read the block count partials
        "aux": 0,
    }


def host_cpu():
    """CPU model and logical CPU count of this host (the GPU box's host when run there)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


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


def counter_bytes_per_update(path: str, N: int):
    """HBM bytes per particle-update by counters: the frame's kernels' PMC bytes per launch (the committed one-stream
    pass of the config, profiles/pmc_<cfg>_n<N>.json) over N.  The deferred design does not move the canonical 3S+8
    bytes, so a batch point's canonical frac is not its DRAM occupancy."""
    if not path or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    frame = [k for k in rows if k.startswith("k_") and k not in ("k_import", "k_export", "k_regen", "k_weights_export")]
    tot = sum(rows[k].get("hbm_bytes") or 0 for k in frame)
    return tot / N if tot else None


# The issue roofline (SURVEY.md §8d "report both fractions"): the kernels of this path have no MFMA work and at the
# sizes that fit the MALL they are bound by instruction issue, not bytes.  From the committed PMC pass of the same
# workload (scripts/pmc_lines.sh): VALU issue = SQ_INSTS_VALU (wave instructions) x the measured cost of one wave
# instruction on its SIMD at >= 4 waves per SIMD, ~4 cycles for this mix (fp64, packed fp32, v_mad_u64_u32, DPP;
# profiles/r04/isa_rates.txt), over 1,024 SIMDs at 2.4 GHz; SALU issue = SQ_INSTS_SALU over the
# CU's one scalar unit (256 CUs, one instruction per cycle).  frac = issue time / the kernel's measured time.
CLOCK_HZ = 2.4e9
SIMDS, CUS = 1024, 256
VALU_CYCLES = 4.0


def issue_roof(path: str, kernel: str, avg_us: float):
    if not path or not os.path.exists(path) or not avg_us:
        return None
    try:
        with open(path) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    alias = {"k_frame": "k_frame2"}
    row = rows.get(kernel) or rows.get(alias.get(kernel, ""), None)
    if not row or "SQ_INSTS_VALU" not in row or "SQ_INSTS_SALU" not in row:
        return None
    t = avg_us * 1e-6
    valu_s = row["SQ_INSTS_VALU"] * VALU_CYCLES / (SIMDS * CLOCK_HZ)
    salu_s = row["SQ_INSTS_SALU"] / (CUS * CLOCK_HZ)
    waves = row.get("SQ_WAVES") or 0
    return {"bound": "issue", "kernel": kernel, "valu_frac": round(valu_s / t, 4), "salu_frac": round(salu_s / t, 4),
            "issue_frac": round(max(valu_s, salu_s) / t, 4),
            "valu_per_wave": round(row["SQ_INSTS_VALU"] / waves, 1) if waves else None,
            "salu_per_wave": round(row["SQ_INSTS_SALU"] / waves, 1) if waves else None,
            "valu_cycles": VALU_CYCLES, "clock_ghz": CLOCK_HZ / 1e9, "pmc_source": os.path.relpath(path, ROOT)}


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


def oracle_frames(cfg, n_frames: int, warm: int = 0):
    """The oracle (single-thread C++ restatement of PE:475-733, the reference's own loop structure with its
    O(N^2) resampler) over a synthetic stream; per-frame wall time around the PF block only."""
    from oracle import pforacle as orc
    from pf_monocular_pose_estimator_amd import synthetic as syn
    st = syn.make_stream(cfg, warm + n_frames)
    prior = st.prior()
    times, iters = [], []
    for fr in st.frames:
        t0 = time.perf_counter()
        out, arr = orc.pf_step(st.markers, st.K, orc.make_params(), prior, fr.current_pose, fr.predicted_pose,
                               fr.prediction, fr.blobs, dt=fr.dt, seed=11 + fr.index, frame_idx=fr.index)
        if fr.index >= warm:
            times.append(time.perf_counter() - t0)
            iters.append(out["iters"])
        if out["resampled"]:
            prior = arr["resampled"]
    return statistics.median(times), statistics.median(iters)


def _c1_stream_rate(seed: int, n_frames: int):
    """One process's C1 stream (seeded): (frames, updates, seconds) of the oracle PF block only."""
    from oracle import pforacle as orc
    from pf_monocular_pose_estimator_amd import synthetic as syn
    c1 = syn.CONFIGS["C1"]
    cfg = syn.StreamConfig(c1.name, M=c1.M, B=c1.B, N=c1.N, seed=seed)
    st = syn.make_stream(cfg, n_frames + 5)
    prior = st.prior()
    tot, upd = 0.0, 0
    for fr in st.frames:
        t0 = time.perf_counter()
        out, arr = orc.pf_step(st.markers, st.K, orc.make_params(), prior, fr.current_pose, fr.predicted_pose,
                               fr.prediction, fr.blobs, dt=fr.dt, seed=11 + fr.index, frame_idx=fr.index)
        if fr.index >= 5:
            tot += time.perf_counter() - t0
            upd += cfg.N * out["iters"]
        if out["resampled"]:
            prior = arr["resampled"]
    return n_frames, upd, tot


def cpu_multiprocess(procs: int, n_frames: int):
    """SURVEY.md §8(d)'s multi-core CPU comparison: one process per core on independent C1 streams, aggregate
    updates/s = sum over processes of (updates / own PF-block time)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    # close + join, not the context manager's terminate(): a SIGTERM'd worker prints an "Aborted" dump into
    # every profiler log
    pool = ctx.Pool(procs)
    try:
        res = pool.starmap(_c1_stream_rate, [(100 + i, n_frames) for i in range(procs)])
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    return {"procs": procs, "value": sum(u / t for _, u, t in res), "unit": "particle-updates/s",
            "sample": f"C1 x {procs} independent streams, {n_frames} frames each after 5 warm-up, one process each"}


def cpu_baseline(cfg, n_frames: int, c1_frames: int):
    from pf_monocular_pose_estimator_amd import synthetic as syn
    model, ncpu = host_cpu()
    tm, k = oracle_frames(cfg, n_frames)
    res = {
        "value": cfg.N * k / tm, "unit": "particle-updates/s", "cores": 1, "kind": "port",
        "sample": f"{n_frames} frames of {cfg.name} (N={cfg.N}, M={cfg.M}, B={cfg.B}); oracle/pf_oracle.cpp "
                  f"fp64, median {tm:.3f} s/frame, k={k}; single thread like the reference's ros::spin",
        "cpu_model": model, "nproc": ncpu,
    }
    if c1_frames > 0:  # BASELINE.json configs[0]: the reference's own CPU-runnable case
        c1 = syn.CONFIGS["C1"]
        t1, k1 = oracle_frames(c1, c1_frames, warm=20)
        res["c1"] = {"value": c1.N * k1 / t1, "unit": "particle-updates/s", "frames_per_sec": 1.0 / t1,
                     "ms_per_frame": t1 * 1e3, "iters_per_frame": k1,
                     "sample": f"C1 (N={c1.N}, M={c1.M}, B={c1.B}): median of {c1_frames} frames after 20 warm-up, "
                               f"1 thread"}
        res["c1_multiprocess"] = cpu_multiprocess(min(8, ncpu or 1), 50)
    return res


def occluded_frames(eng, st, rank: int, n: int, first_index: int):
    """Worst-case frames: one LED hidden (its blob dropped, an outlier added so B is unchanged), so the
    maximum weight never reaches M*min(5,B) and the re-draw loop runs all 80 iterations (PE:535-616)."""
    from pf_monocular_pose_estimator_amd import synthetic as syn
    frames = []
    for j in range(n):
        fr = st.frames[j % len(st.frames)]
        rng = np.random.default_rng(50_000 + j)
        true_px = syn.project(st.K, fr.truth, st.markers)
        near = np.abs(fr.blobs[:, None, :] - true_px[None, 0:1, :]).sum(-1).min(1)
        keep = fr.blobs[np.argsort(near)[1:]]  # drop the blob closest to LED 0
        blobs = np.vstack([keep, rng.uniform([0, 0], [syn.IMAGE_W, syn.IMAGE_H], size=(1, 2))])
        frames.append(eng.make_frame(fr.current_pose, fr.predicted_pose, fr.prediction, blobs=blobs, dt=fr.dt,
                                     seed=(rank << 32) + 90_000 + j, frame_idx=first_index + j))
    return frames


def multi_stream_point(pf, syn, base, S: int, steps: int, warmup: int, state_dtype: int, rng: int, device: int,
                       sid0: int, prune: int, keep_prop: int, groups: int = 1, diag: int = 0):
    """S independent streams of `base` on one GPU, each frame of all S run as ONE batch (pfmpe_step_multi:
    one weighing launch over every stream's blocks, one resampling launch, one finishing launch).  Blob tables
    come from each stream's staged bank; the timed loop is pfmpe_step_multi_batch (the C loop a tracker runs).
    groups > 1: the streams split into that many batches, each driven by its own host thread on its own HIP
    stream (ctypes releases the GIL in the C loop), so one batch's host turnaround (record wait, descriptor
    staging, launch) overlaps the other batches' kernels."""
    import ctypes as C
    engs, frames = [], []
    n = warmup + steps
    try:
        for s in range(S):
            cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=base.N, heavy=base.heavy, seed=1000 * sid0 + s)
            st = syn.make_stream(cfg, n)
            eng = pf.Engine(device=device, max_particles=cfg.N, state_dtype=state_dtype)
            eng.set_model(st.markers, st.K)
            prm = pf.default_params()
            prm.rng_mode = rng
            eng.set_params(prm)
            eng.set_prior(st.prior())
            eng.set_option(pf.OPT_PRUNE, prune)
            if keep_prop >= 0:
                eng.set_option(pf.OPT_KEEP_PROPAGATED, keep_prop)
            if diag:
                eng.set_option(99, diag)
            eng.stage_blob_bank([f.blobs for f in st.frames])
            engs.append(eng)
            frames.append([eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs),
                                          bank_frame=f.index, dt=f.dt, seed=((1000 * sid0 + s) << 32) + 17 + f.index,
                                          frame_idx=f.index) for f in st.frames])
        import threading
        lib = engs[0].lib
        fin, fout = C.sizeof(pf.FrameIn), C.sizeof(pf.FrameOut)
        G = max(1, min(groups, S))
        parts = [list(range(S))[g::G] for g in range(G)]
        runs = []
        for part in parts:
            Sg = len(part)
            ctxs = (C.c_void_p * Sg)(*[engs[s].ctx.value for s in part])
            ins = (pf.FrameIn * (Sg * n))(*[frames[s][f] for f in range(n) for s in part])  # batch-major
            outs = (pf.FrameOut * (Sg * n))()
            runs.append((Sg, ctxs, ins, outs, engs[part[0]]))

        def drive(r, first, count, errs):
            Sg, ctxs, ins, outs, e0 = r
            done = C.c_int()
            pin = C.cast(C.byref(ins, first * Sg * fin), C.POINTER(pf.FrameIn))
            pout = C.cast(C.byref(outs, first * Sg * fout), C.POINTER(pf.FrameOut))
            rc = lib.pfmpe_step_multi_batch(ctxs, Sg, pin, count, pout, C.byref(done))
            if rc != 0:
                errs.append(e0.ctx)
                e0._chk(rc)

        def run_all(first, count):
            errs = []
            if G == 1:
                drive(runs[0], first, count, errs)
                return
            th = [threading.Thread(target=drive, args=(r, first, count, errs)) for r in runs]
            for t in th:
                t.start()
            for t in th:
                t.join()
            if errs:
                raise RuntimeError("pfmpe_step_multi_batch failed in a batch thread")

        run_all(0, warmup)
        t0 = time.perf_counter()  # the C loop a multi-object tracker runs: every batch blocks on its records
        run_all(warmup, steps)
        el = time.perf_counter() - t0
        upd = sum(base.N * r[3][i].iters for r in runs for i in range(warmup * r[0], n * r[0]))
        acc = sum(r[3][i].accepted for r in runs for i in range(warmup * r[0], n * r[0]))
        return {"streams": S, "groups": G, "N_per_stream": base.N, "live_particles": S * base.N,
                "updates_per_s": upd / el, "ms_per_batch": el * 1e3 / steps,
                "frames_per_sec_per_stream": steps / el, "accept_rate": acc / (S * steps)}
    finally:
        for e in engs:
            e.close()


def single_stream_point(pf, syn, base, steps: int, warmup: int, rng: int, device: int, sid: int, args,
                        state_dtype=None, kernels=False):
    """One stream of `base` (f32 state unless given) on one GPU, timed as the main line is (pfmpe_step_batch:
    every frame blocks on its record).  kernels: then a kernel pass of `kframes` more frames, every one HIP-event
    bracketed (kernel_pass, as the main line), and their per-kernel averages, the frame shape and the weighing
    pass."""
    cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=base.N, heavy=base.heavy, seed=sid)
    kframes = max(20, steps) if kernels else 0
    st = syn.make_stream(cfg, warmup + steps + kframes)
    eng = pf.Engine(device=device, max_particles=cfg.N,
                    state_dtype=pf.STATE_F32 if state_dtype is None else state_dtype)
    try:
        eng.set_model(st.markers, st.K)
        prm = pf.default_params()
        prm.rng_mode = rng
        eng.set_params(prm)
        eng.set_prior(st.prior())
        eng.set_option(pf.OPT_FUSED, args.fused)
        eng.set_option(pf.OPT_PRUNE, args.prune)
        if args.keep_prop >= 0:
            eng.set_option(pf.OPT_KEEP_PROPAGATED, args.keep_prop)
        eng.stage_blob_bank([f.blobs for f in st.frames])
        frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                                 dt=f.dt, seed=(sid << 32) + 17 + f.index, frame_idx=f.index) for f in st.frames]
        for f in frames[:warmup]:
            eng.step(f)
        prepared = eng.prepare_batch(frames[warmup:warmup + steps])
        t0 = time.perf_counter()
        outs = eng.run_batch(prepared)
        el = time.perf_counter() - t0
        pt = {"value": sum(cfg.N * o.iters for o in outs) / el, "unit": "particle-updates/s",
              "ms_per_frame": el * 1e3 / steps, "frames": steps,
              "iters_per_frame": float(np.mean([o.iters for o in outs]))}
        if kernels:
            stats, _ = kernel_pass(pf, eng, frames[warmup + steps:])
            pt["kernel_pass_frames"] = kframes
            pt["frame_shape"] = {0: "two-launch", 1: "k_frame", 2: "k_frame2"}.get(eng.info(pf.INFO_LAST_SHAPE))
            wname = {pf.WEIGH_STREAM: "k_weigh_stream", pf.WEIGH_PK: "k_weigh_pk"}.get(
                eng.info(pf.INFO_LAST_WEIGH_PASS), "k_propagate_weigh")
            pt["weigh_pass"] = wname
            rname = "k_resample_owners" if info_or(pf, eng, pf.INFO_LAST_RESAMPLE) == pf.RESAMPLE_OWNERS else "k_resample"
            pt["per_kernel_avg_us"] = {{"k_propagate_weigh": wname, "k_resample": rname}.get(k, k):
                                       round(v[1] * 1e3 / v[0], 3) for k, v in stats.items() if v[0] > 0}
            if pt["per_kernel_avg_us"]:
                dom = max(pt["per_kernel_avg_us"], key=pt["per_kernel_avg_us"].get)
                pmc = os.path.join(ROOT, "profiles", f"pmc_{cfg.name.lower()}_n{cfg.N}.json")
                pt["issue"] = issue_roof(pmc, dom, pt["per_kernel_avg_us"][dom])
        return pt
    finally:
        eng.close()


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

    config = args.config or ("C2" if world == 1 else "C5")
    base = syn.CONFIGS[config]
    sid = rank if args.stream_id < 0 else args.stream_id
    cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=args.particles or base.N, heavy=base.heavy, seed=sid)
    n_frames = args.warmup + args.steps
    kframes = 0 if args.no_timing else (args.kernel_frames or max(20, args.steps))
    st = syn.make_stream(cfg, n_frames + kframes)
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
    if args.keep_prop >= 0:
        eng.set_option(pf.OPT_KEEP_PROPAGATED, args.keep_prop)
    if args.diag:
        eng.set_option(99, args.diag)
    eng.stage_blob_bank([f.blobs for f in st.frames])
    frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                             dt=f.dt, seed=(sid << 32) + 17 + f.index, frame_idx=f.index,
                             force_iters=args.force_iters) for f in st.frames]
    if args.occlude:
        frames = occluded_frames(eng, st, sid, n_frames + kframes, 0)

    for i in range(args.warmup):
        eng.step(frames[i])
    eng.reset_kernel_stats()
    if args.timing_period > 0:  # diagnostics only: brackets inside the timed region
        eng.set_option(pf.OPT_TIMING, args.timing_period)

    if dist:
        dist.barrier()
    timed = frames[args.warmup:n_frames]
    prepared = None if args.python_loop else eng.prepare_batch(timed)  # ctypes arrays built before the clock starts
    t0 = time.perf_counter()
    if args.python_loop:
        outs = [eng.step(f) for f in timed]  # one FFI call per frame
    else:
        outs = eng.run_batch(prepared)  # the C loop a C++ tracker runs; every frame still blocks on its record
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    updates = sum(cfg.N * o.iters for o in outs)
    iters = [o.iters for o in outs]
    accepted = sum(o.accepted for o in outs)
    stats = eng.kernel_stats()
    eng.set_option(pf.OPT_TIMING, 0)
    kiters = iters
    if kframes:  # the kernel pass: the stream's next kframes frames, every one bracketed (kernel_pass)
        stats, kouts = kernel_pass(pf, eng, frames[n_frames:n_frames + kframes])
        kiters = [o.iters for o in kouts]
    if args.dump_records:  # every timed frame's record + a digest of the final particle set, for the tests
        import hashlib
        post = eng.get_particles(1)
        with open(f"{args.dump_records}.{rank}.json", "w") as f:
            json.dump({"stream": sid, "records": [{k: np.asarray(v).tolist() for k, v in o.as_dict().items()}
                                                  for o in outs],
                       "post_sha1": hashlib.sha1(post.tobytes()).hexdigest()}, f)
    shape = eng.info(pf.INFO_LAST_SHAPE)
    weigh_pass = eng.info(pf.INFO_LAST_WEIGH_PASS)
    resample_kind = info_or(pf, eng, pf.INFO_LAST_RESAMPLE)
    fallbacks = eng.info(pf.INFO_FUSED_FALLBACKS)

    elapsed, total_updates = combine_ranks(dist, elapsed, updates)

    worst = None
    if args.worst_frames > 0 and not args.occlude:  # untimed by the driver's contract: reported beside the line
        wf = occluded_frames(eng, st, sid, args.worst_frames, n_frames)
        eng.step(wf[0])  # warm the host-blob path
        prepared = eng.prepare_batch(wf[1:])
        t0 = time.perf_counter()
        wo = eng.run_batch(prepared)
        tw = time.perf_counter() - t0
        wk = float(np.mean([o.iters for o in wo]))
        worst = {"what": "one LED hidden: all 80 re-draw iterations (PE:535-616), host-supplied blobs",
                 "frames": len(wo), "iters_per_frame": wk, "ms_per_frame": tw * 1e3 / len(wo),
                 "updates_per_s": cfg.N * sum(o.iters for o in wo) / tw,
                 "accept_rate": sum(o.accepted for o in wo) / len(wo)}

    multi = None
    default_line = world == 1 and config == "C2" and not args.config and not args.occlude
    sweep = args.multi_sweep or ("1,4,8,16,32" if world == 1 and config == "C2" and not args.occlude else "")
    if sweep == "none":
        sweep = ""
    if sweep and rank == 0:  # untimed by the driver's contract: reported beside the line
        Sb = {"f32": 48, "f16": 24, "f64": 96}[state]
        multi = {"what": "S independent streams of a config per GPU, one batch per frame (pfmpe_step_multi), "
                         "split into `groups` concurrent batches (one host thread and HIP stream each); "
                         "frac = updates/s x (3S+8) B / 8 TB/s (canonical bytes); counter_frac = updates/s x the "
                         "bytes per update the config's one-stream PMC pass measures / 8 TB/s (DRAM occupancy)",
                 "points": []}
        gsweep = [int(x) for x in args.multi_groups.split(",") if x]
        plan = [(base, state_dtype, Sb, S_, G_) for S_ in [int(x) for x in sweep.split(",") if x] for G_ in gsweep
                if not (G_ > 1 and S_ < 2 * G_)]
        if default_line and args.multi_sweep == "":
            # HBM-sized batches: C5 streams (1M particles each; 8M / 32M live particles, above the
            # 256 MiB MALL) as two concurrent batches, and two C4 streams (10M fp16 each) as one batch
            plan += [(syn.CONFIGS["C5"], pf.STATE_F32, 48, 8, 2), (syn.CONFIGS["C5"], pf.STATE_F32, 48, 32, 2),
                     (syn.CONFIGS["C4"], pf.STATE_F16, 24, 2, 1)]
        for cfg_, st_, Sb_, S_, G_ in plan:
            steps_ = args.multi_steps if cfg_.N <= 1_000_000 else max(40, args.multi_steps)  # C4: ~20 ms timed
            pt = multi_stream_point(pf, syn, cfg_, S_, steps_, 5, st_, prm.rng_mode, device, sid, args.prune,
                                    args.keep_prop, G_, args.diag)
            pt["config"] = cfg_.name
            pt["state"] = {pf.STATE_F32: "f32", pf.STATE_F16: "f16", pf.STATE_F64: "f64"}[st_]
            pt["frac"] = round(pt["updates_per_s"] * (3 * Sb_ + 8) / 1e9 / HBM_PEAK_GBPS, 4)
            if cfg_.name in ("C4", "C5"):  # batches of two-launch streams: the one-stream PMC pass's bytes per update
                cb = counter_bytes_per_update(os.path.join(ROOT, "profiles", f"pmc_{cfg_.name.lower()}_n{cfg_.N}.json"),
                                              cfg_.N)
                if cb:
                    pt["counter_bytes_per_update"] = round(cb, 1)
                    pt["counter_frac"] = round(pt["updates_per_s"] * cb / 1e9 / HBM_PEAK_GBPS, 4)
            multi["points"].append(pt)

    exact = None
    if default_line and args.exact_steps > 0 and rank == 0:
        # the parity mode's throughput (fp64 state, the reference's minstd stream: every count, index and pair
        # equals the CPU oracle's), one C2 stream timed like the main line (untimed by the driver's contract)
        exact = single_stream_point(pf, syn, base, args.exact_steps, 10, pf.RNG_REFERENCE, device, sid, args,
                                    state_dtype=pf.STATE_F64)
        exact["what"] = ("C2 in the parity mode: fp64 state + the reference's minstd_rand0 stream (counts, indices and "
                         "pairs identical to the CPU oracle), timed like the main line")

    scale_ref = None
    if world == 1 and config == "C2" and not args.config and not args.occlude and args.scale_ref_steps > 0:
        # the per-GPU workload of the --gpus N > 1 lines (one C5 stream per GPU) on this one GPU, so the
        # N = 1 point of a scaling curve exists for the same workload (untimed by the driver's contract)
        scale_ref = single_stream_point(pf, syn, syn.CONFIGS["C5"], args.scale_ref_steps, 10, prm.rng_mode, device,
                                        sid, args)
        scale_ref["what"] = ("one C5 stream (BASELINE.json configs[4]: M=5, B=50, N=1M, f32) on this GPU, timed like "
                             "the main line: the per-GPU workload of bench.py --gpus N > 1, for its N = 1 point")

    singles = None
    if default_line and rank == 0 and args.single_points not in ("", "none") and args.single_steps > 0:
        # the heavy single-stream configs (BASELINE.json configs[2] / [3]) timed like the main line, each with its
        # own per-kernel HIP-event averages (untimed by the driver's contract)
        singles = {}
        for name in [x for x in args.single_points.split(",") if x]:
            st_ = pf.STATE_F16 if name == "C4" else pf.STATE_F32
            pt = single_stream_point(pf, syn, syn.CONFIGS[name], args.single_steps, 10, prm.rng_mode, device, sid,
                                     args, state_dtype=st_, kernels=True)
            pt["state"] = "f16" if st_ == pf.STATE_F16 else "f32"
            Sb = 24 if st_ == pf.STATE_F16 else 48
            pt["frame_frac"] = round(pt["value"] * (3 * Sb + 8) / 1e9 / HBM_PEAK_GBPS, 4)
            singles[name] = pt

    if rank == 0:
        S = {"f32": 48, "f16": 24, "f64": 96}[state]  # SoA state bytes per particle
        k_mean = float(np.mean(iters)) if iters else 1.0
        ab = algorithmic_bytes(S, cfg.N, float(np.mean(kiters)) if kiters else 1.0)
        roof = None
        timed = {k: v for k, v in stats.items() if v[0] > 0}
        if shape == pf.SHAPE_FRAME2 and "k_frame" in timed:  # PFMPE_K_FRAME times whichever one-launch kernel ran
            timed["k_frame2"] = timed.pop("k_frame")
        wname = {pf.WEIGH_STREAM: "k_weigh_stream", pf.WEIGH_PK: "k_weigh_pk"}.get(weigh_pass)
        if wname and "k_propagate_weigh" in timed:  # the streaming / packed weighing passes
            timed[wname] = timed.pop("k_propagate_weigh")
            ab[wname] = ab["k_propagate_weigh"]
        if resample_kind == pf.RESAMPLE_OWNERS and "k_resample" in timed:  # the deferred resampling
            timed["k_resample_owners"] = timed.pop("k_resample")
            ab["k_resample_owners"] = ab["k_resample"]
        if timed:
            dom = max(timed, key=lambda k: timed[k][1])
            launches, ms = timed[dom]
            avg_s = ms / 1e3 / launches
            achieved = ab.get(dom, 0) / avg_s / 1e9 if avg_s > 0 else 0.0
            pmc = args.pmc or os.path.join(ROOT, "profiles", f"pmc_{cfg.name.lower()}_n{cfg.N}.json")
            traffic = pmc_traffic(pmc, dom)
            upd_bytes = 3 * S + 8
            frame_gbps = total_updates / world / elapsed * upd_bytes / 1e9  # per GPU
            roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    "traffic": None if traffic is None else round(traffic),
                    "traffic_source": os.path.relpath(pmc, ROOT) if traffic is not None else None,
                    "bytes_per_launch": ab.get(dom, 0), "avg_us": round(avg_s * 1e6, 3), "launches_timed": launches,
                    "kernel_pass_frames": kframes,
                    "avg_us_source": (f"HIP-event dispatch timestamps of every frame of a {kframes}-frame kernel pass "
                                      f"right after the (unbracketed) timed region: frames {n_frames}..{n_frames + kframes - 1} "
                                      f"of the stream (scripts/trace_check.py: the same launches in a rocprofv3 trace)"
                                      if kframes else "HIP-event brackets inside the timed region (--timing-period)"),
                    "per_kernel_avg_us": {k: round(v[1] * 1e3 / v[0], 3) for k, v in timed.items()},
                    "frame_level": {"bytes_per_update": upd_bytes, "achieved": round(frame_gbps, 2),
                                    "frac": round(frame_gbps / HBM_PEAK_GBPS, 4),
                                    "what": "updates/s per GPU x (3S+8) B (SURVEY.md §8d), whole frame incl. "
                                            "launch gaps and the host round trip"},
                    "issue": issue_roof(pmc, dom, avg_s * 1e6)}
        cpu = None
        if world == 1 and args.cpu_frames > 0:
            cpu = cpu_baseline(cfg, args.cpu_frames, args.c1_frames)
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
                            + {"C2": " (BASELINE.json configs[1])", "C3": " (configs[2])", "C4": " (configs[3])",
                               "C5": " per GPU (configs[4]: one independent stream per GPU)"}.get(cfg.name, "")
                            + (", worst case: one LED hidden (80 iterations)" if args.occlude else ""),
                "frame_shape": {0: "two-launch", 1: "k_frame", 2: "k_frame2"}.get(shape, str(shape)),
                "fused_fallbacks": fallbacks,
                "state": state,
                "N_particles": cfg.N, "markers": cfg.M, "blobs": cfg.B,
                "frames_per_sec_per_gpu": args.steps / elapsed,
                "iters_per_frame": k_mean, "accept_rate": accepted / max(1, args.steps),
                "rng": args.rng, "parallelism": f"{world} independent camera streams (1 per GPU), no collectives",
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "worst_case": worst,
            "multi_stream": multi,
            "scaling_reference": scale_ref,
            "single_stream": singles,
            "parity_mode": exact,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
