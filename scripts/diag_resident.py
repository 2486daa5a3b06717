"""Resident frame server phases at C2 (diagnostic): per frame, the device duration the server reports (doorbell seen
-> record out) in steady state, and the stamped phases of steady-state frames (PFMPE_DIAG 4; with the server running
pfmpe_debug_stamps reads them on a side stream, so the server is not restarted per frame): doorbell seen, slot
published, first / last block body start, weighing barrier, top, final record."""
import sys, os, time, ctypes as C
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import pf_monocular_pose_estimator_amd as pf
from pf_monocular_pose_estimator_amd import synthetic as syn

lib = pf.load()
lib.pfmpe_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
base = syn.CONFIGS["C2"]
cfg = syn.StreamConfig(base.name, M=base.M, B=base.B, N=N, heavy=base.heavy)
st = syn.make_stream(cfg, 40)
for resident in (1, 0):
    eng = pf.Engine(0, N)
    eng.set_model(st.markers, st.K)
    eng.set_params(pf.default_params())
    eng.set_prior(st.prior())
    eng.set_option(pf.OPT_RESIDENT, resident)
    eng.stage_blob_bank([f.blobs for f in st.frames])
    frames = [eng.make_frame(f.current_pose, f.predicted_pose, f.prediction, B=len(f.blobs), bank_frame=f.index,
                             dt=f.dt, seed=3, frame_idx=f.index) for f in st.frames]
    for f in frames[:5]:
        eng.step(f)
    eng.reset_kernel_stats()
    eng.set_option(pf.OPT_TIMING, 1)
    t0 = time.perf_counter()
    for f in frames[5:]:
        eng.step(f)
    el = (time.perf_counter() - t0) / (len(frames) - 5)
    hn, wn, fn = eng.info(100), eng.info(101), eng.info(102)
    n, ms = eng.kernel_stats()["k_frame"]
    print(f"resident={resident}: {el * 1e6:.2f} us/frame host, device {ms * 1e3 / max(n, 1):.2f} us/frame ({n} timed)")
    if fn:
        print(f"    host record -> next doorbell {hn / fn / 1e3:.2f} us, doorbell -> record {wn / fn / 1e3:.2f} us ({fn})")
    # the C loop (pfmpe_step_batch), timing off
    prepared = eng.prepare_batch(frames[5:])
    eng.run_batch(prepared)
    h0, w0, f0 = eng.info(100), eng.info(101), eng.info(102)
    t0 = time.perf_counter()
    eng.run_batch(prepared)
    el = (time.perf_counter() - t0) / (len(frames) - 5)
    fn = eng.info(102) - f0
    msg = f"    C loop {el * 1e6:.2f} us/frame"
    if fn:
        msg += f"; host record -> next doorbell {(eng.info(100) - h0) / fn / 1e3:.2f} us, doorbell -> record {(eng.info(101) - w0) / fn / 1e3:.2f} us"
    print(msg)
    eng.set_option(pf.OPT_TIMING, 0)
    eng.set_option(99, 4)
    for f in frames[:3]:
        eng.step(f)
    rows = []
    for f in frames[5:]:
        lib.pfmpe_debug_stamps(eng.ctx, None)
        eng.step(f)
        s = (C.c_uint64 * 32)()
        lib.pfmpe_debug_stamps(eng.ctx, s)
        t = np.array(list(s), dtype=np.float64)
        rows.append([(t[i] - t[0]) / 100.0 if t[i] else float("nan") for i in range(32)])
    r = np.median(np.array(rows), axis=0)
    names = {4: "doorbell seen (srv)", 30: "slot published (srv)", 0: "first block body start", 19: "table built (first)",
             8: "table built (last)", 9: "weights (last)", 23: "arrival issued (last)", 31: "barrier passed (first)",
             2: "barrier passed (last)", 3: "top done (last)", 12: "scatter (last)", 5: "count partial (last)",
             6: "final start", 7: "record published", 13: "fin Pm", 14: "fin P", 15: "fin minima", 16: "fin score",
             17: "fin record", 18: "fin published"}
    for i in sorted(names, key=lambda i: (np.nan_to_num(r[i], nan=1e9))):
        print(f"    {names[i]:26s} {r[i]:8.2f}")
    eng.close()
