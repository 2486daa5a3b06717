"""The bench line's kernel timing against a rocprofv3 kernel trace of the same command.

  python3 scripts/trace_check.py <trace dir> <bench log of the traced run> [--untraced <bench log of the same
                                 command without the profiler>] [--warmup W --steps S]

bench.py times its main line without HIP-event brackets and then runs a kernel pass of K more frames with every
frame bracketed (bench.py kernel_pass); roofline.avg_us is that pass's average of the dominant kernel.  Under the
profiler the HIP events read long (its own completion signals on every dispatch), so the line to check is the same
command's run WITHOUT the profiler (--untraced); the traced run's own line is printed beside it.  The trace holds the
same process's launches in order, so for the dominant kernel (one launch per one-launch frame, the first kernel of a
two-launch frame) launch i < W is warm-up, W <= i < W + S the timed frames and W + S <= i < W + S + K the kernel
pass.  Prints each section's mean / median from the trace, the line's figure and the ratio line / trace."""
import argparse
import csv
import json
import statistics
import sys

NAMES = {"k_frame2": "pfmpe::k_frame2<", "k_weigh_pk": "pfmpe::k_weigh_pk<", "k_weigh_pk12": "pfmpe::k_weigh_pk12<",
         "k_weigh_stream": "pfmpe::k_weigh_stream<", "k_resample_owners": "pfmpe::k_resample_owners<",
         "k_frame": "pfmpe::k_frame<"}


def load_line(path):
    return json.loads([ln for ln in open(path).read().splitlines() if ln.startswith('{"metric"')][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("traced_log")
    ap.add_argument("--untraced", default="", help="bench log of the same command without the profiler")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    traced = load_line(a.traced_log)
    line = load_line(a.untraced) if a.untraced else traced
    roof = line["roofline"]
    kern = roof["kernel"]
    K = int(roof.get("kernel_pass_frames") or 0)
    rows = sorted(csv.DictReader(open(f"{a.trace}/run_kernel_trace.csv")), key=lambda t: int(t["Start_Timestamp"]))
    want = NAMES.get(kern, kern)
    cand = {}
    for t in rows:
        if want in t["Kernel_Name"]:
            cand.setdefault(t["Kernel_Name"], []).append((int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3)
    # the main line's instantiation: the first kernel name that matches, launched at least W + S + K times
    name, durs = next(((n, d) for n, d in cand.items() if len(d) >= a.warmup + a.steps + K), (None, []))
    if not name:
        sys.exit(f"no instantiation of {want} with {a.warmup + a.steps + K} launches: "
                 f"{ {n[:60]: len(d) for n, d in cand.items()} }")
    sec = {"warmup": durs[:a.warmup], "timed": durs[a.warmup:a.warmup + a.steps],
           "kernel_pass": durs[a.warmup + a.steps:a.warmup + a.steps + K], "later": durs[a.warmup + a.steps + K:]}
    print(f"kernel {name[:90]}: {len(durs)} launches in the trace")
    for k, v in sec.items():
        if v:
            print(f"  {k:12s} n={len(v):4d} mean {statistics.mean(v):8.2f} us  median {statistics.median(v):8.2f} us"
                  f"  min {min(v):8.2f}  max {max(v):8.2f}")
    tp = statistics.mean(sec["kernel_pass"]) if sec["kernel_pass"] else float("nan")
    tt = statistics.mean(sec["timed"]) if sec["timed"] else float("nan")
    src = "untraced run" if a.untraced else "traced run"
    print(f"line ({src}) avg_us {roof['avg_us']:.2f}, frac {roof['frac']}, issue_frac "
          f"{(roof.get('issue') or {}).get('issue_frac')}; the traced run's own line: avg_us "
          f"{traced['roofline']['avg_us']:.2f}")
    print(f"trace kernel-pass mean {tp:.2f} us -> line / trace {roof['avg_us'] / tp:.3f}; trace timed-frames mean "
          f"{tt:.2f} us -> line / trace {roof['avg_us'] / tt:.3f}")
    fr = roof["bytes_per_launch"] / (tt * 1e-6) / 1e9 / roof["peak"]
    iss = roof.get("issue") or {}
    ifr = iss.get("issue_frac")
    print(f"from the trace's timed frames: frac {fr:.4f} (line {roof['frac']}), issue_frac "
          f"{ifr * roof['avg_us'] / tt if ifr else None} (line {ifr})")


if __name__ == "__main__":
    main()
