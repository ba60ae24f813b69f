"""Gaps between the kernels of one train in a rocprofv3 kernel trace: the
host time the GPU waits for (syncs, launch latency, Python between calls).

  python tools/trace_gaps.py gpurun_out/.../run_kernel_trace.csv [--top 15]

Trains are delimited by the first KD pass (kd_pass_kernel<..., false, false,
1, true>); the second-to-last full train is reported (warm, untimed
instrumentation excluded)."""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--top", type=int, default=15)
args = ap.parse_args()
rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "kd_pass_kernel<" in r["Kernel_Name"]
       and "false, false, 1, true>" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
seg = rows[a:b]
t0 = int(seg[0]["Start_Timestamp"])
prev, busy, gaps = t0, 0, []
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gaps.append((s - prev, r["Kernel_Name"][:80]))
    busy += e - s
    prev = max(prev, e)
span = prev - t0
print(f"train span {span / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, "
      f"gaps {(span - busy) / 1e6:.3f} ms, {len(seg)} launches "
      f"({sum(1 for r in seg if 'fillBuffer' in r['Kernel_Name'])} fills)")
for g, n in sorted(gaps, reverse=True)[:args.top]:
    print(f"{g / 1e3:8.1f} us before {n}")
