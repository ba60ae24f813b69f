"""Short per-kernel table of a rocprofv3 *_kernel_stats.csv (name, calls,
avg us, total ms), longest first."""
import csv
import re
import sys


def short(name):
    m = re.search(r"pd::\(anonymous namespace\)::(\w+)", name)
    if m:
        return m.group(1) + (re.search(r"<([^()]*)>", name).group(1)[:30]
                             if re.search(r"<([^()]*)>", name) else "")
    if "rocprim" in name:
        for k in ("onesweep_iteration", "onesweep_global_offsets", "partition", "scan",
                  "lookback", "transform"):
            if k in name:
                return "rocprim_" + k
    return name[:50]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
lim = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
for r in rows[:lim]:
    print("%-48s %5s %10.1f %9.3f" % (short(r["Name"])[:48], r["Calls"],
                                      float(r["AverageNs"]) / 1e3,
                                      float(r["TotalDurationNs"]) / 1e6))
print("total %.3f ms" % (tot / 1e6))
