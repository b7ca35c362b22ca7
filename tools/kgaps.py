"""Gaps between consecutive kernels of a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``): per kernel name, calls and average
duration; overall, the GPU-busy fraction of the traced span and the median /
mean idle gap before each kernel. usage: kgaps.py run_kernel_trace.csv [name-substring]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else None
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
if sub:   # the window from the first to the last kernel whose name contains sub
    idx = [i for i, k in enumerate(ks) if sub in k[2]]
    ks = ks[idx[0]:idx[-1] + 1]
busy = sum(e - s for s, e, _ in ks)
span = ks[-1][1] - ks[0][0]
gaps = [max(0, ks[i][0] - ks[i - 1][1]) for i in range(1, len(ks))]
print("kernels %d  span %.3f ms  busy %.3f ms (%.1f %%)  gap median %.2f us mean %.2f us max %.1f us"
      % (len(ks), span / 1e6, busy / 1e6, 100.0 * busy / span, statistics.median(gaps) / 1e3,
         statistics.mean(gaps) / 1e3, max(gaps) / 1e3))
per = {}
for i, (s, e, n) in enumerate(ks):
    p = per.setdefault(n[:90], [0, 0, 0])
    p[0] += 1
    p[1] += e - s
    p[2] += gaps[i - 1] if i else 0
for n, (c, t, g) in sorted(per.items(), key=lambda x: -x[1][1]):
    print("%-90s %6d  avg %8.2f us  avg gap before %6.2f us" % (n, c, t / c / 1e3, g / c / 1e3))
