"""Per-step kernel breakdown from a rocprofv3 kernel trace: the window of the
last N occurrences of an anchor kernel (one per step), every kernel in it
averaged per step, plus the idle time between kernels.
usage: kstep.py run_kernel_trace.csv anchor-substring [N [seq]]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
idx = [i for i, k in enumerate(ks) if anchor in k[2]]
if len(idx) < n + 1:
    n = len(idx) - 1
a, b = idx[-n - 1], idx[-1]
win = ks[a:b]
span = ks[b][0] - ks[a][0]
per = {}
busy = 0
for s, e, name in win:
    p = per.setdefault(name[:100], [0, 0])
    p[0] += 1
    p[1] += e - s
    busy += e - s
print("steps %d  per step: span %.1f us  kernels busy %.1f us  idle %.1f us"
      % (n, span / n / 1e3, busy / n / 1e3, (span - busy) / n / 1e3))
for name, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
    print("%-100s  %5.2f/step  avg %8.2f us  per step %8.2f us" % (name, c / n, t / c / 1e3, t / n / 1e3))
if len(sys.argv) > 4 and sys.argv[4] == "seq":   # the last window's launches in order
    s0 = ks[idx[-2]][0]
    prev = None
    for s, e, name in ks[idx[-2]:idx[-1]]:
        print("%9.2f  %7.2f us  gap %6.2f  %s" % ((s - s0) / 1e3, (e - s) / 1e3,
                                                (s - prev) / 1e3 if prev else 0.0, name[:90]))
        prev = e
