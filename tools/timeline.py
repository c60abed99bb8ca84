"""Critical-path view of a rocprofv3 kernel trace: over the last N steps' time span, for each
kernel name, its total time and its EXPOSED time (intervals where it is the only kernel running
on the device), plus device idle time. Usage: python tools/timeline.py run_kernel_trace.csv [nsteps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 4   # window: the last nsteps optimizer steps
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70], r["Stream_Id"]) for r in rows]
ev.sort()
marks = [e[1] for e in ev if "sumsq_kernel" in e[2]]  # one gradient-norm launch per step
t_lo, t_hi = marks[-nsteps - 1], marks[-1]
ev = [e for e in ev if e[0] >= t_lo and e[1] <= t_hi]
span = ev[-1][1] - ev[0][0]
pts = []
for i, (s, e, n, st) in enumerate(ev):
    pts.append((s, 1, i))
    pts.append((e, -1, i))
pts.sort()
active = set()
last = pts[0][0]
excl = defaultdict(float)
tot = defaultdict(float)
idle = 0.0
conc = 0.0
for t, kind, i in pts:
    dt = t - last
    if dt > 0:
        if not active:
            idle += dt
        elif len(active) == 1:
            excl[ev[next(iter(active))][2]] += dt
        else:
            conc += dt
    last = t
    if kind == 1:
        active.add(i)
    else:
        active.discard(i)
for s, e, n, st in ev:
    tot[n] += e - s
print(f"{nsteps} steps: span {span/1e6:.2f} ms  idle {idle/1e6:.2f} ms  concurrent {conc/1e6:.2f} ms  streams {sorted(set(e[3] for e in ev))}")
print(f"{'kernel':70s} {'total ms':>9s} {'exposed ms':>10s}")
for n, v in sorted(excl.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{n:70s} {tot[n]/1e6:9.2f} {v/1e6:10.2f}")
