"""Per-launch view of the last optimizer step of a rocprofv3 kernel trace: every launch in issue
order with its stream, grid, duration and the device-idle time right before it, then the idle gaps
grouped by the (previous kernel -> next kernel) pair and the launches grouped by (kernel, grid).
Usage: python tools/step_launches.py run_kernel_trace.csv [--list] [--top N]"""
import csv
import sys
from collections import defaultdict


def short(n, w=58):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:w] if "<" not in n.split("(")[0] else n[: n.find(">") + 1][:w]


def main():
    path = sys.argv[1]
    show_list = "--list" in sys.argv
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Stream_Id"], grid // max(wg, 1)))
    ev.sort()
    marks = [e[1] for e in ev if "sumsq_kernel" in e[2]]  # one gradient-norm launch per step
    lo, hi = marks[-2], marks[-1]
    ev = [e for e in ev if e[0] >= lo and e[1] <= hi]
    busy_until = lo
    gaps = defaultdict(lambda: [0, 0.0])
    groups = defaultdict(lambda: [0, 0.0])
    prev = "sumsq_kernel"
    idle_total = 0.0
    for s, e, n, st, nwg in ev:
        gap = max(0, s - busy_until)
        idle_total += gap
        if gap > 0:
            g = gaps[(prev, n)]
            g[0] += 1
            g[1] += gap
        if show_list:
            print(f"{(s - lo) / 1e3:9.1f} us  gap {gap / 1e3:6.1f}  dur {(e - s) / 1e3:8.1f}  s{st}  wg {nwg:7d}  {n}")
        grp = groups[(n, nwg)]
        grp[0] += 1
        grp[1] += e - s
        if e > busy_until:
            busy_until = e
            prev = n
    span = hi - lo
    print(f"step span {span / 1e6:.2f} ms, device idle {idle_total / 1e6:.2f} ms in {sum(g[0] for g in gaps.values())} gaps, {len(ev)} launches")
    print("\nidle by (previous -> next kernel):")
    for (a, b), (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {t / 1e3:8.1f} us  {c:4d} x  {a}  ->  {b}")
    print("\nlaunch groups by (kernel, workgroups): total ms, count, avg us")
    for (n, nwg), (c, t) in sorted(groups.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {t / 1e6:7.3f} ms  {c:4d} x  {t / c / 1e3:8.1f} us  wg {nwg:7d}  {n}")


if __name__ == "__main__":
    main()
