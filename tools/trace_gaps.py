"""Where the pipelined batch stream spends the time k_accumulate is not running.

Reads a rocprofv3 --kernel-trace CSV of the pipelined bench (tools/prof.sh pipelined), takes the
steady-state span from the first to the last k_accumulate, and reports per batch: the span, the
time covered by at least one k_accumulate, the time covered by two or more, the time with no
kernel at all, and -- over the time with no k_accumulate -- each kernel's share of the covered
time (a kernel's wall time there divided by the number of kernels running alongside it).

python tools/trace_gaps.py <run_kernel_trace.csv> [LO:HI | sI-J]

LO:HI restricts the window to the k_accumulate launches inside [LO, HI] ms from the first one
(e.g. the timed region, which follows the warm-up's drain; the segment list printed first shows
where the drains are); sI-J restricts it to segments I..J of that list (0-based).
"""
import collections
import csv
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("kzgmi::", "")
    return n.split("<")[0]


def main(path):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    acc = [e for e in ev if e[2] == "k_accumulate"]
    # segments: runs of k_accumulate launches with no stretch of more than 0.5 ms without one
    segs, cur, end = [], [acc[0]], acc[0][1]
    for a in acc[1:]:
        if a[0] - end > 5e5:
            segs.append((cur, a[0] - end))
            cur = []
        cur.append(a)
        end = max(end, a[1])
    segs.append((cur, 0))
    print("k_accumulate segments (launches, then the gap to the next in ms): " +
          ", ".join("%d (%.2f)" % (len(s), g / 1e6) for s, g in segs))
    t0, t1 = acc[0][0], acc[-1][1]
    if len(sys.argv) > 2 and sys.argv[2].startswith("s"):  # segments I..J (0-based) of the list
        i, _, j = sys.argv[2][1:].partition("-")
        acc = [a for s, _ in segs[int(i):int(j or i) + 1] for a in s]
        t0, t1 = acc[0][0], acc[-1][1]
    elif len(sys.argv) > 2:  # a time window in ms from the first k_accumulate
        lo, hi = (float(x) for x in sys.argv[2].split(":"))
        acc = [a for a in acc if a[0] >= t0 + lo * 1e6 and a[1] <= t0 + hi * 1e6]
        t0, t1 = acc[0][0], acc[-1][1]
    nb = len(acc)
    pts = []
    for s, e, n in ev:
        s, e = max(s, t0), min(e, t1)
        if s < e:
            pts.append((s, 1, n))
            pts.append((e, -1, n))
    pts.sort(key=lambda p: (p[0], p[1]))
    active = collections.Counter()
    covered = covered2 = idle = 0.0
    share = collections.Counter()
    last = t0
    for t, d, n in pts:
        dt = t - last
        if dt > 0:
            a = active["k_accumulate"]
            tot = sum(active.values())
            if a >= 1:
                covered += dt
            if a >= 2:
                covered2 += dt
            if tot == 0:
                idle += dt
            elif a == 0:
                for k, v in active.items():
                    if v:
                        share[k] += dt * v / tot
        active[n] += d
        last = t
    span = (t1 - t0) / 1e6
    print("window: %d k_accumulate launches, span %.3f ms" % (nb, span))
    print("per batch: span %.3f ms, k_accumulate covers %.3f ms (%.1f %%), >= 2 k_accumulate %.3f ms"
          % (span / nb, covered / 1e6 / nb, 100 * covered / (t1 - t0), covered2 / 1e6 / nb))
    print("per batch: no k_accumulate %.3f ms, no kernel at all %.3f ms"
          % ((t1 - t0 - covered) / 1e6 / nb, idle / 1e6 / nb))
    print("time with no k_accumulate, shared over the kernels running (ms per batch):")
    for k, v in share.most_common(16):
        print("  %-28s %.3f" % (k, v / 1e6 / nb))


if __name__ == "__main__":
    main(sys.argv[1])
