#!/usr/bin/env python3
"""Device timeline of the drop-in loop from a rocprofv3 run (kernel + memory-copy traces): one env
step = the span between consecutive replay launches (k_replay_put_gather / k_replay_gather).
Prints, per step (median over the steady steps): the period, the device-busy time, each kernel's
and copy's median duration and start offset within the step, and the idle gaps -- where the
drop-in's step goes on the device and where the device waits for the host.

usage: dropin_timeline.py KERNEL_TRACE.csv [MEMORY_COPY_TRACE.csv]"""
import collections
import csv
import statistics
import sys


def load(path, kind):
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Direction") or kind
        if kind == "copy":
            name = "copy " + name
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0].split("<")[0][-28:]))
    return out


def main():
    ev = load(sys.argv[1], "kernel")
    if len(sys.argv) > 2:
        ev += load(sys.argv[2], "copy")
    ev.sort()
    marks = [i for i, e in enumerate(ev) if "replay_put_gather" in e[2] or e[2].endswith("k_replay_gather")]
    steps = []
    for a, b in zip(marks, marks[1:]):
        seg = ev[a:b + 1]
        t0, t1 = seg[0][0], seg[-1][0]
        busy, gaps, last_end = 0, [], t0
        rows = []
        for s, e, n in seg[:-1]:
            if s > last_end:
                gaps.append((s - last_end, n))
            busy += max(0, e - max(s, last_end))
            last_end = max(last_end, e)
            rows.append((n, s - t0, e - s))
        steps.append((t1 - t0, busy, gaps, rows))
    steady = steps[len(steps) // 4:]  # skip warm-up
    per = [s[0] / 1000 for s in steady]
    print(f"{len(steady)} steady steps: period median {statistics.median(per):.1f} us, "
          f"device busy median {statistics.median([s[1] / 1000 for s in steady]):.1f} us")
    by = collections.defaultdict(list)
    for s in steady:
        seen = collections.Counter()
        for n, off, dur in s[3]:
            seen[n] += 1
            by[(n, seen[n])].append((off / 1000, dur / 1000))
    print(f"{'launch':34s} {'n':>5s} {'start':>8s} {'dur':>7s}")
    for k, v in sorted(by.items(), key=lambda kv: statistics.median([x[0] for x in kv[1]])):
        if len(v) < len(steady) // 2:
            continue
        print(f"{k[0] + '#' + str(k[1]):34s} {len(v):5d} {statistics.median([x[0] for x in v]):8.1f} "
              f"{statistics.median([x[1] for x in v]):7.2f}")
    g = collections.defaultdict(list)
    for s in steady:
        for dt, n in s[2]:
            g[n].append(dt / 1000)
    print("idle gaps before (summed per step, median of those > 0):")
    for n, v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:32s} {sum(v) / len(steady):7.1f} us/step  (median {statistics.median(v):.1f})")


if __name__ == "__main__":
    main()
