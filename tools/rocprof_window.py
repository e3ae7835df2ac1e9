#!/usr/bin/env python3
"""Average duration of the roofline kernel's launches inside bench.py's prof window, from a
rocprofv3 --kernel-trace of the same command.

bench.py times the dominant kernel kind live with HIP events over `--prof-steps` steps after the
timed window and its repeats, and prints that window's CLOCK_MONOTONIC bounds and launch count
(roofline.prof_window).  rocprofv3 stamps dispatches on the same clock, so the dispatches of that
kind starting and ending inside the bounds are the same launches.

usage: rocprof_window.py KERNEL_TRACE_CSV BENCH_LOG OUT_JSON
Writes {kernel, window_launches, window_avg_us, live_launches, live_avg_us, run_launches,
run_avg_us, source}."""
import csv
import json
import sys


def base_name(name):
    return name.split("(")[0].split("<")[0].split("::")[-1].strip()


def main():
    trace, log, out = sys.argv[1:4]
    line = [l for l in open(log).read().splitlines() if l.startswith("{")][-1]
    roof = json.loads(line)["roofline"]
    kern, win = roof["kernel"], roof["prof_window"]
    t0, t1 = int(win["t0_ns"]), int(win["t1_ns"])
    n_win = n_run = 0
    ns_win = ns_run = 0.0
    with open(trace, newline="") as f:
        for r in csv.DictReader(f):
            b = base_name(r["Kernel_Name"])
            if not (b == kern or b.startswith(kern + "_")):
                continue
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            n_run += 1
            ns_run += e - s
            if s >= t0 and e <= t1:
                n_win += 1
                ns_win += e - s
    res = {"kernel": kern,
           "window_launches": n_win, "window_avg_us": ns_win / n_win / 1e3 if n_win else None,
           "live_launches": win["launches"], "live_avg_us": roof["avg_launch_us"],
           "run_launches": n_run, "run_avg_us": ns_run / n_run / 1e3 if n_run else None,
           "window_steps": win["steps"],
           "source": "rocprofv3 --kernel-trace of `python3 bench.py --no-cpu-baseline --no-other --shard-steps 0` "
                     "(default steps / warmup / repeats / prof-steps); window = the bench's prof window bounds"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))
    return 0 if n_win else 1


if __name__ == "__main__":
    sys.exit(main())
