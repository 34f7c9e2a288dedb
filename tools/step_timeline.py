#!/usr/bin/env python3
"""One bench step's device timeline from a rocprofv3 kernel (+ memory copy) trace:
every dispatch and copy of the last steps in start order, with its start offset from
the step's first dispatch, its duration and the idle gap before it (us).  A step
starts at each zero3_kernel (the scan's counter reset opens every step).

Usage: python tools/step_timeline.py KERNEL_TRACE_CSV [MEMCPY_TRACE_CSV] [STEPS]
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r"tfbs::|\(anonymous namespace\)::|void ", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:48]


def main():
    ev = []
    for r in csv.DictReader(open(sys.argv[1])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    if len(sys.argv) > 2 and sys.argv[2].endswith(".csv"):
        for r in csv.DictReader(open(sys.argv[2])):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "copy " + r.get("Direction", r.get("Operation", "?"))))
    nsteps = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 3
    ev.sort()
    starts = [i for i, e in enumerate(ev) if e[2].startswith("zero3_kernel")]
    if not starts:
        print("no zero3_kernel dispatch")
        return
    for k, i0 in enumerate(starts[-nsteps:]):
        nxt = starts[starts.index(i0) + 1] if starts.index(i0) + 1 < len(starts) else len(ev)
        t0, prev_end = ev[i0][0], ev[i0][0]
        last_end = max(e[1] for e in ev[i0:nxt])
        print("step %d: %.1f us from the first dispatch's start to the last end" % (k, (last_end - t0) / 1e3))
        for s, e, n in ev[i0:nxt]:
            print("  %8.1f  %7.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3, n))
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
