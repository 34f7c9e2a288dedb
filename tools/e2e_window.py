"""GPU occupancy of bench.py's end-to-end rows + encode window, from a rocprofv3 database.

Usage: python3 tools/e2e_window.py <run_results.db>
(rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o run -- python3 bench.py --workload C5 ...)
Prints the window (first key_encode_kernel to the last bgzf kernel), the time the GPU's kernels and
copies were busy in it, the kernels' totals and the idle gaps by the operations on either side.
"""
import collections
import re
import sqlite3
import sys


def busy(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return (tot + (ce - cs if cs is not None else 0)) / 1e9


def short(n):
    return re.sub(r"tfbs::\(anonymous namespace\)::", "", n)[:44]


def main(db):
    c = sqlite3.connect(db)
    K = [(n, s, e, "kernel") for n, s, e in c.execute("select name, start, end from kernels")]
    M = [(n, s, e, "copy") for n, s, e in c.execute("select name, start, end from memory_copies")]
    t0 = min(s for n, s, e, _ in K if "key_encode" in n or "bgzf" in n)
    t1 = max(e for n, s, e, _ in K if "bgzf" in n)
    A = sorted([a for a in K + M if a[1] >= t0 and a[2] <= t1], key=lambda a: a[1])
    kin = [(s, e) for n, s, e, t in A if t == "kernel"]
    cin = [(s, e) for n, s, e, t in A if t == "copy"]
    print("rows + encode window %.3f s: kernels busy %.3f s, copies %.3f s, either %.3f s"
          % ((t1 - t0) / 1e9, busy(kin), busy(cin), busy(kin + cin)))
    agg = collections.Counter()
    for n, s, e, t in A:
        if t == "kernel":
            agg[short(n)] += (e - s) / 1e9
    for n, v in agg.most_common(8):
        print("  %.4f s  %s" % (v, n))
    gaps, ce = [], A[0][2]
    for i in range(1, len(A)):
        if A[i][1] > ce:
            gaps.append(((A[i][1] - ce) / 1e6, i))
        ce = max(ce, A[i][2])
    by = collections.Counter()
    for g, i in gaps:
        by[(short(A[i - 1][0]), short(A[i][0]))] += g
    print("idle: %d gaps, %.1f ms; by the operations either side:" % (len(gaps), sum(g for g, _ in gaps)))
    for (a, b), v in by.most_common(6):
        print("  %6.1f ms  %s -> %s" % (v, a, b))


if __name__ == "__main__":
    main(sys.argv[1])
