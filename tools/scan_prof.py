#!/usr/bin/env python3
"""Summarise a TFBS_SCAN_PROF dump (a TFBS_SCAN_PROF build of scan_mfma.hip,
tools/variant_build.sh scan_mfma NAME:-DTFBS_SCAN_PROF, run with
TFBS_SCAN_PROF=<file>): per launch (depth class), the waves' time in each phase --
staging (kernel start to the staging barrier), the scan loop, the last queue drain,
the rescoring -- in shader cycles, pairs of window tiles per wave, candidates per
wave, and from the chip-wide 100 MHz clock the launch's span and its tail (the
time after 90 / 99 % of its workgroups ended).  The last scan in the file is read.

Usage: python tools/scan_prof.py FILE [OUT_JSON]
"""
import json
import sys

import numpy as np


def read(path):
    raw = np.fromfile(path, dtype=np.uint64)
    scans, i = [], 0
    while i < len(raw):
        n_srcs, n = int(raw[i]), int(raw[i + 1])
        i += 2
        srcs = raw[i:i + 5 * n_srcs].reshape(n_srcs, 5)
        i += 5 * n_srcs
        scans.append((srcs, raw[i:i + n].reshape(-1, 8, 16)))
        i += n
    return scans


def main():
    srcs, d = read(sys.argv[1])[-1]
    out = {"launches": []}
    for wg_base, ns, g0, ng, idx in srcs.tolist():
        w = d[wg_base:wg_base + ns * ng].astype(np.int64)  # [wg][wave][field]
        live = w[:, :, 0] != 0
        ph = {
            "staging": w[:, :, 1] - w[:, :, 0],
            "loop": w[:, :, 2] - w[:, :, 1],
            "drain": w[:, :, 3] - w[:, :, 2],
            "rescore": w[:, :, 4] - w[:, :, 3],
        }
        tot = sum(ph.values())
        pairs = (w[:, :, 7] & 0xFFFFFFFF)[live]
        cands = (w[:, :, 7] >> 32)[live]
        r0 = w[:, 0, 5][live[:, 0]]
        r1 = w[:, :, 6].max(axis=1)[live[:, 0]]
        span = (r1.max() - r0.min()) / 100.0  # us (100 MHz)
        ends = np.sort(r1 - r0.min()) / 100.0
        wg_us = (r1 - r0) / 100.0
        rec = {
            "launch": int(idx), "workgroups": int(live[:, 0].sum()),
            "phase_cycles_mean_per_wave": {k: float(v[live].mean()) for k, v in ph.items()},
            "phase_share": {k: float(v[live].sum() / tot[live].sum()) for k, v in ph.items()},
            "pairs_per_wave": {"mean": float(pairs.mean()), "p10": float(np.percentile(pairs, 10)),
                               "p90": float(np.percentile(pairs, 90))},
            "cycles_per_pair_in_loop": float(ph["loop"][live].sum() / max(1, pairs.sum())),
            "candidates_per_wave": {"mean": float(cands.mean()), "max": int(cands.max())},
            "span_us": float(span),
            "workgroup_us": {"mean": float(wg_us.mean()), "p50": float(np.median(wg_us)),
                             "max": float(wg_us.max())},
            "tail_us": {"after_90pct_end": float(span - ends[int(0.9 * (len(ends) - 1))]),
                        "after_99pct_end": float(span - ends[int(0.99 * (len(ends) - 1))])},
        }
        if w[:, :, 12].sum() > 0:  # TFBS_ROUND_PROF build: the two-tile rounds' clock split
            rb, rm, rt, rf, nr, nf, rs, pp = (w[:, :, 8 + k][live].sum() for k in range(8))
            loop = ph["loop"][live].sum()
            rec["round_split"] = {
                "rounds_per_wave": float(nr / live.sum()), "fired_share": float(nf / max(1, nr)),
                "cycles_per_round": {"to_first_mfma": float(rb / nr), "first_to_last_mfma": float(rm / nr),
                                     "last_mfma_to_test": float(rt / nr), "firing_path": float(rf / nr)},
                "loop_share": {"to_first_mfma": float(rb / loop), "first_to_last_mfma": float(rm / loop),
                               "last_mfma_to_test": float(rt / loop), "firing_path": float(rf / loop),
                               "restaging": float(rs / loop), "pair_setup": float(pp / loop),
                               "other": float(1 - (rb + rm + rt + rf + rs + pp) / loop)},
            }
        out["launches"].append(rec)
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
