"""Shared helpers: run the oracle and the product on the same region inputs."""
import os
import random

import oracle_py as O
import tfbs_pkg

T = tfbs_pkg.load()

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TD = os.path.join(GOLD, "test_data")


def pattern_dicts(pset):
    """PatternSet -> oracle pattern dicts."""
    out = []
    for p in pset.to_list():
        out.append({"kind": p.kind, "direction": p.direction, "pattern_id": p.pattern_id, "min_score": p.min_score,
                    "weights": [w.acgtn for w in p.weights], "name": p.name})
    return out


def make_regions_synth(seed, first, count, n_samples, lmax, indel_pct=0):
    regs = []
    for j in range(first, first + count):
        r = T.SynthRegion(seed, j, n_samples, lmax, indel_pct)
        regs.append({"merged": r.merged, "ref": r.ref,
                     "records": [("car", pos, ref, alt, car) for pos, ref, alt, car in r.records]})
    return regs


def run_oracle(pset, n_samples, beds, regions, chrom="chr1", min_maf=0):
    """regions: [{"merged": (s,e), "ref": ascii from ext start, "records": [...]}];
    records: ("car", pos, ref, alt, hap_ids) or ("gt", pos, n_alleles, ref, alt, gts)."""
    job = O.Job(n_samples, chrom, pattern_dicts(pset), beds, min_maf)
    keys, stats = [], []
    for reg in regions:
        s, e = reg["merged"]
        rc = job.begin(s, e, reg["ref"])
        assert rc == 0, rc
        for rec in reg["records"]:
            if rec[0] == "car":
                rc = job.add_record_carriers(rec[1], rec[2], rec[3], rec[4])
            else:
                rc = job.add_record_gt(rec[1], rec[2], rec[3], rec[4], rec[5])
            assert rc == 0, rc
        rc = job.end()
        assert rc == 0, rc
        keys.append(job.keys())
        stats.append(job.stats())
    rows = job.rows()
    job.close()
    return keys, rows, stats


def build_batch(pset, n_samples, beds, regions):
    b = T.RegionBatch(pset, n_samples)
    for name, _ in beds:
        b.add_bed(name)
    for reg in regions:
        s, e = reg["merged"]
        b.begin(s, e, reg["ref"])
        for (bi, a, z) in T.select_inner_peaks((s, e), beds):
            b.add_inner(bi, a, z)
        for rec in reg["records"]:
            if rec[0] == "car":
                b.add_record_carriers(rec[1], rec[2], rec[3], rec[4])
            else:
                b.add_record_gt(rec[1], rec[2], rec[3], rec[4], rec[5])
        b.end()
    return b


def run_product(scanner, pset, n_samples, beds, regions, chrom="chr1", min_maf=0, reduce=False, encode=False):
    b = build_batch(pset, n_samples, beds, regions)
    b.scan(scanner, reduce=reduce, encode=encode)
    keys = [b.keys(i) for i in range(b.num_regions)]
    rows, _ = b.rows(chrom, min_maf)
    return keys, rows, b


def synth_patterns(tmpdir, n_pwms, config, seed, thr=1e-4, forward_only=False):
    names = T.synth_write_pwms(str(tmpdir), n_pwms, config, seed)
    return T.parse_pwm_files(os.path.join(str(tmpdir), "pwms.txt"), os.path.join(str(tmpdir), "thr"), thr, names,
                             not forward_only), names


def many_variant_regions(n_samples, lmax, n_sites=(64, 90), seed=12):
    """Regions whose distinct diff count straddles 64 (batch.cpp groups haplotypes by
    a 64-bit diff mask up to 64 distinct diffs and by sorted diff lists beyond):
    SNVs at distinct positions, a few exact duplicate records (one diff), random
    carrier sets, and pairs of records carried by the same haplotypes."""
    rnd = random.Random(seed)
    regs = []
    for j, ns in enumerate(n_sites):
        base = T.SynthRegion(seed, j, n_samples, lmax)
        ref = base.ref
        s, e = base.merged
        es = s - lmax + 1
        positions = rnd.sample(range(len(ref)), ns)
        recs = []
        H = 2 * n_samples
        for k, p in enumerate(positions):
            rb = ref[p]
            if rb == "N":
                continue
            alt = rnd.choice([c for c in "ACGT" if c != rb])
            car = sorted(rnd.sample(range(H), rnd.randint(1, max(1, H // 8))))
            recs.append(("car", es + p, rb, alt, car))
            if k % 17 == 0 and ns > 64:  # the same diff again with other carriers (one rank)
                recs.append(("car", es + p, rb, alt, sorted(rnd.sample(range(H), 3))))
        regs.append({"merged": (s, e), "ref": ref, "records": recs})
    return regs
