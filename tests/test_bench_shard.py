"""Multi-GPU sharding of bench.py on CPU: world_size-2 gloo.

Each rank builds its region shard with bench.shard_batch and reduces with
bench.job_totals, exactly as the N-GPU run does (minus the GPU scan).  The
shards must tile the single-rank workload: no region twice, none missing, and
every region packed byte for byte as the unsharded batch packs it (the packed
input digest: window, inner keys, distinct haplotypes' bases / N masks /
positions, carriers, membership).  The 2-D region x PWM split is checked the
same way: the P pattern shards of a region block partition the pattern_ids,
keep both strands of a PWM together and, with the whole set's window L_max,
pack exactly the unsharded batch's regions."""
import os
import socket
import sys
import tempfile

import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Args:
    samples, regions, seed, indel_pct = 300, 12, 3, 10
    shard, pwm_shards = "regions", None


def _patterns(T, work):
    # length config 3: L = 8 + i % 15, so the pattern shards have different L_max
    names = T.synth_write_pwms(work, 16, 3, 3)
    return T.parse_pwm_files(os.path.join(work, "pwms.txt"), os.path.join(work, "thr"), 1e-3, names)


def _rank(rank, world, port, out, shard):
    import bench
    import tfbs_pkg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = tfbs_pkg.load()

    class A(Args):
        pass

    A.shard = shard
    ps_all = _patterns(T, tempfile.mkdtemp())
    first, count, part, parts = bench.shard_plan(A, rank, world)
    ps = bench.shard_patterns(T, ps_all, part, parts)
    b = bench.shard_batch(T, ps, A, rank, world, window_lmax=ps_all.max_length if parts > 1 else None)
    elapsed = [1.0 + rank, 5.0 - rank]  # max over ranks must win, per entry
    tot = bench.job_totals(dist, "cpu", elapsed, [b.num_windows, b.num_regions, b.num_effective_windows])
    mine = (first, count, part, parts, sorted({p.pattern_id for p in ps.to_list()}),
            [(b.region_stats(r), b.input_digest(r)) for r in range(b.num_regions)])
    every = [None] * world
    dist.all_gather_object(every, mine)
    if rank == 0:
        out.put((tot, every))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, shard):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, shard)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    return res


def _whole(T, ps, n_regions):
    import bench

    class Whole(Args):
        regions = n_regions

    return bench.shard_batch(T, ps, Whole, 0)


def test_two_rank_region_shards_tile_the_workload():
    import tfbs_pkg
    T = tfbs_pkg.load()
    tot, every = _run(2, "regions")
    ps = _patterns(T, tempfile.mkdtemp())
    whole = _whole(T, ps, 2 * Args.regions)
    elapsed, (windows, regions, eff) = tot
    assert elapsed == [2.0, 5.0]
    assert [e[:2] for e in every] == [(0, Args.regions), (Args.regions, Args.regions)]
    got = [x for e in every for x in e[5]]
    assert got == [(whole.region_stats(r), whole.input_digest(r)) for r in range(whole.num_regions)]
    assert regions == whole.num_regions == 2 * Args.regions
    assert windows == whole.num_windows
    assert eff == whole.num_effective_windows


def test_two_rank_region_x_pwm_split():
    """world 2, --shard regions_x_pwms: one region block of 2 R regions, two pattern
    shards; windows add up to the unsharded batch's over all patterns."""
    import tfbs_pkg
    T = tfbs_pkg.load()
    tot, every = _run(2, "regions_x_pwms")
    ps = _patterns(T, tempfile.mkdtemp())
    whole = _whole(T, ps, 2 * Args.regions)
    (first0, count0, part0, parts0, pids0, st0), (first1, count1, part1, parts1, pids1, st1) = every
    assert (first0, count0, part0, parts0) == (0, 2 * Args.regions, 0, 2)
    assert (first1, count1, part1, parts1) == (0, 2 * Args.regions, 1, 2)
    all_pids = sorted({p.pattern_id for p in ps.to_list()})
    assert sorted(pids0 + pids1) == all_pids and not set(pids0) & set(pids1)
    want = [(whole.region_stats(r), whole.input_digest(r)) for r in range(whole.num_regions)]
    assert st0 == want and st1 == want  # the whole set's windows in both shards
    _, (windows, regions, eff) = tot
    assert windows == whole.num_windows
    assert regions == 2 * whole.num_regions


def test_shard_plan_2d_tiles_regions_and_patterns():
    import bench

    class A(Args):
        shard = "regions_x_pwms"
        pwm_shards = 2

    plans = [bench.shard_plan(A, r, 8) for r in range(8)]
    R = A.regions
    assert plans == [((r // 2) * 2 * R, 2 * R, r % 2, 2) for r in range(8)]
    cover = sorted((f, p) for f, _, p, _ in plans)
    assert len(set(cover)) == 8  # every (region block, pattern shard) once
