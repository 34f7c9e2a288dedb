"""Multi-GPU sharding of bench.py on CPU: world_size-2 gloo.

Each rank builds its region shard with bench.shard_batch and reduces with
bench.job_totals, exactly as the N-GPU run does (minus the GPU scan).  The
shards must tile the single-rank workload: no region twice, none missing, the
same distinct haplotypes and windows."""
import os
import socket
import sys
import tempfile

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Args:
    samples, regions, seed, indel_pct = 300, 12, 3, 10


def _patterns(T, work):
    names = T.synth_write_pwms(work, 8, 2, 3)
    return T.parse_pwm_files(os.path.join(work, "pwms.txt"), os.path.join(work, "thr"), 1e-3, names)


def _rank(rank, world, port, out):
    import bench
    import tfbs_pkg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    T = tfbs_pkg.load()
    ps = _patterns(T, tempfile.mkdtemp())
    b = bench.shard_batch(T, ps, Args, rank)
    elapsed = [1.0 + rank, 5.0 - rank]  # max over ranks must win, per entry
    tot = bench.job_totals(dist, "cpu", elapsed, [b.num_windows, b.num_regions, b.num_effective_windows])
    # the shards' regions, in rank order, as the whole job sees them
    mine = [b.region_stats(r) for r in range(b.num_regions)]
    every = [None] * world
    dist.all_gather_object(every, mine)
    if rank == 0:
        out.put((tot, [x for part in every for x in part]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_tile_the_workload():
    import bench
    import tfbs_pkg
    T = tfbs_pkg.load()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    tot, stats = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    ps = _patterns(T, tempfile.mkdtemp())

    class Both(Args):
        regions = 2 * Args.regions

    whole = bench.shard_batch(T, ps, Both, 0)
    elapsed, (windows, regions, eff) = tot
    assert elapsed == [2.0, 5.0]
    assert stats == [whole.region_stats(r) for r in range(whole.num_regions)]
    assert regions == whole.num_regions == 2 * Args.regions
    assert windows == whole.num_windows
    assert eff == whole.num_effective_windows
