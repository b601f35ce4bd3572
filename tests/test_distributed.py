"""Multi-rank path of bench.py on CPU (gloo, world_size 2).

The CRC path shards with no data exchange: each rank checksums its own
blocks.  This checks, with real torch.distributed processes, that
bench.shard_range partitions the batch, that bench.timed_steps reduces the
elapsed time with MAX over ranks (the driver's contract), and that the
per-rank shard results reassemble to the single-process answer.
"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    import time
    import torch
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import bench
    from conftest import Oracle
    from golden.splitmix import stream_bytes
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        oracle = Oracle(os.path.join(os.path.dirname(here), "oracle", "liboracle_crc32c.so"))
        n_total, L, seed = 203, 512, 0x5EED0004
        lo, hi = bench.shard_range(n_total, rank, world)
        data = stream_bytes(seed, lo * L, (hi - lo) * L)
        out = {}

        def step():
            out["crc"] = oracle.batch_fixed(data, L, L, hi - lo)
            if rank == 1:
                time.sleep(0.05)  # the slow rank sets the reported time

        def max_reduce(x):
            t = torch.tensor([x], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())

        own = {}

        def max_reduce_own(x):
            own["s"] = x
            return max_reduce(x)

        t_max = bench.timed_steps(step, 3, 1, lambda: None, dist.barrier, max_reduce_own)
        gathered = [None] * world
        dist.all_gather_object(gathered, (lo, hi, out["crc"].tolist(), t_max))
        # bench.py's per-rank table over the same group
        rec = bench.rank_record(rank, own["s"], (hi - lo) * L * 3, None,
                                {"device": rank, "cpu_numa_nodes": bench.numa_node_of_cpus(os.sched_getaffinity(0))})
        ranks = bench.gather_ranks(dist, world, rec)
        q.put((rank, (gathered, ranks)))
    finally:
        dist.destroy_process_group()


def test_shards_partition_and_max_time():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g, ranks = results[0]
    assert (g, ranks) == results[1]
    assert [r["rank"] for r in ranks] == [0, 1] and [r["device"] for r in ranks] == [0, 1]
    assert sum(r["bytes"] for r in ranks) == 203 * 512 * 3
    assert max(r["elapsed_s"] for r in ranks) == pytest.approx(g[0][3], abs=1e-5)  # the MAX is rank 1's
    (lo0, hi0, c0, t0), (lo1, hi1, c1, t1) = g
    assert lo0 == 0 and hi0 == lo1 and hi1 == 203  # disjoint, covering
    assert t0 == t1 and t0 >= 3 * 0.05  # MAX over ranks: the slow rank's time
    from conftest import Oracle
    from golden.splitmix import stream_bytes
    here = os.path.dirname(os.path.abspath(__file__))
    oracle = Oracle(os.path.join(os.path.dirname(here), "oracle", "liboracle_crc32c.so"))
    whole = oracle.batch_fixed(stream_bytes(0x5EED0004, 0, 203 * 512), 512, 512, 203)
    assert np.array_equal(np.array(c0 + c1, dtype=np.uint32), whole)


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 8), (1 << 20, 8), (10, 3)])
def test_shard_range_cover(n, world):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    spans = [bench.shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and a <= b
