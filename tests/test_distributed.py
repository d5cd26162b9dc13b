"""Multi-process (gloo, world size 2, CPU) coverage of bench.py's N>1 path:
one broadcast of the weight blob from rank 0, per-rank sequence shards, and
the max-over-ranks wall time.  The per-frame path has no collective."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    isd, psd = bench.make_weights(dist, rank, torch.device("cpu"))
    digest = torch.tensor([float(sum(v.double().sum() for v in isd.values())),
                           float(sum(v.double().sum() for v in psd.values())), float(len(psd))],
                          dtype=torch.float64)
    got = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(got, digest)
    t = bench.max_over_ranks(dist, 1.0 + rank, torch.device("cpu"))
    out[rank] = (torch.stack(got).tolist(), t, bench.shard_seed(rank))
    dist.destroy_process_group()


def test_weight_broadcast_and_shards_world2():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    digests0, t0, s0 = res[0]
    digests1, t1, s1 = res[1]
    # every rank holds rank 0's weights
    assert digests0[0] == digests0[1] and digests0 == digests1
    assert digests0[0][2] > 600  # the DC inter-model parameter list
    # wall time is the slowest rank's; shards are distinct sequences
    assert t0 == t1 == 2.0
    assert s0 != s1
