"""CPU, world_size 2 over gloo: the sharded consensus -- blocks
split contiguously over ranks, ONE all-reduce of the support-restricted
sum_j (D_j + y_j) per d-iteration and ONE broadcast of block 1's filter
spectrum per outer iteration -- reproduces the single-process learner.  This is
the exchange schedule the engine runs over RCCL (engine.cpp outer_iteration)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.ccsc_port import DzPort, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    rng = np.random.default_rng(42)
    ni, N = 2, 5                      # 5 blocks over 2 ranks: 3 + 2 (uneven, like 13/12)
    b = rng.standard_normal((10, 9, ni * N))
    d0 = rng.standard_normal((5, 5, 3))
    z0 = rng.standard_normal((14, 13, 3, ni))
    return b, d0, z0, ni, N


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, d0, z0, ni, N = _problem()
    b0, nb = shard(N, rank, world)

    def allreduce(x):
        t = torch.from_numpy(x.copy())
        dist.all_reduce(t)
        return t.numpy()

    def bcast(x):
        t = torch.from_numpy(x.copy())
        dist.broadcast(t, src=0)
        return t.numpy()

    p = DzPort(b[:, :, b0 * ni:(b0 + nb) * ni], d0, z0, 1.0, ni=ni, workers=1, N=N, rank=rank,
               world=world, allreduce=allreduce, bcast=bcast)
    for _ in range(2):
        p.outer()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), z=p.z, D1=p.D[0], u=p.u, b0=b0, nb=nb)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_consensus_equals_single_process(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    b, d0, z0, ni, N = _problem()
    ref = DzPort(b, d0, z0, 1.0, ni=ni, workers=1)
    for _ in range(2):
        ref.outer()
    parts = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    assert [int(q["nb"]) for q in parts] == [3, 2]
    z = np.concatenate([q["z"] for q in parts], axis=3)
    np.testing.assert_allclose(z, ref.z, rtol=0, atol=1e-11)
    np.testing.assert_allclose(parts[0]["D1"], ref.D[0], rtol=0, atol=1e-12)   # block 1 on rank 0
    for q in parts:                                                           # same consensus u
        np.testing.assert_allclose(q["u"], ref.u, rtol=0, atol=1e-13)
