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


def _hs_problem():
    rng = np.random.default_rng(8)
    X, Y, W, K, n = 9, 8, 3, 6, 5          # 5 images over 2 ranks: 3 + 2
    zh = np.fft.fft2(rng.standard_normal((X, Y, 1, K, n)), axes=(0, 1))
    x1 = np.fft.fft2(rng.standard_normal((X, Y, W, n)), axes=(0, 1))
    x2 = np.fft.fft2(rng.standard_normal((X, Y, W, K)), axes=(0, 1))
    return zh, x1, x2, 5000.0


def _hs_worker(rank, world, port, out_dir):
    """The 2-3D learner's rank exchange (engine.cpp SessionHS, dist): each rank forms the
    per-frequency Gram Z_r^H Z_r of its images (+ rho I on rank 0 only) and the right-hand
    sides Z_r^H xi1_r, both summed over the ranks; every rank solves the same system."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    zh, x1, x2, rho = _hs_problem()
    X, Y, W, K, n = zh.shape[0], zh.shape[1], x1.shape[2], zh.shape[3], zh.shape[4]
    base, rem = divmod(n, world)                      # engine.cpp shard(): contiguous images
    nl = base + (1 if rank < rem else 0)
    i0 = rank * base + min(rank, rem)
    Z = zh[:, :, 0, :, i0:i0 + nl].reshape(X * Y, K, nl, order="F").transpose(0, 2, 1)  # [f, p, k]
    ZH = np.conj(Z.transpose(0, 2, 1))                                                  # [f, k, p]
    G = ZH @ Z + (rho * np.eye(K)[None] if rank == 0 else 0.0)
    G = np.broadcast_to(G, (X * Y, K, K))
    h = np.einsum("fkp,fwp->fwk", ZH, x1[:, :, :, i0:i0 + nl].reshape(X * Y, W, nl, order="F"))

    def allreduce(a):
        a = np.ascontiguousarray(a, dtype=np.complex128)
        t = torch.from_numpy(a.view(np.float64).copy())
        dist.all_reduce(t)
        return t.numpy().view(np.complex128).reshape(a.shape)

    G = allreduce(G)
    h = allreduce(h)
    r = h + rho * x2.reshape(X * Y, W, K, order="F")
    out = np.linalg.solve(G[:, None], r[..., None])[..., 0]                             # [f, w, k]
    np.save(os.path.join(out_dir, f"hs_r{rank}.npy"), out.reshape(X, Y, W, K, order="F"))
    dist.barrier()
    dist.destroy_process_group()


def test_hs23_sharded_d_solve_equals_single_process(tmp_path):
    """CPU, world size 2 over gloo: the 2-3D learner's d-solve with images sharded over the
    ranks and the Grams / right-hand sides summed (the engine's multi-rank L23)
    equals the reference's one-process Woodbury/pinv solve (oracle solve_conv_term_D_hs,
    L23:273-300) on every rank."""
    world = 2
    mp.start_processes(_hs_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    from oracle import ccsc_oracle as O
    zh, x1, x2, rho = _hs_problem()
    ref = O.solve_conv_term_D_hs(zh, x1, x2, rho)
    for r in range(world):
        got = np.load(tmp_path / f"hs_r{r}.npy")
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
