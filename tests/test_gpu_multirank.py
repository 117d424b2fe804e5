"""GPU, 2 ranks sharing the box's one MI355X: the engine's sharded path
(contiguous block shards, owner-of-block-1 logic, per-d-iteration consensus
all-reduce, per-outer broadcast of block 1's filter spectrum, tol norms)
through the C-ABI, with the exchanges carried by the host-staged transport
over gloo.  Must equal the single-rank engine and the oracle.  (8-GPU RCCL runs
are the driver's; RCCL differs only in the transport calls.)"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(variant, big=False):
    rng = np.random.default_rng(99)
    ni, N, psf, K = 2, 3, 5, 3          # 3 blocks over 2 ranks: 2 + 1
    # big: 150 x 149 patches (a 154 x 153 slice past one CU's LDS: the global-pass path)
    sx, sy = (150, 149) if big else (12, 11)
    b = rng.standard_normal((sx, sy, ni * N))
    d0 = rng.standard_normal((psf, psf, K))
    X, Y = sx + 4, sy + 4
    z0 = rng.standard_normal((X, Y, K, ni if variant == "dz" else ni * N))
    return b, d0, z0, ni, N, [psf, psf, K]


def _worker(rank, world, port, out_dir, variant, tol, big):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ccsc_code_iccv2017_amd import learners as E

    def host_comm(op, arr):
        t = torch.from_numpy(arr)        # shares memory with the engine's staging buffer
        if op == 0:
            dist.all_reduce(t)
        else:
            dist.broadcast(t, src=0)

    b, d0, z0, ni, N, ks = _case(variant, big)
    v = E.L.CCSC_DZPAR if variant == "dz" else E.L.CCSC_DPAR
    p = E.make_problem(v, b.shape, ks, 1.0, 1.0, 2, tol, "brief", ni=ni, trace_objective=True)
    ctx = E.Context(0, rank, world, host_comm=host_comm)
    b0, nb = E.shard(E.resolve(p), rank, world)
    bl = b[:, :, b0 * ni:(b0 + nb) * ni]
    zl = z0 if variant == "dz" else z0[..., b0 * ni:(b0 + nb) * ni]
    s = E.Session(ctx, p, bl, d0, zl)
    s.step(2)
    d_res, z_res, DZ, _ = s.results()
    it = s.iterlog()
    np.savez(os.path.join(out_dir, f"{variant}_r{rank}.npz"), d=d_res, z=z_res, DZ=DZ,
             oz=it["trace"]["obj_z"], od=it["trace"]["obj_d"], zd=it["trace"]["z_diff"])
    s.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant,tol,big", [("dz", 0.0, False), ("dp", 1e-12, False),
                                             # global-pass slices: the sharded
                                             # support / d-norm / objective exchanges and the
                                             # session's state handling on that path
                                             ("dz", 0.0, True), ("dp", 1e-3, True)])
def test_two_ranks_equal_one_rank(tmp_path, gpu_ctx, variant, tol, big):
    """Session.step over two ranks (the bench's path) equals the oracle."""
    import torch.multiprocessing as mp
    from ccsc_code_iccv2017_amd import learners as E
    from oracle import ccsc_oracle as O

    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path), variant, tol, big),
                       nprocs=2, join=True, start_method="spawn")
    parts = [np.load(tmp_path / f"{variant}_r{r}.npz") for r in range(2)]
    b, d0, z0, ni, N, ks = _case(variant, big)
    fn = O.learn_2d_dzparallel if variant == "dz" else O.learn_2d_dparallel
    d_o, z_o, DZ_o, it_o, tr_o = fn(b, ks, 1.0, 1.0, 2, tol, "brief", {"d": d0, "z": z0}, ni=ni,
                                    trace_objective=True)
    z = np.concatenate([q["z"] for q in parts], axis=3)
    DZ = np.concatenate([q["DZ"] for q in parts], axis=3)
    for q in parts:   # every rank returns block 1's filters and the global objectives
        np.testing.assert_allclose(q["d"], d_o, rtol=0, atol=1e-9 * np.abs(d_o).max())
        np.testing.assert_allclose(q["oz"], np.array(tr_o["obj_z"]), rtol=1e-9)
        np.testing.assert_allclose(q["od"], np.array(tr_o["obj_d"]), rtol=1e-9)
    np.testing.assert_allclose(z, z_o, rtol=0, atol=1e-9 * np.abs(z_o).max())
    np.testing.assert_allclose(DZ, DZ_o, rtol=0, atol=1e-9 * np.abs(DZ_o).max())
    if tol > 0:
        np.testing.assert_allclose(parts[0]["zd"], np.array(tr_o["z_diff"]), rtol=1e-6)


@pytest.mark.parametrize("variant,tol,nblk", [("dz", 0.0, 3), ("dp", 0.0, 2), ("dz", 1e-12, 2)])
def test_multi_device_context_equals_one_device(gpu_ctx, variant, tol, nblk):
    """ccsc_create_multi({0, 0}) + one ccsc_learn over the whole problem (the MEX path of
    one MATLAB call over several GPUs; a repeated device exchanges through host memory,
    distinct devices through RCCL) gives the one-device result: blocks sharded by
    ccsc_shard, outputs written back at each rank's patch offset, iterlog from rank 0."""
    from ccsc_code_iccv2017_amd import learners as E
    rng = np.random.default_rng(31)
    ni, K, psf = 2, 3, 5
    n = ni * nblk
    b = rng.standard_normal((12, 11, n))
    d0 = rng.standard_normal((psf, psf, K))
    z0 = rng.standard_normal((16, 15, K, ni if variant == "dz" else n))
    fn = (E.admm_learn_conv2D_large_dzParallel if variant == "dz"
          else E.admm_learn_conv2D_large_dParallel)
    args = (b, [psf, psf, K], 1.0, 1.0, 2, tol, "brief", {"d": d0, "z": z0})
    d1, z1, DZ1, it1 = fn(*args, ni=ni, ctx=gpu_ctx)
    mctx = E.Context.multi([0, 0])
    try:
        d2, z2, DZ2, it2 = fn(*args, ni=ni, ctx=mctx)
    finally:
        mctx.close()
    np.testing.assert_allclose(d2, d1, rtol=0, atol=1e-10 * np.abs(d1).max())
    np.testing.assert_allclose(z2, z1, rtol=0, atol=1e-10 * np.abs(z1).max())
    np.testing.assert_allclose(DZ2, DZ1, rtol=0, atol=1e-10 * np.abs(DZ1).max())
    np.testing.assert_allclose(it2["obj_vals_z"], it1["obj_vals_z"], rtol=1e-10)
    if tol > 0:
        np.testing.assert_array_equal(it2["trace"]["n_z"], it1["trace"]["n_z"])


def test_multi_device_context_rejects_sessions(gpu_ctx):
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    mctx = E.Context.multi([0, 0])
    try:
        p = E.make_problem(L.CCSC_DZPAR, (12, 11, 4), [5, 5, 3], 1.0, 1.0, 1, 0.0, "none", ni=2)
        with pytest.raises(L.CCSCError) as ei:
            E.Session(mctx, p, np.zeros((12, 11, 4)))
        assert "one-device context" in str(ei.value)
    finally:
        mctx.close()


def _small_dz(seed=31, nblk=3):
    rng = np.random.default_rng(seed)
    ni, K, psf = 2, 3, 5
    n = ni * nblk
    b = rng.standard_normal((12, 11, n))
    d0 = rng.standard_normal((psf, psf, K))
    z0 = rng.standard_normal((16, 15, K, ni))
    return (b, [psf, psf, K], 1.0, 1.0, 3, 0.0, "brief", {"d": d0, "z": z0}), ni


@pytest.mark.parametrize("fail", ["1:1", "0:0", "1:0"])
def test_failing_rank_aborts_group_and_context_recovers(gpu_ctx, monkeypatch, fail):
    """One rank of a multi-device learn fails (test fault injection, CCSC_TEST_FAIL_RANK
    = rank:outer) while the other is blocked in its next exchange: the call returns that
    rank's error (no hang, no crash), and the SAME context then learns again and
    matches the one-device result -- the MEX keeps its context cached across calls."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    args, ni = _small_dz()
    d1, z1, DZ1, it1 = E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=gpu_ctx)
    mctx = E.Context.multi([0, 0])
    try:
        assert mctx.comm_ranks() == (2, "host")
        monkeypatch.setenv("CCSC_TEST_FAIL_RANK", fail)
        with pytest.raises(L.CCSCError) as ei:
            E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=mctx)
        assert "injected fault" in str(ei.value) and f"rank {fail.split(':')[0]}" in str(ei.value)
        monkeypatch.delenv("CCSC_TEST_FAIL_RANK")
        d2, z2, DZ2, it2 = E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=mctx)
    finally:
        mctx.close()
    np.testing.assert_allclose(d2, d1, rtol=0, atol=1e-10 * np.abs(d1).max())
    np.testing.assert_allclose(z2, z1, rtol=0, atol=1e-10 * np.abs(z1).max())
    np.testing.assert_allclose(it2["obj_vals_z"], it1["obj_vals_z"], rtol=1e-10)


@pytest.mark.parametrize("variant", ["dz", "dp"])
def test_rccl_self_group_executes_and_recovers(gpu_ctx, monkeypatch, variant):
    """The RCCL transport on a one-GPU box: a one-device multi context
    under the test hook CCSC_TEST_RCCL_SELF=1 carries a 1-rank RCCL communicator created
    non-blocking (ncclCommInitRankConfig), and every consensus exchange goes through
    collective(): ncclAllReduce per d-iteration, ncclBroadcast per outer iteration
    (dP:114-121, :143), each polled by wait_comm.  A 1-rank all-reduce and broadcast are
    identities, so the learn must equal the transport-free one bit for bit.  Then an injected
    failure aborts the communicator (abort_group -> ncclCommAbort) and the same context
    re-creates it (reset_group) and learns the same result again."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    args, ni = _small_dz(nblk=3)
    fn = (E.admm_learn_conv2D_large_dzParallel if variant == "dz"
          else E.admm_learn_conv2D_large_dParallel)
    if variant == "dp":
        b, ks, lr, lp, mi, tol, vb, init = args
        rng = np.random.default_rng(5)
        init = {"d": init["d"], "z": rng.standard_normal((16, 15, ks[2], b.shape[2]))}
        args = (b, ks, lr, lp, mi, tol, vb, init)
    d1, z1, DZ1, it1 = fn(*args, ni=ni, ctx=gpu_ctx)
    monkeypatch.setenv("CCSC_TEST_RCCL_SELF", "1")
    mctx = E.Context.multi([0])
    monkeypatch.delenv("CCSC_TEST_RCCL_SELF")
    try:
        assert mctx.comm_ranks() == (1, "rccl")
        d2, z2, DZ2, it2 = fn(*args, ni=ni, ctx=mctx)
        np.testing.assert_array_equal(d2, d1)
        np.testing.assert_array_equal(z2, z1)
        np.testing.assert_array_equal(DZ2, DZ1)
        np.testing.assert_array_equal(it2["obj_vals_z"], it1["obj_vals_z"])
        monkeypatch.setenv("CCSC_TEST_FAIL_RANK", "0:1")
        with pytest.raises(L.CCSCError) as ei:
            fn(*args, ni=ni, ctx=mctx)
        assert "injected fault" in str(ei.value)
        monkeypatch.delenv("CCSC_TEST_FAIL_RANK")
        with pytest.raises(L.CCSCError):
            mctx.comm_ranks()                 # aborted until the next learn re-creates it
        d3, _, _, it3 = fn(*args, ni=ni, ctx=mctx)
        assert mctx.comm_ranks() == (1, "rccl")
        np.testing.assert_array_equal(d3, d1)
        np.testing.assert_array_equal(it3["obj_vals_z"], it1["obj_vals_z"])
    finally:
        mctx.close()


def test_one_rank_context_reports_no_transport(gpu_ctx):
    assert gpu_ctx.comm_ranks() == (1, "none")


def _visible_gpus():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_visible_gpus() < 2", reason="needs >= 2 GPUs (runs on the driver's 8-GPU node)")
def test_distinct_devices_over_rccl_equal_one_device(gpu_ctx):
    """ccsc_create_multi over distinct GPUs: ncclCommInitAll, RCCL all-reduce per
    d-iteration and broadcast per outer iteration (dP:114-121, :143) -- the MATLAB
    drop-in over a node.  ncclCommCount must report every device; the result equals
    the one-device learn; an injected failure on the last rank aborts the
    communicators and the context recovers with fresh ones."""
    from ccsc_code_iccv2017_amd import _lib as L
    from ccsc_code_iccv2017_amd import learners as E
    ndev = min(_visible_gpus(), 8)
    args, ni = _small_dz(nblk=ndev + 1)
    d1, z1, DZ1, it1 = E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=gpu_ctx)
    mctx = E.Context.multi(list(range(ndev)))
    try:
        assert mctx.comm_ranks() == (ndev, "rccl")
        d2, z2, DZ2, it2 = E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=mctx)
        np.testing.assert_allclose(d2, d1, rtol=0, atol=1e-10 * np.abs(d1).max())
        np.testing.assert_allclose(z2, z1, rtol=0, atol=1e-10 * np.abs(z1).max())
        np.testing.assert_allclose(DZ2, DZ1, rtol=0, atol=1e-10 * np.abs(DZ1).max())
        np.testing.assert_allclose(it2["obj_vals_z"], it1["obj_vals_z"], rtol=1e-10)
        os.environ["CCSC_TEST_FAIL_RANK"] = f"{ndev - 1}:1"
        try:
            with pytest.raises(L.CCSCError) as ei:
                E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=mctx)
            assert "injected fault" in str(ei.value)
        finally:
            del os.environ["CCSC_TEST_FAIL_RANK"]
        d3, _, _, _ = E.admm_learn_conv2D_large_dzParallel(*args, ni=ni, ctx=mctx)
        assert mctx.comm_ranks() == (ndev, "rccl")
        np.testing.assert_allclose(d3, d1, rtol=0, atol=1e-10 * np.abs(d1).max())
    finally:
        mctx.close()


def _hs_case():
    rng = np.random.default_rng(77)
    sb, W, psf, K, n = (12, 11), 3, 5, 4, 5      # 5 images over 2 ranks: 3 + 2
    r = psf // 2
    b = rng.random(sb + (W, n))
    sm = 0.5 * rng.random(sb + (W, n))
    init = {"d": rng.standard_normal((psf, psf, K)),
            "z": rng.standard_normal((sb[0] + 2 * r, sb[1] + 2 * r, K, n))}
    return b, sm, init, [psf, psf, W, K]


def _hs_worker(rank, world, port, out_dir, K):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ccsc_code_iccv2017_amd import learners as E

    def host_comm(op, arr):
        t = torch.from_numpy(arr)
        if op == 0:
            dist.all_reduce(t)
        else:
            dist.broadcast(t, src=0)

    b, sm, init, ks = _hs_case()
    ks = ks[:3] + [K]
    d0 = init["d"] if K == 4 else np.random.default_rng(5).standard_normal((ks[0], ks[1], K))
    z0 = init["z"] if K == 4 else np.random.default_rng(6).standard_normal(init["z"].shape[:2] + (K, b.shape[-1]))
    p = E.make_problem(E.L.CCSC_HS23, b.shape, ks, 1.0, 0.2, 3, 0.0, "brief")
    ctx = E.Context(0, rank, world, host_comm=host_comm)
    i0, ni = E.shard(E.resolve(p), rank, world)
    s = E.Session(ctx, p, b[..., i0:i0 + ni], d0, z0[..., i0:i0 + ni], smooth_init=sm[..., i0:i0 + ni])
    done = False
    while s.outer < 3 and not done:
        done = s.step(1)
    d_res, z_res, DZ, obj = s.results(want_obj=True)
    it = s.iterlog()
    np.savez(os.path.join(out_dir, f"hs_r{rank}.npz"), d=d_res, z=z_res, DZ=DZ, obj=obj,
             oz=it["trace"]["obj_z"], od=it["trace"]["obj_d"], i0=i0, ni=ni)
    s.close()
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("K", [4, 100])
def test_hs23_two_ranks_equal_oracle(tmp_path, gpu_ctx, K):
    """The 2-3D learner over two ranks (VERDICT r05 missing item 5; L23's d-solve couples every
    image per frequency, admm_learn.m:289-295): images sharded 3 + 2, each rank's Gram (on the
    matrix cores, gramchol_big.hip) and right-hand sides Z^H xi1 summed over the ranks, the
    objective's sums and max(b) reduced -- equals the oracle on the whole problem."""
    import torch.multiprocessing as mp
    from oracle import ccsc_oracle as O

    mp.start_processes(_hs_worker, args=(2, _free_port(), str(tmp_path), K), nprocs=2, join=True,
                       start_method="spawn")
    parts = [np.load(tmp_path / f"hs_r{r}.npz") for r in range(2)]
    b, sm, init, ks = _hs_case()
    ks = ks[:3] + [K]
    if K != 4:
        init = {"d": np.random.default_rng(5).standard_normal((ks[0], ks[1], K)),
                "z": np.random.default_rng(6).standard_normal(init["z"].shape[:2] + (K, b.shape[-1]))}
    d_o, z_o, Dz_o, obj_o, tr_o = O.learn_hs23(b, ks, 1.0, 0.2, 3, 0.0, "brief", init, sm)
    assert [int(q["ni"]) for q in parts] == [3, 2]
    z = np.concatenate([q["z"] for q in parts], axis=3)
    Dz = np.concatenate([q["DZ"] for q in parts], axis=3)
    for q in parts:
        np.testing.assert_allclose(q["d"], d_o, rtol=0, atol=1e-8 * np.abs(d_o).max())
        assert abs(float(q["obj"]) - obj_o) <= 1e-9 * abs(obj_o)
        for i in range(tr_o["outer"]):
            np.testing.assert_allclose(q["oz"][i], tr_o["obj_z"][i], rtol=1e-9)
            np.testing.assert_allclose(q["od"][i], tr_o["obj_d"][i], rtol=1e-9)
    np.testing.assert_allclose(z, z_o, rtol=0, atol=1e-8 * np.abs(z_o).max())
    np.testing.assert_allclose(Dz, Dz_o, rtol=0, atol=1e-8 * np.abs(Dz_o).max())
