"""One-shot xGMI all-reduce kernels (csrc/kernels/xgmi_ar.hip) on ONE MI355X.

Several "ranks" live in this one process: each has its own communicator (buffer, epoch counters, error
word), the buffers are mapped to each other directly (``xgmi_connect_local``) instead of through IPC
handles, and the ranks run as the grid slices of one launch (``*_multi`` ops: separate launches on
separate streams may share a hardware queue and would then wait on each other forever) -- the kernel
protocol (push into every peer's slot, per-(workgroup, source) flags, epoch parity, rank-order reduce)
is exactly the multi-GPU one, with local HBM standing in for the xGMI links.  The two-process IPC path runs end to end in
``test_tp_gpu.py`` (TP=2 engine on one GPU with ``SYMMETRY_XGMI=1``).  Spins are bounded, so a rank
that never arrives shows up as the error word, not a hang.  Reference: fp32 torch sums in rank order.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _comms(ops, world, slot_bytes=1 << 20):
    hs = [int(ops.xgmi_create(slot_bytes, world, r, 0)) for r in range(world)]
    for h in hs:
        ops.xgmi_connect_local(h, hs)
    return hs


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [4096, 8 * 3001, 262144])
def test_xgmi_all_reduce(gpu, world, dtype, n):
    from symmetry_amd.ops import _native

    ops = _native.ops()
    if world * -(-n // 1024) > 1024:
        pytest.skip("the grid slices of one launch would not all be co-resident")
    hs = _comms(ops, world)
    g = torch.Generator(device="cpu").manual_seed(n + world)
    try:
        for it in range(3):  # consecutive collectives alternate the slot parity
            xs = [torch.randn(n, generator=g).to(gpu, dtype) for _ in range(world)]
            outs = [torch.full_like(x, float("nan")) for x in xs]
            ops.xgmi_all_reduce_multi(xs, outs, hs)
            torch.cuda.synchronize()
            ref = torch.zeros(n, dtype=torch.float32, device=gpu)
            for x in xs:
                ref += x.float()
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                torch.testing.assert_close(outs[r].float(), ref.to(dtype).float(), rtol=0, atol=0)
                assert torch.equal(outs[r], outs[0])  # every rank bit-identical
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("T,d,P", [(1, 4096, 8), (4, 8192, 8), (10, 4096, 1), (64, 4096, 4)])
def test_xgmi_add_prep(gpu, world, T, d, P):
    from symmetry_amd.ops import _native, reference

    ops = _native.ops()
    if world * T * P > 1024:
        pytest.skip("the grid slices of one launch would not all be co-resident")
    hs = _comms(ops, world, slot_bytes=T * d * 4 + 256)
    g = torch.Generator(device="cpu").manual_seed(T * d + P)
    try:
        w = (torch.rand(d, generator=g) + 0.5).to(gpu, torch.bfloat16)
        resid0 = torch.randn(T, d, generator=g).to(gpu)
        for it in range(2):
            ys = [torch.randn(T, d, generator=g).to(gpu) for _ in range(world)]
            resids = [resid0.clone() for _ in range(world)]
            xws = [torch.empty(T, d, dtype=torch.bfloat16, device=gpu) for _ in range(world)]
            sss = [torch.empty(T, P, dtype=torch.float32, device=gpu) for _ in range(world)]
            ops.xgmi_add_prep_multi(ys, resids, w, xws, sss, hs)
            torch.cuda.synchronize()
            ysum = torch.zeros(T, d, device=gpu)
            for y in ys:
                ysum += y
            r_ref, xw_ref, ss_ref = resid0.clone(), torch.empty_like(xws[0]), torch.empty_like(sss[0])
            reference.add_prep(ysum, r_ref, w, xw_ref, ss_ref)
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                torch.testing.assert_close(resids[r], r_ref, rtol=0, atol=0)
                torch.testing.assert_close(xws[r].float(), xw_ref.float(), rtol=1e-2, atol=1e-2)
                torch.testing.assert_close(sss[r], ss_ref, rtol=1e-4, atol=1e-3)
                assert torch.equal(resids[r], resids[0]) and torch.equal(sss[r], sss[0])
            resid0 = resids[0].clone()
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


def test_xgmi_all_reduce_graph_replay(gpu):
    """Captured once, replayed: the device-side epoch counters keep the ranks in step."""
    from symmetry_amd.ops import _native

    ops = _native.ops()
    world, n = 2, 8192
    hs = _comms(ops, world)
    try:
        xs = [torch.zeros(n, device=gpu) for _ in range(world)]
        outs = [torch.zeros(n, device=gpu) for _ in range(world)]
        ops.xgmi_all_reduce_multi(xs, outs, hs)  # warm (epoch 1)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):  # capture only: nothing runs
            ops.xgmi_all_reduce_multi(xs, outs, hs)
            ops.xgmi_all_reduce_multi(outs, outs, hs)
        for it in range(4):
            for r in range(world):
                xs[r].fill_(float(10 * it + r + 1))
            graph.replay()
            torch.cuda.synchronize()
            expect = world * sum(float(10 * it + r + 1) for r in range(world))
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                assert torch.all(outs[r] == expect), (it, r, outs[r][:4].tolist(), expect)
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


def test_xgmi_rejects_oversized_and_bad_shapes(gpu):
    from symmetry_amd.ops import _native

    ops = _native.ops()
    h = int(ops.xgmi_create(4096, 1, 0, 0))
    try:
        with pytest.raises(RuntimeError):
            ops.xgmi_all_reduce(torch.zeros(4096, device=gpu), torch.zeros(4096, device=gpu), h)  # not connected
        ops.xgmi_connect_local(h, [h])
        with pytest.raises(RuntimeError):
            ops.xgmi_all_reduce(torch.zeros(2048, device=gpu), torch.zeros(2048, device=gpu), h)  # 8 KB > slot
        with pytest.raises(RuntimeError):
            ops.xgmi_all_reduce(torch.zeros(12, device=gpu), torch.zeros(12, device=gpu), h)  # n % 8
        x = torch.arange(1024, dtype=torch.float32, device=gpu)
        out = torch.empty_like(x)
        ops.xgmi_all_reduce(x, out, h)  # world 1: a copy
        torch.cuda.synchronize()
        assert torch.equal(out, x) and ops.xgmi_error(h) == 0
        keys = (torch.arange(5, dtype=torch.int64, device=gpu) << 32) | (0xFFFFFFFF - torch.arange(5, device=gpu) * 7)
        ids = torch.zeros(5, dtype=torch.int32, device=gpu)
        ops.xgmi_keys_max(keys, ids, h)  # world 1: unpack the own keys
        torch.cuda.synchronize()
        assert ids.tolist() == [0, 7, 14, 21, 28] and ops.xgmi_error(h) == 0
    finally:
        ops.xgmi_destroy(h)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_xgmi_mixed_geometry_with_slow_rank(gpu, world):
    """The decode sequence of a TP layer stack, every collective with a different workgroup split of the same
    slot bytes -- add_prep with 8 parts per row, add_prep with 4 parts, the sampling keys (one workgroup at
    byte 0), a plain chunked all-reduce -- repeated, with one rank's slice held back 50 us before it pushes
    (rotating).  The per-communicator collective counter keeps every collective on its own slot parity
    whatever the split (the per-workgroup epochs of round 2 could alias them); results are bit-exact."""
    from symmetry_amd.ops import _native, reference

    ops = _native.ops()
    d = 4096
    hs = _comms(ops, world, slot_bytes=24 * d * 4 + 256)
    g = torch.Generator(device="cpu").manual_seed(world)
    w = (torch.rand(d, generator=g) + 0.5).to(gpu, torch.bfloat16)
    try:
        for it in range(4):
            slow = it % world
            for T, P in ((4, 8), (24, 4)):
                ys = [torch.randn(T, d, generator=g).to(gpu) for _ in range(world)]
                r0 = torch.randn(T, d, generator=g).to(gpu)
                resids = [r0.clone() for _ in range(world)]
                xws = [torch.empty(T, d, dtype=torch.bfloat16, device=gpu) for _ in range(world)]
                sss = [torch.empty(T, P, dtype=torch.float32, device=gpu) for _ in range(world)]
                ops.xgmi_add_prep_multi(ys, resids, w, xws, sss, hs, slow, 50)
                ysum = torch.zeros(T, d, device=gpu)
                for y in ys:
                    ysum += y
                r_ref, xw_ref, ss_ref = r0.clone(), torch.empty_like(xws[0]), torch.empty_like(sss[0])
                reference.add_prep(ysum, r_ref, w, xw_ref, ss_ref)
                torch.cuda.synchronize()
                for r in range(world):
                    torch.testing.assert_close(resids[r], r_ref, rtol=0, atol=0)
                    assert torch.equal(resids[r], resids[0]) and torch.equal(sss[r], sss[0])
            B = 10
            vals = [torch.randint(0, 1 << 30, (B,), generator=g) for _ in range(world)]
            idx = [torch.randint(0, 1 << 20, (B,), generator=g) for _ in range(world)]
            keys = [((v << 32) | (0xFFFFFFFF - i)).to(gpu) for v, i in zip(vals, idx)]
            ids = [torch.full((B,), -1, dtype=torch.int32, device=gpu) for _ in range(world)]
            ops.xgmi_keys_max_multi(keys, ids, hs, (slow + 1) % world, 50)
            stacked = torch.stack([k.cpu() for k in keys])
            best = stacked.max(0).values
            expect = (0xFFFFFFFF - (best & 0xFFFFFFFF)).to(torch.int32)
            n = 32 * 1024
            xs = [torch.randn(n, generator=g).to(gpu) for _ in range(world)]
            outs = [torch.empty_like(x) for x in xs]
            ops.xgmi_all_reduce_multi(xs, outs, hs, slow, 50)
            ref = torch.zeros(n, device=gpu)
            for x in xs:
                ref += x
            torch.cuda.synchronize()
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                assert torch.equal(ids[r].cpu(), expect), (it, r)
                torch.testing.assert_close(outs[r], ref, rtol=0, atol=0)
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


def test_xgmi_declared_fault_stops_every_wait(gpu):
    """Fault containment: rank 1 of a world-2 communicator never runs.  (a) A collective already spinning on it
    ends promptly once the host declares the fault (``xgmi_set_error``, what rank 0's health monitor does), not
    after the 30 s wait limit; (b) with the word set, 200 further collectives -- a captured 70B TP=8 step holds
    161 -- finish at once instead of waiting 30 s EACH.  The word is sticky (the communicator stays failed)."""
    import time

    from symmetry_amd.ops import _native

    ops = _native.ops()
    hs = _comms(ops, 2)
    x = torch.randn(8192, device=gpu)
    try:
        t0 = time.perf_counter()
        ops.xgmi_all_reduce(x, x, hs[0])  # waits for rank 1's flag
        time.sleep(0.3)
        ops.xgmi_set_error(hs[0], 2)
        torch.cuda.synchronize()
        first = time.perf_counter() - t0
        assert first < 5.0, first
        t1 = time.perf_counter()
        for _ in range(100):
            ops.xgmi_all_reduce(x, x, hs[0])
            ops.xgmi_keys_max(torch.zeros(4, dtype=torch.int64, device=gpu),
                              torch.zeros(4, dtype=torch.int32, device=gpu), hs[0])
        torch.cuda.synchronize()
        rest = time.perf_counter() - t1
        assert rest < 5.0, rest
        assert ops.xgmi_error(hs[0]) == 2 and ops.xgmi_error(hs[0]) == 2  # sticky
    finally:
        ops.xgmi_set_error(hs[0], 0)
        for h in hs:
            ops.xgmi_destroy(h)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_xgmi_a2a_unpadded_exchange(gpu, world, dtype):
    """R3 expert all-to-all (xgmi_a2a): every rank sends block q (rows [q cap, q cap + counts[q]), counts only on
    the device) to rank q, which receives it as block `source`; side ints (expert ids) travel with the rows and
    read -1 past each block's count; rows past the count are never written (only routed rows cross the links).
    Four rounds (both slot parities, twice), a rotating rank held back 30 us."""
    from symmetry_amd.ops import _native

    ops = _native.ops()
    cap, d = 40, 256
    esz = torch.finfo(dtype).bits // 8
    slot = (int(ops.xgmi_a2a_slot(cap, d * esz)) + 255) // 256 * 256
    hs = _comms(ops, world, slot_bytes=slot)
    g = torch.Generator(device="cpu").manual_seed(world * 10 + esz)
    try:
        for it in range(4):
            cnt = torch.randint(0, cap + 1, (world, world), generator=g, dtype=torch.int32)
            cnt[0, world - 1] = cap  # a full block
            cnt[world - 1, 0] = 0    # an empty one
            srcs = [torch.randn(world * cap, d, generator=g).to(gpu, dtype) for _ in range(world)]
            sides = [torch.randint(0, 1 << 20, (world * cap,), generator=g, dtype=torch.int32).to(gpu)
                     for _ in range(world)]
            counts = [cnt[r].to(gpu) for r in range(world)]
            dsts = [torch.full((world * cap, d), float("nan"), device=gpu, dtype=dtype) for _ in range(world)]
            dsides = [torch.full((world * cap,), -7, dtype=torch.int32, device=gpu) for _ in range(world)]
            dcnts = [torch.full((world,), -7, dtype=torch.int32, device=gpu) for _ in range(world)]
            ops.xgmi_a2a_multi(srcs, counts, sides, dsts, dsides, dcnts, cap, hs, it % world, 30)
            torch.cuda.synchronize()
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                assert dcnts[r].tolist() == cnt[:, r].tolist()
                for s in range(world):
                    n = int(cnt[s, r])
                    got, want = dsts[r][s * cap:(s + 1) * cap], srcs[s][r * cap:r * cap + n]
                    assert torch.equal(got[:n], want), (r, s, n)
                    assert torch.isnan(got[n:].float()).all(), (r, s, n)  # nothing past the count was written
                    gs = dsides[r][s * cap:(s + 1) * cap]
                    assert torch.equal(gs[:n], sides[s][r * cap:r * cap + n]) and (gs[n:] == -1).all()
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("M", [1, 10, 16])
@pytest.mark.parametrize("form", ["gemm8", "gemm4", "xres", "gemm8_shuf"])
def test_xgmi_gemm_all_reduce_resid_one_launch(gpu, world, M, form):
    """Row-parallel decode projection + xGMI all-reduce + residual add + next-norm prep as ONE launch
    (DECODE_EPI_XAR): every workgroup pushes its fp32 tiles into every rank's slot, waits for the other ranks'
    copies of the same tiles, sums them in rank order and runs the residual epilogue.  All ranks in one launch
    (grid z = rank).  fp32 torch reference; every rank bit-identical; twice (both slot parities)."""
    from symmetry_amd.models.layout import preshuffle
    from symmetry_amd.ops import _native

    ops = _native.ops()
    N, K = {"gemm8": (1024, 512), "gemm4": (1024, 1792), "xres": (2048, 1024), "gemm8_shuf": (1024, 512)}[form]
    if world == 8 and form.startswith("gemm8"):
        # all 8 ranks' grids share this one GPU: 8 x 64 512-thread workgroups are not co-resident, 8 x 32 are (on 8
        # GPUs each rank's grid has a GPU of its own: the TP = 8 o projection is N = 4096, K = 512 per rank)
        N = 512
    shuf = form in ("xres", "gemm8_shuf")
    hs = _comms(ops, world, slot_bytes=16 * N * 8 + 256)
    g = torch.Generator(device="cpu").manual_seed(M * 31 + world)
    try:
        for it in range(2):
            W = (torch.randn(N, K, generator=g) * K ** -0.5).to(gpu, torch.bfloat16)
            Wk = preshuffle(W) if shuf else W
            wn = (torch.rand(N, generator=g) + 0.5).to(gpu, torch.bfloat16)
            xs = [torch.randn(M, K, generator=g).to(gpu, torch.bfloat16) for _ in range(world)]
            r0 = torch.randn(M, N, generator=g).to(gpu)
            resids = [r0.clone() for _ in range(world)]
            xws = [torch.empty(M, N, dtype=torch.bfloat16, device=gpu) for _ in range(world)]
            sss = [torch.empty(M, N // 16, device=gpu) for _ in range(world)]
            ok = ops.xgmi_gemm_ar_resid_multi(xs, Wk, shuf, resids, wn, xws, sss, hs, form == "xres")
            if not ok:
                pytest.skip("grid not co-resident for this world size")
            torch.cuda.synchronize()
            ysum = sum(x.float() @ W.float().t() for x in xs)
            r_ref = r0 + ysum
            for r in range(world):
                assert ops.xgmi_error(hs[r]) == 0
                torch.testing.assert_close(resids[r], r_ref, rtol=2e-3, atol=2e-3)
                assert torch.equal(resids[r], resids[0]) and torch.equal(sss[r], sss[0])
                torch.testing.assert_close(xws[r].float(), (resids[r] * wn.float()).bfloat16().float(), rtol=0, atol=0)
                torch.testing.assert_close(sss[r], (resids[r] ** 2).view(M, N // 16, 16).sum(-1), rtol=1e-5, atol=1e-4)
    finally:
        for h in hs:
            ops.xgmi_destroy(h)


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("xres", [False, True])
def test_xgmi_gemm_ar_resid_skewed_alternating(gpu, world, xres):
    """The default 8-GPU decode path's fused launches as a decode step issues them: o-shaped and down-shaped
    row-parallel projections alternating on ONE communicator (they share its per-output-tile epoch counters,
    N = d for both), 6 consecutive launches (both slot parities, three times), a rotating rank held back 40 us
    before its workgroups start.  Each launch's residual feeds the next (a stale or mixed-epoch granule shows
    up as a wrong sum downstream); every rank bit-identical; fp32 torch reference per launch."""
    from symmetry_amd.models.layout import preshuffle
    from symmetry_amd.ops import _native

    ops = _native.ops()
    N = 512 if world == 8 and not xres else 1024  # 8 ranks' 512-thread grids on one GPU: 8 x 32 fit, 8 x 64 do not
    # (K, preshuffled) of the o- and down-shaped calls: the x-resident walk needs K % 1024 == 0 and preshuffled W
    shapes = [(1024, True), (2048, True)] if xres else [(512, False), (1792, False)]
    M = 4
    hs = _comms(ops, world, slot_bytes=16 * N * 8 + 256)
    g = torch.Generator(device="cpu").manual_seed(world * 7 + int(xres))
    try:
        wn = (torch.rand(N, generator=g) + 0.5).to(gpu, torch.bfloat16)
        r = torch.randn(M, N, generator=g).to(gpu)
        resids = [r.clone() for _ in range(world)]
        for it in range(6):
            K, shuf = shapes[it % 2]
            W = (torch.randn(N, K, generator=g) * K ** -0.5).to(gpu, torch.bfloat16)
            xs = [torch.randn(M, K, generator=g).to(gpu, torch.bfloat16) for _ in range(world)]
            xws = [torch.empty(M, N, dtype=torch.bfloat16, device=gpu) for _ in range(world)]
            sss = [torch.empty(M, N // 16, device=gpu) for _ in range(world)]
            before = resids[0].clone()
            ok = ops.xgmi_gemm_ar_resid_multi(xs, preshuffle(W) if shuf else W, shuf, resids, wn, xws, sss, hs, xres,
                                              it % world, 40)
            if not ok:
                pytest.skip("grid not co-resident for this world size")
            torch.cuda.synchronize()
            want = before + sum(x.float() @ W.float().t() for x in xs)
            for q in range(world):
                assert ops.xgmi_error(hs[q]) == 0, (it, q)
                torch.testing.assert_close(resids[q], want, rtol=2e-3, atol=2e-3)
                assert torch.equal(resids[q], resids[0]) and torch.equal(sss[q], sss[0]), (it, q)
    finally:
        for h in hs:
            ops.xgmi_destroy(h)
