"""Multi-GPU pieces of the path: one process per GPU, torch.distributed over RCCL.

The reference has no distributed code; these are the two exchanges
the path actually needs:

* ``all_gather_rows`` — the per-epoch global OT (MRI_PET_OT_OT_per_epoch_attn.py:940-960)
  extracts features per data-parallel shard; one all-gather gives every rank the
  full (N x d) embedding set and labels before the solve.
* ``sharded_feature_cost`` — for a sample coupling Ts that is block-diagonal along
  the shards (Ts = I/B per batch, MRI_PET_OT_nojax.py:688), the feature cost
  decomposes as M = sum_r (t1_r + t2_r - 2 X_r^T Ts_r Y_r): ONE all-reduce(SUM)
  of the d x d2 float64 partials (1 MiB at d = 512... 32 MiB at d = 2048) replaces
  gathering the embeddings.  The Sinkhorn solve is then replicated (it is tiny).

* ``sinkhorn_row_sharded`` — ONE large coupled problem (BASELINE config 5) with the
  cost rows split over the ranks: per iteration the only exchange is an
  all-reduce(SUM) of the column sums K^T u (m + 1 values incl. the break count);
  every rank then takes the same stop / break decisions.  ``coupled_solve_sharded``
  is the whole per-epoch pipeline: all-gather the PET embedding shards, build this
  rank's cost rows, agree on the global max, solve.

Independent problems (per-rank minibatches / labels) need no collective at all;
bench.py scales that way ("weak", replicas).
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _lib as L
from . import ops


def all_gather_rows(local: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate every rank's (n_r, ...) tensor along dim 0 in rank order.
    Unequal n_r are padded to the max for the collective and trimmed after."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    nmax = max(sizes)
    pad = local.new_zeros((nmax,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = local
    out = local.new_empty((world * nmax,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, pad.contiguous(), group=group)
    return torch.cat([out[r * nmax: r * nmax + sizes[r]] for r in range(world)])


def _local_feature_cost(X, Y, Ts=None, ts_diag=None, weights="pot"):
    return ops.feature_cost(X, Y, Ts=Ts, ts_diag=ts_diag, weights=weights)


def sharded_feature_cost(X_local: torch.Tensor, Y_local: torch.Tensor, Ts_local=None,
                         ts_diag_local=None, weights: str = "pot", group=None) -> torch.Tensor:
    """Global feature cost from per-rank shards with block-diagonal Ts (one all-reduce)."""
    M = _local_feature_cost(X_local, Y_local, Ts=Ts_local, ts_diag=ts_diag_local, weights=weights)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(M, op=dist.ReduceOp.SUM, group=group)
    return M


def sharded_batch_feature_plan(mri_local: torch.Tensor, pet_local: torch.Tensor, global_batch: int,
                               eps: float = 1e-2, numItermax: int = 2000, stopThr: float = 1e-9,
                               group=None):
    """Per-batch PET->MRI feature plan of a data-parallel batch sharded over ranks:
    Ts = I / B_global restricted to the local rows, one all-reduce, replicated solve."""
    B = mri_local.shape[0]
    ts = torch.full((B,), 1.0 / global_batch, dtype=torch.float64, device=mri_local.device)
    M = sharded_feature_cost(mri_local.detach(), pet_local.detach(), ts_diag_local=ts, group=group)
    d, d2 = M.shape
    a = torch.full((d,), 1.0 / d, dtype=torch.float64, device=M.device)
    b = torch.full((d2,), 1.0 / d2, dtype=torch.float64, device=M.device)
    res = ops.sinkhorn(a, b, M, float(eps), max_iter=numItermax, stop_thr=stopThr, flavor="pot",
                       sync_every=0, want_plan=True)  # no host poll in the loop
    return res.plan, res


def gather_epoch_features(mri_local: torch.Tensor, pet_local: torch.Tensor,
                          labels_local: torch.Tensor, group=None):
    """All-gather the per-shard backbone features and labels of one epoch
    (feature_extract, MRI_PET_OT_OT_per_epoch_attn.py:889-912, run data-parallel)."""
    return (all_gather_rows(mri_local, group), all_gather_rows(pet_local, group),
            all_gather_rows(labels_local, group))


# --------------------------------------------------------------------------- per-epoch label split
def split_label_plans(pets, mris, comm, solve):
    """The per-label sample couplings of one epoch (get_coupling_egw_ott_fixed,
    MRI_PET_OT_OT_per_epoch_attn.py:954: one independent entropic GW per label) with the
    labels dealt over the ranks: rank r solves labels r, r + W, r + 2W, ... (``solve(pets,
    mris) -> (plans, result)`` on its share) and ONE all-reduce(SUM) of an L x P x P
    float64 buffer (P = the largest group, zeros where a rank does not own the label)
    gives every rank every plan.  Each plan has exactly one nonzero contribution, so the
    sum reproduces this rank's solve of it bit for bit.  That solve equals the unsplit
    one bit for bit when the share takes the same GW kernel form as the whole batch
    (otf_gw.hip gw_launch picks the small-problem kernel only when EVERY group of a
    launch has <= 64 samples, as with the reference's --max-jax-samples 64); when the
    groups straddle 64 a rank's share can take the other form and its plans agree with
    the unsplit solve to rounding (same algorithm and iterates, different reduction
    order).  Returns ``(plans, result of this rank's solve or None)``."""
    L = len(pets)
    world, rank = comm.nranks, comm.rank
    own = list(range(rank, L, world))
    sizes = [(int(p.shape[0]), int(m.shape[0])) for p, m in zip(pets, mris)]
    P = max(max(a, b) for a, b in sizes) if sizes else 0
    dev = pets[0].device if pets else torch.device("cpu")
    buf = torch.zeros((L, P, P), dtype=torch.float64, device=dev)
    res = None
    if own:
        plans_own, res = solve([pets[k] for k in own], [mris[k] for k in own])
        for k, T in zip(own, plans_own):
            buf[k, : T.shape[0], : T.shape[1]] = T
    comm.all_reduce(buf)
    return [buf[k, : sizes[k][0], : sizes[k][1]] for k in range(L)], res


def per_epoch_coupling_split(mri: torch.Tensor, pet: torch.Tensor, labels: torch.Tensor, comm,
                             eps: float = 5e-3, max_per_label: int | None = 64, **kw):
    """``compute_pet_to_mri_coupling`` (MRI_PET_OT_OT_per_epoch_attn.py:940-960) of the
    all-gathered epoch features with the per-label GW work split over the ranks
    (``split_label_plans``).  The feature stage after it -- the 2048 x 2048 fot cost from
    all plans (a ~0.5 GFLOP float64 GEMM pair) and its OTT solve -- stays replicated: it is
    one latency-bound resident launch (~1 ms), where a row-sharded solve would add one
    cross-rank all-reduce per Sinkhorn iteration and an all-reduce of the 32 MiB cost
    partials would cost more than building the cost.  Returns ``(Tv, info)``."""
    from .perturbot import per_epoch_coupling_device
    return per_epoch_coupling_device(mri, pet, labels, eps=eps, max_per_label=max_per_label,
                                     comm=comm, **kw)


# --------------------------------------------------------------------------- row-sharded solve
class DevicePasses:
    """HIP backend of ``sinkhorn_row_sharded``: otf_sinkhorn_pass / otf_sinkhorn_finish
    on this rank's rows (include/otfuse.h)."""

    def __init__(self, a_local, b, C_local, reg, max_iter, stop_thr, cost_scale, n_total,
                 check_every=10, err_squared=False):
        ops._dev(C_local, "C_local")
        if C_local.dtype not in ops._VEC:
            raise TypeError("C_local must be float16, float32 or float64")
        self.cost_f16 = C_local.dtype == torch.float16
        self.dt = torch.float32 if self.cost_f16 else C_local.dtype
        self.n, self.m = C_local.shape
        self.C = ops._rowmajor(C_local, ops._VEC[C_local.dtype])
        self.a = a_local.to(self.C.device, self.dt).contiguous()
        self.b = b.to(self.C.device, self.dt).contiguous()
        if self.a.numel() != self.n or self.b.numel() != self.m:
            raise ValueError("a_local / b do not match C_local")
        self.cost_scale = None if cost_scale is None else cost_scale.to(self.dt).contiguous()
        dev = self.C.device
        self.ws = ops.sinkhorn_workspace(self.n, self.m, self.dt, max_iter, dev)
        self.info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=dev)
        self.errlog = torch.zeros(max_iter // max(check_every, 1) + 2, dtype=torch.float64, device=dev)
        self.opts = L.SinkhornOpts(reg=float(reg), stop_thr=float(stop_thr), max_iter=int(max_iter),
                                   check_every=int(check_every), flavor=L.OTF_FLAVOR_POT,
                                   err_squared=int(err_squared), sync_every=0,
                                   engine=L.ENGINE_STREAM, cost_f16=int(self.cost_f16),
                                   n_total=int(n_total))
        self._esz = torch.empty((), dtype=self.dt).element_size()

    def _common(self):
        return (self.a.data_ptr(), self.b.data_ptr(), self.C.data_ptr(), self.n, self.m,
                self.C.stride(0), ops._DT[self.dt], L.ptr(self.cost_scale))

    def run_pass(self, p: int) -> torch.Tensor:
        """Enqueue pass p; returns the (m_pad + 1) column-sum buffer to all-reduce."""
        ptr = ctypes.c_void_p()
        ln = ctypes.c_int64()
        L.check(L.lib().otf_sinkhorn_pass(
            *self._common(), ctypes.byref(self.opts), int(p), self.info.data_ptr(),
            self.errlog.data_ptr(), self.ws.data_ptr(), self.ws.numel(), ctypes.byref(ptr),
            ctypes.byref(ln), L.stream_handle(self.C.device)), "otf_sinkhorn_pass")
        off = ptr.value - self.ws.data_ptr()
        return self.ws[off: off + ln.value * self._esz].view(self.dt)

    def stopped(self) -> bool:
        return bool(self.info[0].item())

    def _outputs(self, want_plan, plan_dtype):
        dev = self.C.device
        u = torch.empty(self.n, dtype=self.dt, device=dev)
        v = torch.empty(self.m, dtype=self.dt, device=dev)
        P = ops._alloc_rowmajor(self.n, self.m, plan_dtype or self.dt, dev, 4) if want_plan else None
        return u, v, P

    def solve_with_comm(self, comm, want_plan=True, plan_dtype=None) -> ops.SinkhornResult:
        """Every pass + its RCCL all-reduce + the finish in ONE C call
        (otf_sinkhorn_row_sharded): no Python / host round trip per iteration."""
        u, v, P = self._outputs(want_plan, plan_dtype)
        L.check(L.lib().otf_sinkhorn_row_sharded(
            *self._common(), ctypes.byref(self.opts), comm.handle if comm is not None else None,
            u.data_ptr(), v.data_ptr(), L.ptr(P), P.stride(0) if P is not None else 0,
            ops._DT[P.dtype] if P is not None else 0, self.info.data_ptr(), self.errlog.data_ptr(),
            self.ws.data_ptr(), self.ws.numel(), L.stream_handle(self.C.device)),
            "otf_sinkhorn_row_sharded")
        return ops.SinkhornResult(u=u, v=v, plan=P, info_dev=self.info, errlog_dev=self.errlog)

    def finish(self, want_plan=True, plan_dtype=None) -> ops.SinkhornResult:
        dev = self.C.device
        u, v, P = self._outputs(want_plan, plan_dtype)
        L.check(L.lib().otf_sinkhorn_finish(
            *self._common(), ctypes.byref(self.opts), u.data_ptr(), v.data_ptr(), L.ptr(P),
            P.stride(0) if P is not None else 0, ops._DT[P.dtype] if P is not None else 0,
            self.info.data_ptr(), self.errlog.data_ptr(), self.ws.data_ptr(), self.ws.numel(),
            L.stream_handle(dev)), "otf_sinkhorn_finish")
        return ops.SinkhornResult(u=u, v=v, plan=P, info_dev=self.info, errlog_dev=self.errlog)


def sinkhorn_row_sharded(a_local: torch.Tensor, b: torch.Tensor, C_local: torch.Tensor, reg: float,
                         max_iter: int = 1000, stop_thr: float = 1e-9,
                         cost_scale: torch.Tensor | None = None, n_total: int | None = None,
                         check_every: int = 10, err_squared: bool = False, sync_every: int = 0,
                         want_plan: bool = True, plan_dtype=None, group=None, backend=None,
                         comm=None):
    """POT ``sinkhorn_knopp`` on a problem whose cost rows are split over the ranks.

    Rank r passes its rows ``C_local`` (n_r x m), ``a_local = a[R_r]`` and the full
    ``b``; the result holds this rank's rows of u and of the plan, and the full v.
    One all-reduce(SUM) of m + 1 values per iteration.  With an RCCL
    ``comm`` (otfuse.comm.Communicator) the whole loop is one C call and the
    all-reduces are RCCL kernels on the same stream; otherwise the passes are
    driven from Python over torch.distributed (any backend; gloo in the CPU tests).
    With ``sync_every`` > 0 the host polls the (rank-identical) stop flag to end early.
    """
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if n_total is None:
        n_total = C_local.shape[0]
        if world > 1:
            t = torch.tensor([n_total], dtype=torch.int64, device=C_local.device)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            n_total = int(t.item())
    be = (backend or DevicePasses)(a_local, b, C_local, reg, max_iter, stop_thr, cost_scale,
                                   n_total, check_every, err_squared)
    if comm is not None and isinstance(be, DevicePasses) and sync_every == 0:
        return be.solve_with_comm(comm, want_plan, plan_dtype)
    for p in range(max_iter + 1):
        cs = be.run_pass(p)
        if world > 1:
            dist.all_reduce(cs, op=dist.ReduceOp.SUM, group=group)
        if sync_every > 0 and p >= 1 and p % sync_every == 0 and p < max_iter and be.stopped():
            break
    return be.finish(want_plan, plan_dtype)


class XPeer:
    """One rank's side of the in-kernel cross-rank exchange (``otf_xpeer_*``): an
    exchange buffer on this GPU that every rank's persistent sweep writes its column-sum
    partials into over xGMI, and the peers' buffers mapped here (IPC handles exchanged
    once through ``torch.distributed``, any backend).  Every rank must make the same
    sequence of ``sinkhorn_xsweep`` calls on it."""

    def __init__(self, m: int, group=None):
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self._group = group
        self.m = int(m)
        lib = L.lib()
        hs = int(lib.otf_xpeer_handle_size())
        h = (ctypes.c_ubyte * hs)()
        ptr = ctypes.c_void_p()
        L.check(lib.otf_xpeer_create(self.rank, self.world, self.m, ctypes.byref(ptr), h),
                "otf_xpeer_create")
        self._h = ptr
        mine = bytes(h)
        if self.world > 1:
            allh = [None] * self.world
            dist.all_gather_object(allh, mine, group=group)
        else:
            allh = [mine]
        buf = b"".join(allh)
        rc = lib.otf_xpeer_connect(self._h, buf)
        if rc != 0:
            lib.otf_xpeer_destroy(self._h)
            self._h = None
            L.check(rc, "otf_xpeer_connect")

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("XPeer is closed")
        return self._h

    def close(self):
        """Collective over the exchange's group (the one it was built on): every member
        must call it after its last solve on this exchange.  The device is synchronised
        (this rank's grids are done) and the members meet at a barrier of that group
        (every peer's grids are done storing into this rank's buffer) before the buffer is
        freed; a one-member exchange has no peer and skips the barrier."""
        if self._h is not None:
            torch.cuda.synchronize()
            if self.world > 1 and dist.is_available() and dist.is_initialized():
                dist.barrier(group=self._group)
            L.lib().otf_xpeer_destroy(self._h)
            self._h = None

    def __del__(self):  # noqa: D105
        # garbage collection is not collective: free without the barrier only if the
        # caller never closed it (the device sync in otf_xpeer_destroy still runs)
        try:
            if self._h is not None:
                L.lib().otf_xpeer_destroy(self._h)
                self._h = None
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def xsweep_engine(engine: str, n_local: int, world: int, group=None) -> str:
    """The cross-rank engine every rank of the exchange takes: the shard row
    counts are all-gathered over the group; with unequal shards "auto" becomes "sweep" on
    every rank and "mesh" is refused on every rank (the same exception everywhere, so no
    rank is left waiting on the exchange).  Equal shards keep the request, and the library
    then decides from (n, m, device), which are the same on every rank."""
    if engine == "sweep" or world <= 1:
        return engine
    sizes = [None] * world
    dist.all_gather_object(sizes, int(n_local), group=group)
    if len(set(sizes)) == 1:
        return engine
    if engine == "mesh":
        raise ValueError(f"engine='mesh' needs equal row shards over the ranks, got {sizes}")
    return "sweep"


def sinkhorn_xsweep(a_local: torch.Tensor, b: torch.Tensor, C_local: torch.Tensor, reg: float,
                    xpeer: XPeer, n_total: int, max_iter: int = 1000, stop_thr: float = 1e-9,
                    cost_scale: torch.Tensor | None = None, check_every: int = 10,
                    err_squared: bool = False, want_plan: bool = True, plan_dtype=None,
                    workspace: torch.Tensor | None = None, engine: str = "auto") -> ops.SinkhornResult:
    """POT ``sinkhorn_knopp`` on a problem whose cost rows are split over the ranks, as
    ONE persistent launch per rank (``otf_sinkhorn_xsweep``): the column sums are
    exchanged inside the launch through ``xpeer`` -- no all-reduce call per iteration.
    Same contract as ``sinkhorn_row_sharded`` (this rank's rows of u and the plan, the
    full v); float32 compute, fp32 or fp16 cost rows.

    ``engine``: "mesh" keeps this rank's K in the register files for the whole solve
    (whole 512-column tiles, one workgroup per 128 x 512 tile on the device; the mesh's
    reducers exchange their column-sum partials, "xmesh"), "sweep" streams the cost rows
    every iteration, "auto" takes the mesh where the slab fits.  The ranks agree on it
    first (``xsweep_engine``: the mesh only on equal shards), so every rank runs the same
    engine and reduces POT's error in the same order."""
    ops._dev(C_local, "C_local")
    if C_local.dtype not in (torch.float32, torch.float16):
        raise TypeError("sinkhorn_xsweep: float32 or float16 cost rows")
    if engine not in ("auto", "sweep", "mesh"):
        raise ValueError(f"engine must be 'auto', 'sweep' or 'mesh', not {engine!r}")
    n, m = C_local.shape
    if m != xpeer.m:
        raise ValueError(f"C_local has {m} columns, the exchange was built for {xpeer.m}")
    dev = C_local.device
    C = ops._rowmajor(C_local, ops._VEC[C_local.dtype])
    a = a_local.to(dev, torch.float32).contiguous()
    bb = b.to(dev, torch.float32).contiguous()
    if a.numel() != n or bb.numel() != m:
        raise ValueError("a_local / b do not match C_local")
    cs = None if cost_scale is None else cost_scale.to(dev, torch.float32).contiguous()
    engine = xsweep_engine(engine, n, xpeer.world, xpeer._group)
    opts = L.SinkhornOpts(reg=float(reg), stop_thr=float(stop_thr), max_iter=int(max_iter),
                          check_every=int(check_every), flavor=L.OTF_FLAVOR_POT,
                          err_squared=int(err_squared), sync_every=0, engine=L.ENGINES[engine],
                          cost_f16=int(C.dtype == torch.float16), n_total=int(n_total))
    if workspace is None:
        workspace = ops.sinkhorn_workspace(n, m, torch.float32, max_iter, dev)
    u = torch.empty(n, dtype=torch.float32, device=dev)
    v = torch.empty(m, dtype=torch.float32, device=dev)
    P = ops._alloc_rowmajor(n, m, plan_dtype or torch.float32, dev, 4) if want_plan else None
    info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=dev)
    errlog = torch.empty(max_iter // max(check_every, 1) + 2, dtype=torch.float64, device=dev)
    L.check(L.lib().otf_sinkhorn_xsweep(
        a.data_ptr(), bb.data_ptr(), C.data_ptr(), n, m, C.stride(0), ops._DT[torch.float32],
        L.ptr(cs), ctypes.byref(opts), xpeer.handle, u.data_ptr(), v.data_ptr(), L.ptr(P),
        P.stride(0) if P is not None else 0, ops._DT[P.dtype] if P is not None else 0,
        info.data_ptr(), errlog.data_ptr(), workspace.data_ptr(), workspace.numel(),
        L.stream_handle(dev)), "otf_sinkhorn_xsweep")
    res = ops.SinkhornResult(u=u, v=v, plan=P, info_dev=info, errlog_dev=errlog)
    res._keep = (C, a, bb, cs, workspace)
    return res


def coupled_solve_sharded(X_local: torch.Tensor, Y_local: torch.Tensor, reg: float,
                          max_iter: int = 200, stop_thr: float = 0.0, cost_dtype=torch.float16,
                          want_plan: bool = True, sync_every: int = 0, group=None, comm=None,
                          xpeer: XPeer | None = None, engine: str = "auto"):
    """The per-epoch global OT of one large problem over the data-parallel ranks:
    all-gather the PET embedding shards (RCCL), cost rows of this rank's MRI shard
    against every PET embedding (fp16 storage by default, BASELINE config 5), one
    all-reduce(MAX) for scale_cost="max_cost", then the row-sharded Sinkhorn with
    uniform marginals.  With an ``xpeer`` exchange the solve is the in-kernel cross-rank
    sweep (``sinkhorn_xsweep``), otherwise the row-sharded solve with one all-reduce per
    iteration.  ``engine`` picks the cross-rank engine of the xpeer form ("auto": the
    register-resident mesh where this rank's slab fits, else the sweep; sinkhorn_xsweep).
    Returns (SinkhornResult of this rank's rows, n_total)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    x_sizes = None
    if comm is not None and comm.nranks > 1:
        # shard sizes may differ (a ragged last shard): the row counts of X and Y are
        # exchanged through the communicator, never assumed equal -- a wrong n_total
        # would make a = 1/n_total sum to != 1 and a fixed-count all-gather would read
        # garbage or hang
        Y_all, _ = comm.all_gather_rows(Y_local)
        nx = torch.tensor([float(X_local.shape[0])], dtype=torch.float64, device=X_local.device)
        x_sizes = [int(x) for x in comm.all_gather(nx).cpu().tolist()]
    elif comm is not None:
        Y_all = Y_local
    else:
        Y_all = all_gather_rows(Y_local, group) if world > 1 else Y_local
    C, cmax, unit = ops.pairwise_cost_ex(X_local, Y_all, zero_diag=False, out_dtype=cost_dtype)
    # the max in true cost units, agreed over ranks; each rank's stored unit may differ
    gmax = cmax * unit
    if comm is not None:
        comm.all_reduce(gmax, op="max")
        n_total = sum(x_sizes) if x_sizes is not None else X_local.shape[0]
    else:
        n = torch.tensor([X_local.shape[0]], dtype=torch.int64, device=X_local.device)
        if world > 1:
            dist.all_reduce(gmax, op=dist.ReduceOp.MAX, group=group)
            dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
        n_total = int(n.item())
    m = Y_all.shape[0]
    a = torch.full((X_local.shape[0],), 1.0 / n_total, dtype=torch.float32, device=X_local.device)
    b = torch.full((m,), 1.0 / m, dtype=torch.float32, device=X_local.device)
    if xpeer is not None:
        return sinkhorn_xsweep(a, b, C, reg, xpeer, n_total, max_iter=max_iter, stop_thr=stop_thr,
                               cost_scale=gmax / unit, want_plan=want_plan, engine=engine), n_total
    res = sinkhorn_row_sharded(a, b, C, reg, max_iter=max_iter, stop_thr=stop_thr,
                               cost_scale=gmax / unit, n_total=n_total, sync_every=sync_every,
                               want_plan=want_plan, group=group, comm=comm)
    return res, n_total
