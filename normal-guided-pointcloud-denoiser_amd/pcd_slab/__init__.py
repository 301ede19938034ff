"""Spatial-slab multi-GPU denoising: one process per GPU, RCCL halo exchange.

The frozen snapshot is cut into P slabs of equal point count along its longest bbox axis.  Rank r owns the points
of slab r and holds, in addition, a HALO: every snapshot point whose coordinate on that axis lies within `halo`
of the slab.  Its grid is built over owned + halo points on the global cell lattice (pcd_grid_params), so its
spatial order is a subsequence of the one-GPU order and distance ties break exactly as on one GPU.

Per iteration the rank runs the fused loop on its OWN rows only and keeps the halo rows current between stages (the
only places a stage reads another rank's points).  The product path is ONE library call per iteration
(pcd_slab_iterate: the stages, the RCCL halo exchanges on a stream of their own, overlapped with the rows that read
no halo row, and the two all-reduces; libpcd owns the RCCL communicator, pcd_comm).  The same sequence also runs
stage by stage from Python (native=False: pcd_denoiser_stage + pack/unpack + torch.distributed), the path the CPU
tests drive with an oracle engine:
    KNN_NVT1                        kNN + first vote + VU smoothing of own points
    exchange FN                     NVT2 reads the smoothed normals of the neighbours
    NVT2                            classes + edge vectors
    per phase: [flat/new: SUM -> all-reduce(sum) -> CENTRE -> MAXDIST -> all-reduce(max)] APPLY -> exchange POS
    FINISH                          n := f_n (the halo rows' f_n arrived with the FN exchange)
The global flat centre / delta (Denoiser.py:106-107) are the only collectives; halo traffic is point-to-point
between slab neighbours.  Exactness is checked, not assumed: every k-ball must stay inside the slab widened by the
halo (pcd_denoiser_set_coverage).  Every `check_every` iterations the driver reads the device error word (one host
sync and a 1-int all-reduce); when a k-ball has left a rank's coverage it restores the state of the last checkpoint,
widens the halo (x `halo_growth`), re-plans every rank from the frozen snapshot and replays the iterations since the
checkpoint -- the result is the one a wide-enough halo gives from the start.

Slabs are cut at quantiles of a per-point COST weight (default 1 = equal counts).  rebalance() re-plans with weights
from the last iteration's classes (edge / corner points run the dearer 3x3-solve steps), the same machinery as the
thin-halo re-plan.

The driver is engine-agnostic: `HipSlabEngine` (libpcd, the product path) or any object with the same methods
(the CPU tests use an oracle engine, tests/slab_cpu_engine.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

import pcd_native as nat


# ----------------------------------------------------------------------------------------------- partition
def _cut(snap: torch.Tensor, world: int, axis: int | None = None, weights: torch.Tensor | None = None):
    """The slab cut of `snap` (every rank computes the same one): (axis, axis key, owner rank of each point, per-rank
    lo / hi of the owned keys).  Equal point counts along the longest bbox axis, or (weights, [N] >= 0) equal shares of
    the cumulative weight; each rank owns at least one point; ties on the axis broken by index (stable sort)."""
    n = snap.size(0)
    assert world >= 1 and n >= world, "need at least one point per rank"
    if axis is None:
        axis = int(torch.argmax(snap.max(0).values - snap.min(0).values).item())
    key = snap[:, axis].contiguous()
    order = torch.sort(key, stable=True).indices
    if weights is None:
        bounds = [(r * n) // world for r in range(world + 1)]
    else:
        cw = torch.cumsum(weights.to(snap.device, torch.float64)[order], 0)
        tot = float(cw[-1])
        cuts = torch.tensor([tot * r / world for r in range(1, world)], dtype=torch.float64, device=snap.device)
        inner = torch.searchsorted(cw, cuts).tolist() if world > 1 else []
        bounds = [0] + [int(b) for b in inner] + [n]
        for r in range(1, world + 1):                           # at least one point per rank, monotone
            bounds[r] = min(max(bounds[r], bounds[r - 1] + 1), n - (world - r))
    owner = torch.empty(n, dtype=torch.int64, device=snap.device)
    lo, hi = [], []
    for r in range(world):
        owner[order[bounds[r]:bounds[r + 1]]] = r
        ks = key[order[bounds[r]:bounds[r + 1]]]
        lo.append(float(ks[0]))
        hi.append(float(ks[-1]))
    return axis, key, owner, lo, hi


@dataclass
class Spheres:
    """Coverage spheres of the sparse points near a cut (cut_spheres): centre ids (global), radii, and the snapshot
    members each centre's owner must hold -- per owner rank, the union of its spheres' members (global ids, unique),
    so a plan holds them whatever the spheres' overlap."""
    ids: torch.Tensor
    radii: torch.Tensor
    by_rank: dict

    @staticmethod
    def around(snap: torch.Tensor, ids: torch.Tensor, radii: torch.Tensor, owner: torch.Tensor, k_hint: int = 16,
               chunk_members: int = 32_000_000) -> "Spheres":
        """owner: [N] rank of every snapshot point (the plan's cut).  The members are found a chunk of centres at a
        time (at most ~chunk_members pairs in flight), so wide spheres -- a long planned horizon -- stay bounded in
        memory."""
        dev = nat.device()
        if ids.numel() == 0:
            return Spheres(ids.to(snap.device), torch.zeros(0, device=snap.device), {})
        g = nat.Grid(snap.to(dev), k_hint=k_hint)
        q = snap.to(dev)[ids.to(dev)].contiguous()
        # (membership at a hair over the radius: the coverage test asks for the ball strictly inside it)
        r = (radii.to(dev, torch.float32) * 1.0001).contiguous()
        own_c = owner.to(dev)[ids.to(dev)]
        n = snap.size(0)
        cum = torch.cumsum(g.radius_counts(q, r), 0)
        keys, start, nq = [], 0, ids.numel()
        while start < nq:
            base = int(cum[start - 1]) if start else 0
            end = int(torch.searchsorted(cum, torch.tensor([base + chunk_members], device=dev), right=True))
            end = min(max(end, start + 1), nq)
            sl, j = g.radius(q[start:end], r[start:end])
            keys.append(torch.unique(torch.repeat_interleave(own_c[start:end], sl.diff()) * n + j))
            start = end
        allk = torch.unique(torch.cat(keys))
        rk = allk // n
        by_rank = {int(x): (allk[rk == x] % n).to(snap.device) for x in torch.unique(rk).tolist()}
        return Spheres(ids.to(snap.device), radii.to(snap.device, torch.float32), by_rank)


@dataclass
class SlabPlan:
    """Owned / halo membership of every rank, identical on all ranks (computed from the same snapshot)."""
    world: int
    axis: int
    halo: float
    owner: torch.Tensor                         # int64 [N]: rank owning each snapshot point
    lo: list                                    # per rank: min coordinate of the owned points on `axis`
    hi: list                                    # per rank: max coordinate
    local: list = field(default_factory=list)   # per rank: int64 global indices of owned + halo, ascending
    spheres: "Spheres | None" = None            # points whose k-ball reaches past the band halo (cut_spheres)

    @staticmethod
    def build(snap: torch.Tensor, world: int, halo: float, axis: int | None = None,
              weights: torch.Tensor | None = None, spheres: "Spheres | None" = None) -> "SlabPlan":
        """weights (optional, [N] >= 0, identical on every rank): cut at quantiles of the cumulative weight along the
        axis instead of equal point counts (each rank still owns at least one point).  spheres (optional): every
        member of a sphere is local to the owner of its centre, beyond the band."""
        snap = snap.detach()
        axis, key, owner, lo, hi = _cut(snap, world, axis, weights)
        local = []
        for r in range(world):
            inside = (key >= lo[r] - halo) & (key <= hi[r] + halo)
            if spheres is not None and r in spheres.by_rank:
                inside = inside.clone()
                inside[spheres.by_rank[r].to(inside.device)] = True
            local.append(torch.nonzero(inside | (owner == r)).flatten())
        return SlabPlan(world, axis, float(halo), owner, lo, hi, local, spheres)

    def coverage(self, r: int):
        """Box the rank's local snapshot covers: the slab widened by the halo on `axis` (open ends at the outer
        slabs and on the other axes)."""
        big = 3.0e38
        lo, hi = [-big] * 3, [big] * 3
        if r > 0:
            lo[self.axis] = self.lo[r] - self.halo
        if r < self.world - 1:
            hi[self.axis] = self.hi[r] + self.halo
        return lo, hi

    def transfer(self, src: int, dst: int) -> torch.Tensor:
        """Global indices (ascending) of points owned by `src` that `dst` holds as halo."""
        loc = self.local[dst]
        return loc[self.owner[loc] == src]


# ----------------------------------------------------------------------------------------------- transport
class TorchTransport:
    """The slab driver's CONTROL plane over a torch.distributed CPU group (gloo): the RCCL unique id, the few scalars
    of the plan, the coverage verdicts.  The DATA plane is libpcd's own communicator (pcd_comm, native_comm): RCCL
    over xGMI (rccl=True: one GPU per rank, the product path) or host callbacks over this gloo group (rccl=False:
    ranks sharing one GPU, the tests and the one-GPU rehearsal).  There is exactly one RCCL communicator per process,
    and it belongs to the library; an NCCL torch group is refused.  The staged path (SlabDenoiser(native=False))
    exchanges halo rows over this group itself, staged through host memory."""

    def __init__(self, group=None, rccl: bool = False):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if dist.get_backend(group) != "gloo":
            raise ValueError("pcd_slab: the control group must be gloo (CPU); RCCL is libpcd's own (pcd_comm) -- "
                             "pass TorchTransport(rccl=True) for an RCCL data plane")
        self.host = True
        self.rccl = bool(rccl)
        self._comm = None

    def exchange(self, sends: dict, recv_shapes: dict, device) -> dict:
        """sends: peer -> tensor; recv_shapes: peer -> shape.  Returns peer -> received tensor on `device`."""
        dist = self.dist
        ops, outs, staged = [], {}, {}
        for peer, shape in recv_shapes.items():
            buf = torch.empty(shape, dtype=torch.float32)
            outs[peer] = buf
            ops.append(dist.P2POp(dist.irecv, buf, peer, self.group))
        for peer, t in sends.items():
            staged[peer] = t.cpu()
            ops.append(dist.P2POp(dist.isend, staged[peer], peer, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return {p: b.to(device) for p, b in outs.items()}

    def send(self, t: torch.Tensor, dst: int):
        self.dist.send(t.contiguous().cpu(), dst, self.group)

    def recv(self, t: torch.Tensor, src: int) -> torch.Tensor:
        h = torch.empty(t.shape, dtype=t.dtype)
        self.dist.recv(h, src, self.group)
        t.copy_(h)
        return t

    def native_comm(self) -> "nat.Comm":
        """libpcd's data plane for pcd_slab_iterate and the slab hand-out (collective on first use, then cached): an
        RCCL communicator (rccl=True; its unique id travels over this gloo group), else host callbacks over this
        group -- the same library code path, each exchange staged through pinned host memory."""
        if self._comm is not None:
            return self._comm
        dist, grp = self.dist, self.group
        if self.rccl:
            self._comm = nat.Comm.rccl(self.world, self.rank, lambda t: self.broadcast_(t, 0))
            return self._comm

        def exchange(peers, send, soff, recv, roff):
            ops = []
            for q, peer in enumerate(peers):
                if roff[q + 1] > roff[q]:
                    ops.append(dist.P2POp(dist.irecv, torch.from_numpy(recv[roff[q]:roff[q + 1]]), peer, grp))
                if soff[q + 1] > soff[q]:
                    ops.append(dist.P2POp(dist.isend, torch.from_numpy(send[soff[q]:soff[q + 1]].copy()), peer, grp))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()

        def allreduce(buf, op):
            t = torch.from_numpy(buf)
            dist.all_reduce(t, dist.ReduceOp.MAX if op == nat.OP_MAX else dist.ReduceOp.SUM, grp)

        self._comm = nat.Comm.host(self.world, self.rank, exchange, allreduce)
        return self._comm

    def close(self):
        """Tear libpcd's communicator down (collective in spirit: every rank calls it at the same point, after its
        last use -- drivers and engines holding it must be gone or done)."""
        if self._comm is not None:
            torch.cuda.synchronize()
            self._comm.destroy()
            self._comm = None
        self.dist.barrier(self.group)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        h = t.cpu() if t.device.type != "cpu" else t
        self.dist.broadcast(h, src, self.group)
        if h is not t:
            t.copy_(h)
        return t

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        dist = self.dist
        red = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op]
        h = t.cpu() if t.device.type != "cpu" else t
        dist.all_reduce(h, red, self.group)
        if h is not t:
            t.copy_(h)
        return t


class LocalTransport:
    """world = 1: nothing to exchange."""
    rank, world, host, rccl = 0, 1, True, False

    def exchange(self, sends, recv_shapes, device):
        assert not sends and not recv_shapes
        return {}

    def all_reduce(self, t, op):
        return t

    def broadcast_(self, t, src=0):
        return t

    def native_comm(self):
        def never(*_):
            raise RuntimeError("world 1 has nothing to exchange")
        return nat.Comm.host(1, 0, never, never)


# ----------------------------------------------------------------------------------------------- HIP engine
class HipSlabEngine:
    """libpcd's fused loop over one rank's local snapshot (owned + halo), driven stage by stage."""

    def __init__(self, local_pos, local_n, owned_local, k_max, origin, cell, coverage, seeding=True, spheres=None):
        dev = nat.device()
        self.device = dev
        self.grid = nat.Grid(local_pos.to(dev), cell=cell, origin=origin)
        perm = self.grid.perm().long()                      # spatial row -> local index
        self.row_of = torch.empty_like(perm)
        self.row_of[perm] = torch.arange(perm.numel(), device=dev)
        self.n = perm.numel()
        self.fused = nat.FusedDenoiser(self.grid, k_max)
        self.fused.load(local_pos.to(dev), local_n.to(dev))
        self.fused.set_seeding(seeding)
        own_rows = torch.sort(self.row_of[owned_local.to(dev)]).values.to(torch.int32)
        # every local point owned (one rank): all rows, no row list (the single-GPU launch shapes)
        self.fused.set_rows(None if own_rows.numel() == self.n else own_rows)
        self.fused.set_coverage(*coverage)
        if spheres is not None:
            self.fused.set_coverage_spheres(spheres.to(dev))      # (local order: the loaded rows' order)
        self.red4 = torch.zeros(4, dtype=torch.float64, device=dev)
        self.red1 = torch.zeros(1, dtype=torch.float32, device=dev)

    def rows(self, local_idx: torch.Tensor) -> torch.Tensor:
        return self.row_of[local_idx.to(self.device)].to(torch.int32).contiguous()

    def stage(self, params, stage, phase=0, red=None):
        self.fused.stage(params, stage, phase, red)

    def pack(self, fld, rows):
        return self.fused.pack(fld, rows)

    def unpack(self, fld, rows, data):
        self.fused.unpack(fld, rows, data)

    def check(self):
        self.fused.check()

    def status(self) -> int:
        return self.fused.status()

    def coverage_excess(self) -> tuple:
        return self.fused.coverage_excess()

    # the one-call iteration (pcd_slab_iterate)
    native = True

    def set_routes(self, peers, send_rows, recv_rows, own_lo, own_hi):
        self.fused.set_routes(peers, send_rows, recv_rows, own_lo, own_hi)

    def slab_iterate(self, comm, params, iterations=1):
        self.fused.slab_iterate(comm, params, iterations)

    def readset_stats(self) -> tuple:
        """(iterations, send rows, receive rows) of the read-set exchange since the routes were set (summed)."""
        return self.fused.readset_stats()

    def slab_iterate_timed(self, comm, params) -> dict:
        """One slab iteration with the library's per-stage HIP events (pcd_denoiser_set_timing), ms."""
        self.fused.set_timing(True)
        self.fused.slab_iterate(comm, params, 1)
        slots = self.fused.timing()
        self.fused.set_timing(False)
        names = nat.FusedDenoiser.TIMING_SLOTS
        out = {names[i]: float(slots[i]) for i in range(min(len(slots), len(names)))}
        out["knn_nvt1"] = float(sum(slots[:4]))
        out["iteration"] = float(sum(slots))
        return out

    def set_state(self, local_idx, pos, n):
        """Current positions / normals of the given local points (a re-planned rank taking over the state)."""
        rows = self.rows(local_idx)
        pad = torch.zeros((rows.numel(), 1), dtype=torch.float32, device=self.device)
        self.fused.unpack(nat.FIELD_POS, rows, torch.cat([pos.to(self.device, torch.float32), pad], 1))
        self.fused.unpack(nat.FIELD_NRM, rows, torch.cat([n.to(self.device, torch.float32), pad], 1))

    def classes(self) -> torch.Tensor:
        """Classes of the last NVT2 stage per local point (int64, local order)."""
        cls = torch.empty(self.n, dtype=torch.int64, device=self.device)
        self.fused.store(classes=cls)
        return cls

    def store(self):
        pos = torch.empty((self.n, 3), dtype=torch.float32, device=self.device)
        n = torch.empty_like(pos)
        self.fused.store(pos, n)
        return pos, n


# ----------------------------------------------------------------------------------------------- driver
@dataclass
class RankShare:
    """One rank's share of a plan, as the coordinator hands it out: its local snapshot (owned + halo), the owned
    rows, the halo routes (peer -> local indices to send / receive) and the boxes the engine checks and overlaps on."""
    local: torch.Tensor                 # int64 [nl]: global ids, ascending
    owned_local: torch.Tensor           # int64 [no]: local indices of the owned points, ascending
    pos: torch.Tensor                   # float32 [nl, 3]: the frozen snapshot's rows
    n: torch.Tensor                     # float32 [nl, 3]
    peers: list
    send_local: list                    # per peer: int64 local indices of own points the peer holds as halo
    recv_local: list                    # per peer: int64 local indices of the peer's points held here as halo
    coverage: tuple                     # (lo3, hi3): the slab widened by the halo
    own_box: tuple | None               # (lo3, hi3): the owned slab, strict (None at world 1)
    lattice: tuple                      # (origin3, cell) of the global cell lattice (HIP engine)
    halo: float
    axis: int
    state: tuple | None = None          # (pos, n) [nl, 3] of the current iterate to take over (a re-plan)
    xr: torch.Tensor | None = None      # float32 [nl]: coverage sphere radius of each local point (0: none)


def _share(plan: SlabPlan, r: int, snap_pos, snap_n, lattice, state=None) -> RankShare:
    """The coordinator's cut of `plan` for rank r (everything on snap_pos's device)."""
    world = plan.world
    local = plan.local[r]
    owner_l = plan.owner[local]
    owned_local = torch.nonzero(owner_l == r).flatten()
    to_local = None
    peers, send_local, recv_local = [], [], []
    for q in range(world):
        if q == r:
            continue
        out = plan.transfer(r, q)            # own points q holds (global, ascending)
        inc = plan.transfer(q, r)            # q's points held here
        if out.numel() == 0 and inc.numel() == 0:
            continue
        if to_local is None:
            to_local = torch.full((plan.owner.numel(),), -1, dtype=torch.int64, device=local.device)
            to_local[local] = torch.arange(local.numel(), device=local.device)
        peers.append(q)
        send_local.append(to_local[out])
        recv_local.append(to_local[inc])
    own_box = None
    if peers:
        # the OWNED slab, strict: a snapshot point ON a cut may be owned by the neighbour, so the box is shrunk by
        # one float32 ulp on the cut faces (rows whose k-ball stays inside it read no halo row)
        import numpy as np
        big = 3.0e38
        lo, hi = [-big] * 3, [big] * 3
        if r > 0:
            lo[plan.axis] = float(np.nextafter(np.float32(plan.lo[r]), np.float32(np.inf)))
        if r < world - 1:
            hi[plan.axis] = float(np.nextafter(np.float32(plan.hi[r]), np.float32(-np.inf)))
        own_box = (lo, hi)
    st = None if state is None else (state[0][local.to(state[0].device)], state[1][local.to(state[1].device)])
    xr = None
    sp = plan.spheres
    if sp is not None and sp.ids.numel():
        mine = plan.owner[sp.ids] == r
        if bool(mine.any()):
            if to_local is None:
                to_local = torch.full((plan.owner.numel(),), -1, dtype=torch.int64, device=local.device)
                to_local[local] = torch.arange(local.numel(), device=local.device)
            xr = torch.zeros(local.numel(), dtype=torch.float32, device=local.device)
            xr[to_local[sp.ids[mine]]] = sp.radii[mine].to(local.device)
    return RankShare(local, owned_local, snap_pos[local], snap_n[local], peers, send_local, recv_local,
                     plan.coverage(r), own_box, lattice, plan.halo, plan.axis, st, xr)


class SlabDenoiser:
    """The body of Processor.denoise (Processor.py:119-139) over spatial slabs, one rank per GPU.

    Rank 0 is the COORDINATOR, the one process that holds the whole cloud as the reference's single process does
    (Processor.py:115-121): snap_pos / snap_n are read on rank 0 only (the other ranks may pass None).  It estimates
    the halo, cuts the slabs, and hands every rank its share -- slab + halo rows of the frozen snapshot, owned rows,
    routes -- over libpcd's communicator (pcd_comm_sendrecv: RCCL over xGMI in the product path).  No other rank ever
    holds or plans over the whole cloud.  A re-plan (thin halo, rebalance) gathers the owned state to rank 0, which
    cuts again and hands out the new shares.  halo: slab widening in snapshot units (None: cut_halo, on rank 0 --
    the snapshot's own largest k-ball reach past a face, x 1.25).
    check_every: iterations between coverage checks (0: never -- check() raises at the caller's request instead);
    halo_growth / max_replans: the thin-halo recovery."""

    def __init__(self, snap_pos, snap_n, k_max, transport=None, halo=None, engine_factory=None, seeding=True,
                 k_hint=None, check_every=1, halo_growth=2.0, max_replans=4, weights=None, native=None,
                 sphere_quantile=0.999, step_bound=None, horizon=None):
        """native: one pcd_slab_iterate call per iteration over libpcd's own transport (default for the HIP engine);
        False: the same stages driven from Python over torch.distributed.  sphere_quantile: the default halo covers
        this quantile of the near-face k-ball needs; the points beyond it keep coverage spheres (cut_spheres).
        step_bound: the loop's per-iteration displacement bound (params.d: every step's move is clamped below it),
        which prices the drift the first plan must cover; horizon: the iterations a plan is sized to cover (default
        check_every) -- the default halo of every later plan (rebalance, a coverage re-plan) prices each point's
        measured drift over that many iterations ahead (cut_spheres), so a run of `horizon` iterations needs no
        coverage re-plan."""
        self.t = transport or LocalTransport()
        rank, world = self.t.rank, self.t.world
        # cell lattice of the ranks' snapshot indices: the fused loop's (pcd_native.fused_k_hint) unless given
        self.k_max, self.k_hint, self.seeding = k_max, k_hint or nat.fused_k_hint(k_max) or 32, seeding
        self.engine_factory = engine_factory
        self.native = (engine_factory is None) if native is None else bool(native)
        self.comm = self.t.native_comm() if self.native else None
        self.check_every, self.halo_growth, self.max_replans = int(check_every), float(halo_growth), int(max_replans)
        self.replans = 0
        self.replan_log = []       # per re-plan: why (coverage: what failed and by how much / rebalance) and the new halo
        self.e = None
        # the default halo (halo=None, HIP engine, world > 1) is the band + coverage spheres of cut_spheres, recomputed
        # for every new cut (rebalance); a coverage failure grows only the component that failed, by what it lacked
        self._auto_halo = halo is None and world > 1 and engine_factory is None
        self._sphere_quantile = float(sphere_quantile)
        self._band_floor = 0.0     # the band a coverage failure grew to (a re-cut never goes below it)
        self._sphere_scale = 1.0   # the spheres' growth by coverage failures
        self.step_bound = float(step_bound) if step_bound else 0.0
        self.horizon = int(horizon) if horizon else max(int(check_every), 1)
        self.iterations_done = 0   # iterations since load (the drift estimate's clock)
        self._ckpt_iter = 0
        if rank == 0:
            self.snap_pos, self.snap_n = snap_pos.detach().contiguous(), snap_n.detach().contiguous()
            self.dev = self.snap_pos.device
            self._spheres = None
            if halo is None:
                if world > 1:
                    halo, sid, srad = cut_spheres(self.snap_pos, world, k_max, quantile=sphere_quantile, weights=weights,
                                                  step=self.step_bound, horizon=self.horizon)
                    self._spheres = (Spheres.around(self.snap_pos, sid, srad, _cut(self.snap_pos, world, None, weights)[2])
                                     if engine_factory is None else None)
                else:
                    halo = 0.0
            self._lattice = (nat.grid_params(self.snap_pos.to(nat.device()), k_hint=self.k_hint)
                             if engine_factory is None else ([0.0, 0.0, 0.0], 0.0))
            self._weights = weights                 # (the cut's cost weights: a halo re-plan keeps them)
            plan = SlabPlan.build(self.snap_pos, world, halo, weights=weights, spheres=self._spheres)
            nt = torch.tensor([self.snap_pos.size(0)], dtype=torch.int64)
        else:
            self.snap_pos = self.snap_n = None
            self.dev = nat.device() if engine_factory is None else torch.device("cpu")
            plan, nt = None, torch.zeros(1, dtype=torch.int64)
        self.n_total = int(self.t.broadcast_(nt, 0)) if world > 1 else int(nt)
        self.plan = plan                         # (the coordinator's; None on the other ranks)
        self._setup(plan)
        self._since = 0            # iterations since the last checkpoint
        self._pending = []         # their params (replayed after a re-plan)
        self._ckpt = None

    # -------------------------------------------------------------------------------- coordinator <-> ranks
    def _p2p_send(self, t: torch.Tensor, dst: int):
        if self.native:
            self.comm.sendrecv(dst, t.contiguous().to(nat.device()), -1, None)
        else:
            self.t.send(t, dst)

    def _p2p_recv(self, shape, dtype, src: int) -> torch.Tensor:
        if self.native:
            return self.comm.sendrecv(-1, None, src, torch.empty(shape, dtype=dtype, device=nat.device()))
        return self.t.recv(torch.empty(shape, dtype=dtype, device=self.dev), src)

    def _send_share(self, s: RankShare, dst: int):
        """Four messages: a fixed header, the index arrays, the float64 boxes, the float32 rows."""
        ints = [s.local, s.owned_local, torch.tensor(s.peers, dtype=torch.int64),
                torch.tensor([x.numel() for x in s.send_local], dtype=torch.int64),
                torch.tensor([x.numel() for x in s.recv_local], dtype=torch.int64)] + s.send_local + s.recv_local
        ints = torch.cat([x.to(self.dev, torch.int64) for x in ints])
        nan = float("nan")
        own = s.own_box or ([nan] * 3, [nan] * 3)
        flt = torch.tensor(list(s.coverage[0]) + list(s.coverage[1]) + list(own[0]) + list(own[1])
                           + list(s.lattice[0]) + [s.lattice[1], s.halo, float(s.axis)], dtype=torch.float64)
        cols = [s.pos, s.n] + (list(s.state) if s.state is not None else []) + \
               ([s.xr[:, None]] if s.xr is not None else [])
        rows = torch.cat([c.to(self.dev, torch.float32) for c in cols], 1)
        head = torch.tensor([s.local.numel(), s.owned_local.numel(), len(s.peers), int(s.state is not None),
                             ints.numel(), int(s.xr is not None), 0, 0], dtype=torch.int64)
        for t in (head, ints, flt, rows):
            self._p2p_send(t, dst)

    def _recv_share(self) -> RankShare:
        head = self._p2p_recv((8,), torch.int64, 0).cpu().tolist()
        nl, no, npeers, has_state, nints, has_xr = head[:6]
        ints = self._p2p_recv((nints,), torch.int64, 0).to(self.dev)
        flt = self._p2p_recv((20,), torch.float64, 0).cpu().tolist()
        rows = self._p2p_recv((nl, (12 if has_state else 6) + (1 if has_xr else 0)), torch.float32, 0).to(self.dev)
        o = 0
        local, o = ints[o:o + nl], o + nl
        owned_local, o = ints[o:o + no], o + no
        peers, o = ints[o:o + npeers].tolist(), o + npeers
        ns, o = ints[o:o + npeers].tolist(), o + npeers
        nr, o = ints[o:o + npeers].tolist(), o + npeers
        send_local, recv_local = [], []
        for c in ns:
            send_local.append(ints[o:o + c])
            o += c
        for c in nr:
            recv_local.append(ints[o:o + c])
            o += c
        own = None if flt[6] != flt[6] else (flt[6:9], flt[9:12])
        st = (rows[:, 6:9], rows[:, 9:12]) if has_state else None
        xr = rows[:, -1].contiguous() if has_xr else None
        return RankShare(local, owned_local, rows[:, 0:3], rows[:, 3:6], peers, send_local, recv_local,
                         (flt[0:3], flt[3:6]), own, (flt[12:15], flt[15]), flt[16], int(flt[17]), st, xr)

    def _gather_to0(self, x: torch.Tensor):
        """Per-point values of every rank's own points (owned-local order, [n_own, c] float32) -> the global
        [N, c] on the coordinator (None elsewhere).  The coordinator knows every rank's owned ids from its plan, so
        only the values travel.  Collective."""
        rank, world = self.t.rank, self.t.world
        x = x.to(self.dev, torch.float32).contiguous()
        if rank != 0:
            self._p2p_send(x, 0)
            return None
        out = torch.empty((self.n_total, x.size(1)), dtype=torch.float32, device=self.dev)
        out[self.owned_global.to(self.dev)] = x
        for r in range(1, world):
            ids = torch.nonzero(self.plan.owner == r).flatten().to(self.dev)
            out[ids] = self._p2p_recv((ids.numel(), x.size(1)), torch.float32, r).to(self.dev)
        return out

    # -------------------------------------------------------------------------------- plan -> engine + routes
    def _setup(self, plan, state=None):
        """Hand out `plan` (coordinator) / take this rank's share, then build the engine and halo routes; state =
        (global pos, global n) of the CURRENT iterate on the coordinator (None: the snapshot, a fresh start)."""
        rank, world = self.t.rank, self.t.world
        self.e = None                                           # free the old engine's device state first
        if rank == 0:
            self.plan = plan
            for r in range(1, world):
                self._send_share(_share(plan, r, self.snap_pos, self.snap_n, self._lattice, state), r)
            s = _share(plan, 0, self.snap_pos, self.snap_n, self._lattice, state)
        else:
            s = self._recv_share()
        self.halo, self.axis = s.halo, s.axis
        self.local = s.local
        self.owned_local = s.owned_local
        self.owned_global = self.local[self.owned_local]
        if self.engine_factory is None:
            self.e = HipSlabEngine(s.pos, s.n, self.owned_local, self.k_max, s.lattice[0], s.lattice[1], s.coverage,
                                   self.seeding, spheres=s.xr)
        else:
            self.e = self.engine_factory(s.pos, s.n, self.owned_local, self.k_max, s.coverage)
        if s.state is not None:
            # the engine loaded the snapshot (its `orig` for the global clamp); the current iterate goes on top
            self.e.set_state(torch.arange(self.local.numel(), device=self.local.device), s.state[0], s.state[1])
        # halo routes: rows I send to each peer and rows I receive from it (both ascending global index)
        self.send_rows, self.recv_rows = {}, {}
        for q, peer in enumerate(s.peers):
            if s.send_local[q].numel():
                self.send_rows[peer] = self.e.rows(s.send_local[q])
            if s.recv_local[q].numel():
                self.recv_rows[peer] = self.e.rows(s.recv_local[q])
        self.halo_points = sum(r.numel() for r in self.recv_rows.values())
        if self.native:
            # routes + the OWNED slab (NVT2 / the phases run the rows that read no halo row while an exchange is in
            # flight)
            peers = sorted(set(self.send_rows) | set(self.recv_rows))
            empty = torch.zeros(0, dtype=torch.int32, device=nat.device())
            own = s.own_box if peers else None
            self.e.set_routes(peers, [self.send_rows.get(q, empty) for q in peers],
                              [self.recv_rows.get(q, empty) for q in peers], own[0] if own else None,
                              own[1] if own else None)

    def _owned_state_now(self):
        """(pos, n) of this rank's own points, owned-local order (a checkpoint)."""
        rows = self.e.rows(self.owned_local)
        return self.e.pack(nat.FIELD_POS, rows)[:, :3].clone(), self.e.pack(nat.FIELD_NRM, rows)[:, :3].clone()

    def _global_state(self, owned_pos, owned_n):
        g = self._gather_to0(torch.cat([owned_pos, owned_n], 1))
        return None if g is None else (g[:, :3], g[:, 3:])

    def _replan(self, halo=None, weights=None, state="now", sphere_scale=None, at=None, horizon=None):
        """Re-cut every rank from the frozen snapshot, taking over `state` (global current pos, n on the
        coordinator, None on the other ranks, reached after `at` iterations; "now": gather the present iterate).
        halo / sphere_scale (coordinator): the grown band and the factor for the coverage spheres (None: unchanged);
        weights: a new cost-weighted cut.  With the default halo the band and the spheres are recomputed for the
        state's positions and the drift of `horizon` iterations ahead (cut_spheres: a moved cut has new sparse points
        near it, and the drift since the snapshot has moved every ball), never below `halo`.  Collective: all ranks
        call it together."""
        if isinstance(state, str):
            state = self._global_state(*self._owned_state_now())
            at = self.iterations_done
        plan = None
        if self.t.rank == 0:
            if weights is not None:
                self._weights = weights
            if self._auto_halo:
                band, sid, srad = cut_spheres(self.snap_pos, self.t.world, self.k_max, quantile=self._sphere_quantile,
                                              axis=self.plan.axis, weights=self._weights,
                                              query=None if state is None else state[0], iterations=at or 0,
                                              step=self.step_bound, horizon=horizon or self.horizon)
                halo = max(band, self._band_floor, halo or 0.0)
                owner = _cut(self.snap_pos, self.t.world, self.plan.axis, self._weights)[2]
                self._spheres = Spheres.around(self.snap_pos, sid, srad * self._sphere_scale, owner)
            else:
                halo = self.plan.halo if halo is None else halo
            plan = SlabPlan.build(self.snap_pos, self.t.world, halo, axis=self.plan.axis, weights=self._weights,
                                  spheres=self._spheres)
        self._setup(plan, state)

    def _any_rank(self, flag: bool) -> bool:
        """Does any rank raise `flag`?  Through libpcd's communicator (pcd_allreduce_scalars) on the native path."""
        if self.t.world == 1:
            return flag
        if self.native:
            f = torch.tensor([1 if flag else 0], dtype=torch.int32, device=nat.device())
            self.comm.allreduce_(f, nat.OP_MAX)
            return bool(f.item())
        f = torch.tensor([1 if flag else 0], dtype=torch.int32)
        self.t.all_reduce(f, "max")
        return bool(f.item())

    def _max_over_ranks(self, vals):
        """Element-wise max of a few float32 scalars over the ranks (libpcd's communicator on the native path)."""
        if self.t.world == 1:
            return list(vals)
        if self.native:
            t = torch.tensor(vals, dtype=torch.float32, device=nat.device())
            self.comm.allreduce_(t, nat.OP_MAX)
        else:
            t = torch.tensor(vals, dtype=torch.float32)
            self.t.all_reduce(t, "max")
        return [float(x) for x in t.cpu()]

    def _growth(self):
        """What the failed coverage checks lacked (max over the ranks): the new band and the spheres' factor.  A
        sphere-less row whose ball left the band box widens the band by 1.5 x its reach past it (at least x 1.1); a
        sphere row that left its sphere grows every sphere by 1.25 x its ratio; what did not fail stays.  Engines
        without the diagnostics (the CPU oracle engine) widen both by halo_growth."""
        bits = self.e.status()
        have = hasattr(self.e, "coverage_excess")
        b, s = self.e.coverage_excess() if have else (0.0, 0.0)
        band_fail, sph_fail = float(bool(bits & 4)), float(bool(bits & 8))
        band_fail, sph_fail, b, s, have = self._max_over_ranks([band_fail, sph_fail, b, s, 1.0 if have else 0.0])
        if not have:
            return self.halo * self.halo_growth, self.halo_growth, {"legacy_growth": self.halo_growth}
        halo = max(self.halo * 1.1, self.halo + 1.5 * b) if band_fail else self.halo
        scale = 1.25 * max(s, 1.0) if sph_fail else None
        return halo, scale, {"band_failed": bool(band_fail), "band_excess": b, "sphere_failed": bool(sph_fail),
                             "sphere_ratio": s}

    def _verify(self):
        """Coverage check of the iterations since the checkpoint; on a thin halo: restore the checkpoint, grow what
        failed, re-plan and replay them."""
        while self._any_rank(bool(self.e.status() & 2)):
            if self.replans >= self.max_replans:
                raise nat.PcdError(f"pcd_slab: halo still too thin after {self.replans} re-plans "
                                   f"(halo {self.halo:.4g})")
            halo, scale, why = self._growth()
            self._band_floor = max(self._band_floor, halo)
            if scale is not None:
                self._sphere_scale *= scale
            # (the checkpoint is in the order of the plan it was taken under: gathered before the re-cut)
            gstate = self._global_state(*self._ckpt)
            before = self.halo
            self._replan(halo if self.t.rank == 0 else None, state=gstate,
                         sphere_scale=scale if self.t.rank == 0 else None, at=self._ckpt_iter,
                         horizon=max(self.horizon, len(self._pending)))
            self.replan_log.append(dict(why, reason="coverage", halo_before=before, halo_after=self.halo,
                                        sphere_scale=scale))
            if self.t.rank == 0:
                import sys
                print(f"pcd_slab: coverage re-plan {self.replans + 1}: {self.replan_log[-1]}", file=sys.stderr,
                      flush=True)
            self.replans += 1
            self._ckpt = self._owned_state_now()            # the restored checkpoint, in the new plan's order
            for p in self._pending:
                self._one(p)
        self._pending = []

    # -------------------------------------------------------------------------------- iteration
    def _exchange(self, fld):
        sends = {p: self.e.pack(fld, rows) for p, rows in self.send_rows.items()}
        shapes = {p: (rows.numel(), 4) for p, rows in self.recv_rows.items()}
        dev = next(iter(self.recv_rows.values())).device if self.recv_rows else None
        got = self.t.exchange(sends, shapes, dev)
        for p, data in got.items():
            self.e.unpack(fld, self.recv_rows[p], data)

    def _phases(self, params):
        e, t = self.e, self.t
        for ph in range(params.nphases):
            if params.phase_kind[ph] in (nat.STEP_FLAT, nat.STEP_NEW):
                red4 = e.red4
                e.stage(params, nat.STAGE_PHASE_SUM, ph, red4)
                t.all_reduce(red4, "sum")
                e.stage(params, nat.STAGE_PHASE_CENTRE, ph, red4)
                red1 = e.red1
                e.stage(params, nat.STAGE_PHASE_MAXDIST, ph, red1)
                t.all_reduce(red1, "max")
                e.stage(params, nat.STAGE_PHASE_APPLY, ph, red1)
            else:
                e.stage(params, nat.STAGE_PHASE_APPLY, ph, None)
            if not params.jacobi:          # Gauss-Seidel: the next phase reads these positions
                self._exchange(nat.FIELD_POS)

    def _one(self, params):
        e = self.e
        if self.native:
            e.slab_iterate(self.comm, params, 1)
            return
        e.stage(params, nat.STAGE_KNN_NVT1)
        self._exchange(nat.FIELD_FN)
        e.stage(params, nat.STAGE_NVT2)
        self._phases(params)
        e.stage(params, nat.STAGE_FINISH)
        if params.jacobi:                  # Jacobi across classes: one position refresh per iteration
            self._exchange(nat.FIELD_POS)

    def iterate(self, params, iterations: int = 1):
        for _ in range(iterations):
            if self.check_every > 0 and self._ckpt is None:
                self._ckpt = self._owned_state_now()
                self._ckpt_iter = self.iterations_done
                self._pending = []
            self._one(params)
            self.iterations_done += 1
            if not self.step_bound:
                self.step_bound = float(params.d)     # (the drift bound of later plans: every move is below d)
            if self.check_every > 0:
                self._pending.append(params)
                self._since += 1
                if self._since >= self.check_every:
                    self.verify()

    def verify(self):
        """Check the iterations since the last checkpoint now (re-planning and replaying them on a thin halo); the
        next iteration takes a fresh checkpoint.  Collective."""
        if self._pending:
            self._verify()
        self._since, self._pending, self._ckpt = 0, [], None

    def checkpoint(self):
        """verify(), then checkpoint the present state at once, so that the next `check_every` iterations run
        without taking one (the bench's timed region: no host synchronisation inside it).  Collective."""
        self.verify()
        if self.check_every > 0:
            self._ckpt = self._owned_state_now()
            self._ckpt_iter = self.iterations_done

    def rebalance(self, class_weights=(1.0, 1.3, 1.4), horizon=None):
        """Re-cut the slabs by cost: each point weighs class_weights[its class in the last NVT2 stage] (flat, edge,
        corner: the edge / feature steps solve a 3x3 system over their neighbours).  Collective.  Iterations since the
        last coverage check are verified first (a thin halo there re-plans and replays them), so the state carried
        into the new cut is exact.  horizon: the iterations the new plan is sized to cover (default self.horizon)."""
        self.verify()
        cls = self.e.classes()
        cls = cls[self.owned_local.to(cls.device)]
        w_tab = torch.tensor(class_weights, dtype=torch.float32, device=cls.device)
        w_own = w_tab[cls.clamp(0, len(class_weights) - 1)]
        weights = self._gather_to0(w_own[:, None])
        before = self.halo
        self._replan(weights=None if weights is None else weights[:, 0].to(self.snap_pos.device), horizon=horizon)
        self.replan_log.append({"reason": "rebalance", "halo_before": before, "halo_after": self.halo})
        self._since, self._pending, self._ckpt = 0, [], None

    def iterate_timed(self, params) -> dict:
        """One iteration with CUDA/HIP events on the launch stream around each stage group (ms)."""
        if self.native:
            return self.e.slab_iterate_timed(self.comm, params)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
        e = self.e
        ev[0].record()
        e.stage(params, nat.STAGE_KNN_NVT1)
        ev[1].record()
        self._exchange(nat.FIELD_FN)
        ev[2].record()
        e.stage(params, nat.STAGE_NVT2)
        ev[3].record()
        self._phases(params)
        ev[4].record()
        e.stage(params, nat.STAGE_FINISH)
        if params.jacobi:
            self._exchange(nat.FIELD_POS)
        ev[5].record()
        ev[5].synchronize()
        names = ["knn_nvt1", "fn_exchange", "nvt2", "phases_with_exchange", "finish"]
        return {nm: ev[i].elapsed_time(ev[i + 1]) for i, nm in enumerate(names)}

    def check(self):
        self.e.check()

    def owned_state(self):
        """(global ids, positions, normals) of this rank's own points."""
        pos, n = self.e.store()
        idx = self.owned_local.to(pos.device)
        return self.owned_global, pos[idx], n[idx]


def _quantile(x: torch.Tensor, q: float) -> float:
    """(torch.quantile refuses inputs past 16M elements)"""
    return float(torch.sort(x).values[int(q * (x.numel() - 1))]) if x.numel() else 0.0


def cut_spheres(snap_pos: torch.Tensor, world: int, k: int, margin: float = 1.25, quantile: float = 0.999,
                axis: int | None = None, sphere_margin: float = 1.5, weights: torch.Tensor | None = None,
                query: torch.Tensor | None = None, iterations: int = 0, step: float = 0.0, horizon: int = 1,
                first_step: float = 1.75):
    """(band halo, sphere centre ids, sphere radii) for the cut SlabPlan.build makes with the same `weights` (None:
    equal counts), covering the next `horizon` iterations from the state `query` (the current positions after
    `iterations` iterations; None: the snapshot itself).  step: the loop's per-iteration displacement bound d (every
    step's move is clamped below it, Denoiser.py's `norm < d` keeps); 0 prices no drift.

    Each near-face point needs its k-ball's reach past its slab's faces now plus the growth of that reach over the
    iterations ahead; its sphere must hold |q - o| + d_k(q) over them.  Measured on configs[4]'s 80M cloud, 8 slabs
    (tools/halo_policy_probe.py, profiles/r6/halo_policy_probe_25_80m_r6.txt), after the first iteration, j iterations
    ahead: both grow INDEPENDENTLY of how fast the point moved so far; the reach by ~0.16 d j at the 0.999-quantile
    and ~2 d sqrt(j) at most, |q - o| + d_k by ~2.35 d sqrt(j) at most (j = 2 .. 23); the first iteration moves the
    fastest points by up to 1.7 d.  So, with ahead = horizon - 1 and lead = first_step before any iteration (else 0):
    need = reach + d (lead + 0.8 sqrt(ahead) + 0.2 ahead); the band is `margin` x the `quantile` of the needs (at least
    the median d_k); every point that needs more keeps a sphere around its snapshot position o (all its snapshot
    members local to its owner) of radius max(sphere_margin x d_k, 1.1 x (|q - o| + d_k + d (lead + 2.4 sqrt(ahead)))).
    A cost-weighted re-cut moves the faces, so the band and the spheres are recomputed for it (SlabDenoiser._replan)."""
    idx, reach, dk, disp = _cut_reach(snap_pos, world, k, axis, weights, query=query)
    if idx.numel() == 0:
        z = torch.zeros(0, dtype=torch.int64)
        return 0.0, z, torch.zeros(0)
    ahead = max(int(horizon) - 1, 0)
    lead = first_step if (iterations == 0 and ahead > 0) else 0.0
    grow_b = float(step) * (lead + 0.8 * math.sqrt(ahead) + 0.2 * ahead)
    grow_s = float(step) * (lead + 2.4 * math.sqrt(ahead))
    need = (reach + grow_b).clamp(min=0)
    band = margin * max(_quantile(need, quantile), _quantile(dk, 0.5))
    out = margin * need > band
    radii = torch.maximum(sphere_margin * dk, 1.1 * (disp + dk + grow_s))
    return band, idx[out], radii[out]


def _cut_reach(snap_pos: torch.Tensor, world: int, k: int, axis: int | None = None,
               weights: torch.Tensor | None = None, chunk: int = 8_000_000, query: torch.Tensor | None = None):
    """Per point near a face of the cut (_cut with `weights`): (global id, reach of its k-ball past its slab's faces,
    d_k, displacement from the snapshot), the ball centred at its `query` position (None: the snapshot; the kNN is
    over the snapshot, as K1 searches).  'Near' = within default_halo of a face (the sampled bound, the quantile's
    population) OR any point whose own k-ball crosses a face: d_k comes from every point (in chunks), so a sparse
    outlier far from a face with a ball past it -- which a sampled bound misses -- is priced too (round 6: the 80M /
    8-rank rehearsal's first iteration failed its coverage check on such points)."""
    dev = nat.device()
    pos = snap_pos.to(dev)
    qpos = pos if query is None else query.to(dev, torch.float32)
    axis, key, rank_of, lo, hi = _cut(pos, world, axis, None if weights is None else weights.to(dev))
    band = default_halo(pos, k)
    lo_t = torch.tensor(lo, device=dev, dtype=key.dtype)[rank_of]
    hi_t = torch.tensor(hi, device=dev, dtype=key.dtype)[rank_of]
    first, last = rank_of == 0, rank_of == world - 1
    g = nat.Grid(pos, k_hint=k)
    n = pos.size(0)
    dk = torch.empty(n, dtype=torch.float32, device=dev)
    for c0 in range(0, n, chunk):
        _, d2 = g.knn(qpos[c0:c0 + chunk].contiguous(), k, with_d2=True, idx_bits=32)
        dk[c0:c0 + chunk] = d2[:, -1].sqrt()
        del d2
    qk = qpos[:, axis]
    up = torch.where(last, torch.zeros_like(dk), qk + dk - hi_t)
    down = torch.where(first, torch.zeros_like(dk), lo_t - qk + dk)
    reach = torch.maximum(up, down)
    near = ((qk > hi_t - band) & ~last) | ((qk < lo_t + band) & ~first) | (reach > 0)
    idx = torch.nonzero(near).flatten()
    disp = torch.zeros(idx.numel(), dtype=torch.float32, device=dev) if query is None else \
        (qpos[idx] - pos[idx]).norm(dim=1)
    return idx, reach[idx], dk[idx], disp


def cut_halo(snap_pos: torch.Tensor, world: int, k: int, margin: float = 1.25, axis: int | None = None,
             weights: torch.Tensor | None = None) -> float:
    """The halo the equal-count cut into `world` slabs needs at the snapshot, times `margin` for the drift of later
    iterations: every snapshot point's k-ball (radius d_k, its k-th neighbour distance) must lie inside its slab
    widened by the halo on the cut axis, so the halo is the largest reach of a ball past its slab's faces,
    max_q (q + d_k(q) - hi_r, lo_r - q + d_k(q)) over the points near a face.  The balls that reach farthest belong
    to the sparsest points near a cut (noise outliers), which default_halo's sample maximum prices everywhere three
    times over.  Only the points within default_halo of a face are searched.  The coverage check still reports any
    later ball that leaves the halo (a re-plan widens it)."""
    if world == 1:
        return 0.0
    idx, reach, _, _ = _cut_reach(snap_pos, world, k, axis, weights)
    if idx.numel() == 0:
        return 0.0
    return margin * float(reach.max().clamp(min=0))


def default_halo(snap_pos: torch.Tensor, k: int, sample: int = 65536, factor: float = 3.0) -> float:
    """factor x the largest k-th neighbour distance over an even sample of snapshot points (queries are current
    positions, which drift from the snapshot; the coverage check reports a halo that turns out too thin)."""
    dev = nat.device()
    pos = snap_pos.to(dev)
    g = nat.Grid(pos, k_hint=k)
    stride = max(1, pos.size(0) // sample)
    q = pos[::stride].contiguous()
    _, d2 = g.knn(q, k, with_d2=True)
    return factor * math.sqrt(float(d2[:, -1].max()))


def gather_global(state, n_total: int, transport) -> tuple:
    """All-gather every rank's (ids, pos, n) into global arrays (tests / final output)."""
    ids, pos, n = state
    if transport.world == 1:
        out_p = torch.empty((n_total, 3), dtype=pos.dtype, device=pos.device)
        out_n = torch.empty_like(out_p)
        out_p[ids.to(pos.device)] = pos
        out_n[ids.to(pos.device)] = n
        return out_p, out_n
    dist = transport.dist
    pay = torch.cat([ids.to(torch.float64)[:, None], pos.double(), n.double()], 1)
    dev = "cpu" if transport.host else pay.device
    pay = pay.to(dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(transport.world)]
    dist.all_gather(sizes, torch.tensor([pay.size(0)], dtype=torch.int64, device=dev), transport.group)
    mx = int(max(s.item() for s in sizes))
    padded = torch.zeros((mx, 7), dtype=torch.float64, device=dev)
    padded[: pay.size(0)] = pay
    bufs = [torch.zeros_like(padded) for _ in range(transport.world)]
    dist.all_gather(bufs, padded, transport.group)
    out_p = torch.empty((n_total, 3), dtype=torch.float32)
    out_n = torch.empty_like(out_p)
    for b, s in zip(bufs, sizes):
        b = b[: int(s.item())].cpu()
        gi = b[:, 0].long()
        out_p[gi] = b[:, 1:4].float()
        out_n[gi] = b[:, 4:7].float()
    return out_p, out_n


# ----------------------------------------------------------------------------------------------- mesh update
class HipMeshEngine:
    """Mesh.updateVertices' Jacobi sweep (pcd_mesh_update / pcd_mesh_update_f32) over one rank's local mesh: the
    faces incident to its own vertices (ascending global face id) and every vertex of those faces."""

    def __init__(self, v, f, fn, fp32=True):
        dev = nat.device()
        self.fp32 = bool(fp32)
        dt, it = (torch.float32, torch.int32) if fp32 else (torch.float64, torch.int64)
        self.v = v.to(dev, dt).contiguous()
        self.f = f.to(dev, it).contiguous()
        self.fn = fn.to(dev, dt).contiguous()
        self.vf, self.ni = nat.mesh_vta(self.f, self.v.size(0), out_dtype=it)

    def sweep(self):
        (nat.mesh_update_f32 if self.fp32 else nat.mesh_update)(self.v, self.f, self.fn, self.vf, self.ni, 1)


class MeshSlabs:
    """Mesh.updateVertices (PatchGeneration/Modules/Mesh.py:377-418) over vertex slabs, one rank per GPU (SURVEY.md
    §8(e): the mesh update shards by vertex ownership).

    Rank 0, the coordinator, holds the mesh (v [nv, 3], f [nf, 3], face normals fn [nf, 3]; the other ranks pass None)
    and cuts the vertices into slabs of equal count along the longest bbox axis.  Rank r owns the vertices of slab r;
    its local mesh is every face incident to an owned vertex (in ascending global face id, so each vertex sums its
    faces in the reference's order) and every vertex of those faces -- the owned ones plus a one-ring halo.  A sweep
    is the Jacobi update of the local mesh, then the halo rows are refreshed from their owners (point-to-point to the
    slab neighbours).  An owned vertex sees all of its faces and the previous sweep's positions of their corners, so
    the owned rows equal the one-GPU sweep bit for bit (fp64 and fp32).  engine_factory(v, f, fn) -> an object with
    `v` (local rows, updated in place) and `sweep()`: the HIP engine by default (the CPU tests use the oracle's)."""

    def __init__(self, v, f, fn, transport=None, fp32=True, engine_factory=None, native=None):
        self.t = transport or LocalTransport()
        rank, world = self.t.rank, self.t.world
        self.native = (engine_factory is None) if native is None else bool(native)
        self.comm = self.t.native_comm() if (self.native and world > 1) else None
        dev = nat.device() if engine_factory is None else torch.device("cpu")
        self.dev = dev
        share = None
        if rank == 0:
            v, f, fn = torch.as_tensor(v), torch.as_tensor(f).long(), torch.as_tensor(fn)
            nv = v.size(0)
            assert world >= 1 and nv >= world, "need at least one vertex per rank"
            vd = v.to(dev)
            axis = int(torch.argmax(vd.max(0).values - vd.min(0).values))
            order = torch.sort(vd[:, axis].contiguous(), stable=True).indices
            owner = torch.empty(nv, dtype=torch.int64, device=dev)
            for r in range(world):
                owner[order[(r * nv) // world:((r + 1) * nv) // world]] = r
            fdev, fndev = f.to(dev), fn.to(dev)
            fown = owner[fdev]                                           # [nf, 3]
            shares = []
            for r in range(world):
                faces = torch.nonzero((fown == r).any(1)).flatten()      # ascending global face id
                # ascending global vertex id: the corners of those faces and every owned vertex (an isolated one has
                # no face: degree 0, the reference's 0 / 0)
                lverts = torch.unique(torch.cat([fdev[faces].flatten(), torch.nonzero(owner == r).flatten()]))
                to_local = torch.full((nv,), -1, dtype=torch.int64, device=dev)
                to_local[lverts] = torch.arange(lverts.numel(), device=dev)
                shares.append((lverts, faces, to_local))
            self.owner, self.n_total = owner, nv
            for r in range(world):
                lverts, faces, to_local = shares[r]
                peers, send_l, recv_l = [], [], []
                for q in range(world):
                    if q == r:
                        continue
                    lq = shares[q][0]
                    out = lq[owner[lq] == r]                             # mine, held by q
                    inc = lverts[owner[lverts] == q]                     # q's, held by me
                    if out.numel() or inc.numel():
                        peers.append(q)
                        send_l.append(to_local[out])
                        recv_l.append(to_local[inc])
                pkg = (lverts, torch.nonzero(owner[lverts] == r).flatten(), to_local[fdev[faces]],
                       vd[lverts], fndev[faces], peers, send_l, recv_l)
                if r == 0:
                    share = pkg
                else:
                    self._send_pkg(pkg, r)
        else:
            share = self._recv_pkg()
            self.owner, self.n_total = None, None
        lverts, owned, lf, lv, lfn, self.peers, self.send_local, self.recv_local = share
        self.local, self.owned_local = lverts, owned
        self.owned_global = lverts[owned]
        if self.n_total is None:
            self.n_total = -1
        self.e = (engine_factory or (lambda a, b, c: HipMeshEngine(a, b, c, fp32)))(lv, lf, lfn)
        self.halo_rows = sum(int(x.numel()) for x in self.recv_local)

    # -- coordinator -> rank (the mesh share), as pcd_slab.SlabDenoiser hands out its slabs
    def _p2p_send(self, t, dst):
        if self.comm is not None:
            self.comm.sendrecv(dst, t.contiguous().to(nat.device()), -1, None)
        else:
            self.t.send(t, dst)

    def _p2p_recv(self, shape, dtype, src):
        if self.comm is not None:
            return self.comm.sendrecv(-1, None, src, torch.empty(shape, dtype=dtype, device=nat.device()))
        return self.t.recv(torch.empty(shape, dtype=dtype, device=self.dev), src)

    def _send_pkg(self, pkg, dst):
        lverts, owned, lf, lv, lfn, peers, send_l, recv_l = pkg
        ints = torch.cat([x.to(self.dev, torch.int64).flatten() for x in
                          [lverts, owned, lf, torch.tensor(peers, dtype=torch.int64),
                           torch.tensor([x.numel() for x in send_l], dtype=torch.int64),
                           torch.tensor([x.numel() for x in recv_l], dtype=torch.int64)] + send_l + recv_l])
        rows = torch.cat([lv.to(self.dev, torch.float64).flatten(), lfn.to(self.dev, torch.float64).flatten()])
        head = torch.tensor([lverts.numel(), owned.numel(), lf.size(0), len(peers), ints.numel(), rows.numel(), 0, 0],
                            dtype=torch.int64)
        for t in (head, ints, rows):
            self._p2p_send(t, dst)

    def _recv_pkg(self):
        nl, no, nf, npeers, nints, nrows = self._p2p_recv((8,), torch.int64, 0).cpu().tolist()[:6]
        ints = self._p2p_recv((nints,), torch.int64, 0).to(self.dev)
        rows = self._p2p_recv((nrows,), torch.float64, 0).to(self.dev)
        o = 0
        lverts, o = ints[o:o + nl], o + nl
        owned, o = ints[o:o + no], o + no
        lf, o = ints[o:o + 3 * nf].view(nf, 3), o + 3 * nf
        peers, o = ints[o:o + npeers].tolist(), o + npeers
        ns, o = ints[o:o + npeers].tolist(), o + npeers
        nr, o = ints[o:o + npeers].tolist(), o + npeers
        send_l, recv_l = [], []
        for c in ns:
            send_l.append(ints[o:o + c])
            o += c
        for c in nr:
            recv_l.append(ints[o:o + c])
            o += c
        lv, lfn = rows[:3 * nl].view(nl, 3), rows[3 * nl:].view(nf, 3)
        return lverts, owned, lf, lv, lfn, peers, send_l, recv_l

    # -- sweeps
    def _exchange(self):
        """Halo rows from their owners, peer by peer in ascending rank (no cycle of blocking pairs)."""
        v = self.e.v
        for q, peer in enumerate(self.peers):
            out = v[self.send_local[q].to(v.device)].contiguous()
            inc = torch.empty((self.recv_local[q].numel(), 3), dtype=v.dtype, device=v.device)
            if self.comm is not None:
                self.comm.sendrecv(peer if out.numel() else -1, out if out.numel() else None,
                                   peer if inc.numel() else -1, inc if inc.numel() else None)
            else:
                dist = self.t.dist
                ops = []
                hi = torch.empty(inc.shape, dtype=inc.dtype)
                if inc.numel():
                    ops.append(dist.P2POp(dist.irecv, hi, peer, self.t.group))
                if out.numel():
                    ops.append(dist.P2POp(dist.isend, out.cpu(), peer, self.t.group))
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
                inc = hi.to(v.device)
            if inc.numel():
                v[self.recv_local[q].to(v.device)] = inc

    def update(self, k=15):
        """k Jacobi sweeps (Mesh.updateVertices' loop), each followed by the halo refresh."""
        for _ in range(int(k)):
            self.e.sweep()
            if self.t.world > 1:
                self._exchange()

    def owned_state(self):
        """(global vertex ids, positions) of this rank's own vertices."""
        return self.owned_global, self.e.v[self.owned_local.to(self.e.v.device)]
