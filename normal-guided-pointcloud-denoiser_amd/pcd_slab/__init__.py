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

    @staticmethod
    def build(snap: torch.Tensor, world: int, halo: float, axis: int | None = None,
              weights: torch.Tensor | None = None) -> "SlabPlan":
        """weights (optional, [N] >= 0, identical on every rank): cut at quantiles of the cumulative weight along the
        axis instead of equal point counts (each rank still owns at least one point)."""
        snap = snap.detach()
        n = snap.size(0)
        assert world >= 1 and n >= world, "need at least one point per rank"
        ext = snap.max(0).values - snap.min(0).values
        if axis is None:
            axis = int(torch.argmax(ext).item())
        key = snap[:, axis].contiguous()
        order = torch.sort(key, stable=True).indices           # ties by index: deterministic on every rank
        owner = torch.empty(n, dtype=torch.int64, device=snap.device)
        if weights is None:
            bounds = [(r * n) // world for r in range(world + 1)]
        else:
            cw = torch.cumsum(weights.to(snap.device, torch.float64)[order], 0)
            tot = float(cw[-1])
            cuts = torch.tensor([tot * r / world for r in range(1, world)], dtype=torch.float64, device=snap.device)
            inner = torch.searchsorted(cw, cuts).tolist() if world > 1 else []
            bounds = [0] + [int(b) for b in inner] + [n]
            for r in range(1, world + 1):                       # at least one point per rank, monotone
                bounds[r] = min(max(bounds[r], bounds[r - 1] + 1), n - (world - r))
        lo, hi, local = [], [], []
        for r in range(world):
            owner[order[bounds[r]:bounds[r + 1]]] = r
        for r in range(world):
            ks = key[order[bounds[r]:bounds[r + 1]]]
            lo.append(float(ks[0]))
            hi.append(float(ks[-1]))
        for r in range(world):
            inside = (key >= lo[r] - halo) & (key <= hi[r] + halo)
            local.append(torch.nonzero(inside | (owner == r)).flatten())
        return SlabPlan(world, axis, float(halo), owner, lo, hi, local)

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
    """Halo exchange and scalar all-reduces over torch.distributed: NCCL (= RCCL on ROCm, over xGMI) moves device
    tensors directly; gloo stages through host memory.  With NCCL, Work.wait() only makes the current (launch) stream
    wait for the communication stream -- the exchanges stay stream-ordered and the host is not blocked; the halo
    costs are measured per stage by SlabDenoiser.iterate_timed (fn_exchange, phases_with_exchange)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host = dist.get_backend(group) == "gloo"

    def exchange(self, sends: dict, recv_shapes: dict, device) -> dict:
        """sends: peer -> tensor; recv_shapes: peer -> shape.  Returns peer -> received tensor on `device`."""
        dist = self.dist
        ops, outs, staged = [], {}, {}
        for peer, shape in recv_shapes.items():
            buf = torch.empty(shape, dtype=torch.float32, device="cpu" if self.host else device)
            outs[peer] = buf
            ops.append(dist.P2POp(dist.irecv, buf, peer, self.group))
        for peer, t in sends.items():
            staged[peer] = t.cpu() if self.host else t.contiguous()
            ops.append(dist.P2POp(dist.isend, staged[peer], peer, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return {p: (b.to(device) if self.host else b) for p, b in outs.items()}

    def native_comm(self) -> "nat.Comm":
        """libpcd's transport for pcd_slab_iterate (collective): an RCCL communicator of its own when this group is
        NCCL (= RCCL), else host callbacks over this (gloo) group -- the same library code path, each exchange staged
        through pinned host memory."""
        dist, grp = self.dist, self.group
        if not self.host:
            return nat.Comm.rccl(self.world, self.rank, lambda t: self.broadcast_(t.to(nat.device()), 0).cpu())

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

        return nat.Comm.host(self.world, self.rank, exchange, allreduce)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.host and t.device.type != "cpu":
            h = t.cpu()
            self.dist.broadcast(h, src, self.group)
            t.copy_(h)
        else:
            self.dist.broadcast(t, src, self.group)
        return t

    def all_reduce(self, t: torch.Tensor, op: str) -> torch.Tensor:
        dist = self.dist
        red = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op]
        if self.host and t.device.type != "cpu":
            h = t.cpu()
            dist.all_reduce(h, red, self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, red, self.group)
        return t


class LocalTransport:
    """world = 1: nothing to exchange."""
    rank, world = 0, 1

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

    def __init__(self, local_pos, local_n, owned_local, k_max, origin, cell, coverage, seeding=True):
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

    # the one-call iteration (pcd_slab_iterate)
    native = True

    def set_routes(self, peers, send_rows, recv_rows, own_lo, own_hi):
        self.fused.set_routes(peers, send_rows, recv_rows, own_lo, own_hi)

    def slab_iterate(self, comm, params, iterations=1):
        self.fused.slab_iterate(comm, params, iterations)

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
class SlabDenoiser:
    """The body of Processor.denoise (Processor.py:119-139) over spatial slabs, one rank per GPU.

    snap_pos / snap_n: the WHOLE cloud (the frozen snapshot is the initial positions, as in Selector.__init__);
    rank 0's copy is broadcast, so every rank plans from identical data and keeps it (the frozen snapshot a re-plan
    cuts again).  halo: slab widening in snapshot units (None: 3x the largest k-th neighbour distance of a sample,
    see default_halo, estimated on rank 0 and broadcast).  check_every: iterations between coverage checks
    (0: never -- check() raises at the caller's request instead); halo_growth / max_replans: the thin-halo
    recovery."""

    def __init__(self, snap_pos, snap_n, k_max, transport=None, halo=None, engine_factory=None, seeding=True,
                 k_hint=None, check_every=1, halo_growth=2.0, max_replans=4, weights=None, native=None):
        """native: one pcd_slab_iterate call per iteration over libpcd's own transport (default for the HIP engine);
        False: the same stages driven from Python over torch.distributed."""
        self.t = transport or LocalTransport()
        rank, world = self.t.rank, self.t.world
        if world > 1:
            snap_pos = self.t.broadcast_(snap_pos.contiguous().clone())
            snap_n = self.t.broadcast_(snap_n.contiguous().clone())
        if halo is None:
            # one rank grids the whole cloud for the estimate and broadcasts it (every rank planning from the same
            # value; the others never build a grid over the global cloud)
            h = torch.zeros(1, dtype=torch.float64, device=snap_pos.device)
            if rank == 0:
                h.fill_(default_halo(snap_pos, k_max))
            halo = float(self.t.broadcast_(h)) if world > 1 else float(h)
        self.snap_pos, self.snap_n = snap_pos, snap_n
        # cell lattice of the ranks' snapshot indices: the fused loop's (pcd_native.fused_k_hint) unless given
        self.k_max, self.k_hint, self.seeding = k_max, k_hint or nat.fused_k_hint(k_max) or 32, seeding
        self.engine_factory = engine_factory
        self.native = (engine_factory is None) if native is None else bool(native)
        self.comm = self.t.native_comm() if self.native else None
        self.check_every, self.halo_growth, self.max_replans = int(check_every), float(halo_growth), int(max_replans)
        self.replans = 0
        self.e = None
        self._lattice = None
        self._setup(SlabPlan.build(snap_pos, world, halo, weights=weights))
        self._since = 0            # iterations since the last checkpoint
        self._pending = []         # their params (replayed after a re-plan)
        self._ckpt = None

    # -------------------------------------------------------------------------------- plan -> engine + routes
    def _setup(self, plan, state=None):
        """Build this rank's engine and halo routes for `plan`; state = (global pos, global n) of the CURRENT
        iterate to take over (None: the snapshot itself, i.e. a fresh start)."""
        rank, world = self.t.rank, self.t.world
        self.plan = plan
        self.local = plan.local[rank]                           # global ids, ascending
        pos_l, n_l = self.snap_pos[self.local], self.snap_n[self.local]
        owned_mask = plan.owner[self.local] == rank
        self.owned_local = torch.nonzero(owned_mask).flatten()
        self.owned_global = self.local[self.owned_local]
        self.e = None                                           # free the old engine's device state first
        if self.engine_factory is None:
            if self._lattice is None:
                self._lattice = nat.grid_params(self.snap_pos.to(nat.device()), k_hint=self.k_hint)
            origin, cell = self._lattice
            self.e = HipSlabEngine(pos_l, n_l, self.owned_local, self.k_max, origin, cell, plan.coverage(rank),
                                   self.seeding)
        else:
            self.e = self.engine_factory(pos_l, n_l, self.owned_local, self.k_max, plan.coverage(rank))
        if state is not None:
            # the engine loaded the snapshot (its `orig` for the global clamp); the current iterate goes on top
            lid = torch.arange(self.local.numel(), device=self.local.device)
            self.e.set_state(lid, state[0][self.local.to(state[0].device)], state[1][self.local.to(state[1].device)])
        # halo routes: rows I send to each peer and rows I receive from it (both ascending global index)
        to_local = torch.full((self.snap_pos.size(0),), -1, dtype=torch.int64, device=self.local.device)
        to_local[self.local] = torch.arange(self.local.numel(), device=self.local.device)
        self.send_rows, self.recv_rows = {}, {}
        for peer in range(world):
            if peer == rank:
                continue
            out = plan.transfer(rank, peer)
            inc = plan.transfer(peer, rank)
            if out.numel():
                self.send_rows[peer] = self.e.rows(to_local[out])
            if inc.numel():
                self.recv_rows[peer] = self.e.rows(to_local[inc])
        self.halo_points = sum(r.numel() for r in self.recv_rows.values())
        if self.native:
            # routes + the OWNED slab (the rows whose k-ball stays strictly inside it read no halo row: NVT2 / the
            # phases run them while an exchange is in flight).  Strict bounds: a snapshot point ON a cut may be owned
            # by the neighbour, so the box is shrunk by one float32 ulp on the cut faces.
            import numpy as np
            big = 3.0e38
            lo, hi = [-big] * 3, [big] * 3
            if rank > 0:
                lo[plan.axis] = float(np.nextafter(np.float32(plan.lo[rank]), np.float32(np.inf)))
            if rank < world - 1:
                hi[plan.axis] = float(np.nextafter(np.float32(plan.hi[rank]), np.float32(-np.inf)))
            peers = sorted(set(self.send_rows) | set(self.recv_rows))
            empty = torch.zeros(0, dtype=torch.int32, device=nat.device())
            self.e.set_routes(peers, [self.send_rows.get(q, empty) for q in peers],
                              [self.recv_rows.get(q, empty) for q in peers], lo if peers else None,
                              hi if peers else None)

    def _owned_state_now(self):
        """(pos, n) of this rank's own points, owned-local order (a checkpoint)."""
        rows = self.e.rows(self.owned_local)
        return self.e.pack(nat.FIELD_POS, rows)[:, :3].clone(), self.e.pack(nat.FIELD_NRM, rows)[:, :3].clone()

    def _gather_owned(self, x: torch.Tensor) -> torch.Tensor:
        """Per-point values of this rank's own points (owned-local order, [n_own, c] float32) -> the global [N, c]
        on every rank.  Every rank knows the others' owned ids from the plan, so only the values travel (padded
        all-gather).  Collective."""
        n_tot = self.snap_pos.size(0)
        dev = x.device
        out = torch.empty((n_tot, x.size(1)), dtype=torch.float32, device=dev)
        if self.t.world == 1:
            out[self.owned_global.to(dev)] = x
            return out
        counts = torch.bincount(self.plan.owner, minlength=self.t.world).tolist()
        cdev = "cpu" if self.t.host else dev
        pay = torch.zeros((max(counts), x.size(1)), dtype=torch.float32, device=cdev)
        pay[: x.size(0)] = x.to(cdev)
        bufs = [torch.empty_like(pay) for _ in range(self.t.world)]
        self.t.dist.all_gather(bufs, pay, self.t.group)
        for r, b in enumerate(bufs):
            ids = torch.nonzero(self.plan.owner == r).flatten().to(dev)
            out[ids] = b[: counts[r]].to(dev)
        return out

    def _global_state(self, owned_pos, owned_n):
        g = self._gather_owned(torch.cat([owned_pos, owned_n], 1))
        return g[:, :3], g[:, 3:]

    def _replan(self, halo=None, weights=None, state=None):
        """Re-cut every rank from the frozen snapshot, taking over `state` (global current pos, n; default: the
        present iterate).  Collective: all ranks call it together."""
        if state is None:
            state = self._global_state(*self._owned_state_now())
        halo = self.plan.halo if halo is None else halo
        self._setup(SlabPlan.build(self.snap_pos, self.t.world, halo, axis=self.plan.axis, weights=weights), state)

    def _any_rank(self, flag: bool) -> bool:
        if self.t.world == 1:
            return flag
        dev = "cpu" if self.t.host else self.snap_pos.device
        f = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        self.t.all_reduce(f, "max")
        return bool(f.item())

    def _verify(self):
        """Coverage check of the iterations since the checkpoint; on a thin halo: restore the checkpoint, widen the
        halo, re-plan and replay them."""
        gstate = None
        while self._any_rank(bool(self.e.status() & 2)):
            if self.replans >= self.max_replans:
                raise nat.PcdError(f"pcd_slab: halo still too thin after {self.replans} re-plans "
                                   f"(halo {self.plan.halo:.4g})")
            if gstate is None:                  # (the checkpoint is in the order of the plan it was taken under)
                gstate = self._global_state(*self._ckpt)
            self._replan(self.plan.halo * self.halo_growth, state=gstate)
            self.replans += 1
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
            if self.check_every > 0 and self._since == 0:
                self._ckpt = self._owned_state_now()
                self._pending = []
            self._one(params)
            if self.check_every > 0:
                self._pending.append(params)
                self._since += 1
                if self._since >= self.check_every:
                    self._verify()
                    self._since = 0

    def rebalance(self, class_weights=(1.0, 1.3, 1.4)):
        """Re-cut the slabs by cost: each point weighs class_weights[its class in the last NVT2 stage] (flat, edge,
        corner: the edge / feature steps solve a 3x3 system over their neighbours).  Collective.  Iterations since the
        last coverage check are verified first (a thin halo there re-plans and replays them), so the state carried
        into the new cut is exact."""
        if self.check_every > 0 and self._since > 0:
            self._verify()
        cls = self.e.classes()
        cls = cls[self.owned_local.to(cls.device)]
        w_tab = torch.tensor(class_weights, dtype=torch.float32, device=cls.device)
        w_own = w_tab[cls.clamp(0, len(class_weights) - 1)]
        weights = self._gather_owned(w_own[:, None])[:, 0].to(self.snap_pos.device)
        self._replan(weights=weights)
        self._since, self._pending = 0, []

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
