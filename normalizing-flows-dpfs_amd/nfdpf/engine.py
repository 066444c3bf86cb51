"""Filtering driver: DPF.filtering_pos (DPFs.py:144-216) on the HIP path.

Per time step the tiled pipeline ``nfdpf_filter_step_tiled`` (two launches at C2: gate +
resampling + motion + nf_dyn inverse, then proposal + nf_dyn forward + densities +
measurement; the normalisation of step t is deferred into step t+1) or the one-workgroup-per-
row ``nfdpf_filter_step``, preceded by the Sinkhorn launches when the OT gate fires.
Histories are preallocated (B, T, N, .) tensors written in place (the reference grows them
with torch.cat, O(T^2) copies).  In device-RNG mode the ESS gate never syncs the host: each
step's launches read the previous step's per-(row, tile) softmax partials from device memory.

Batch sharding (world size > 1, rows [rank B, (rank + 1) B) per rank):
  * soft resampling: the pass runs speculatively with every gate assumed off and no exchange,
    then ONE all-gather of all steps' partials verifies the T batch-global gates
    (DPFs.py:163-165); a fired gate reruns the pass with a per-step all-gather;
  * OT: a per-step all-gather of the partials feeds the gate (or the speculative pass, as
    above), and each Sinkhorn call runs its rows with the local stop rule keeping every
    state's potentials, takes the MIN of the stop iteration over ranks (resamplers.py:126-129)
    and finishes at that state (ops.ot_resample_sharded: no iteration runs twice);
  * one all-reduce of the obs-likelihood sums at the end.
"""
from __future__ import annotations

import ctypes
import math
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from . import ops
from .pack import (blob, cglow_tensors, encoder_tensors, filter_flow_tensors, flows_tensors,
                   paired_mlp_tensors, pass_flow_tensors, splittable)


@dataclass
class FilterConfig:
    N: int
    NF_dyn: bool = False
    dyn_flow: str = "RealNVP"  # "RealNVP" (RealNVP_cond, [mean, std] context) or "MAF" (--NF-dyn-flow)
    NF_cond: bool = False
    measurement: str = "cos"
    resampler: str = "ot"
    alpha: float = 0.5
    eps: float = 0.1
    scaling: float = 0.75
    threshold: float = 1e-3
    max_iter: int = 100
    pos_noise: float = 20.0
    vel_noise: float = 20.0
    width: float = 128.0
    init_with_true_state: bool = False
    n_flows: int = 2
    hidden: int = 8
    meas_prior_std: float = 2.5
    rng_mode: str = "device"     # "device" (Philox on the GPU) | "host" (reference CPU generator)
    seed: int = 2
    force_resample: bool = False
    kernel: str = "tiled"        # "tiled" (multi-CU pipeline per step) | "fused" (one launch per step)
    split_nets: bool = True      # tiled: coupling nets on wave pairs (csrc/split.hpp) where the flows allow
    # sharded tiled soft pass: run every step with the ESS gate assumed off and no per-step
    # exchange, then gather all steps' softmax partials once and verify the gates (a fired
    # gate reruns the pass with the per-step exchange); None = on when the batch is sharded
    speculate_gate: Optional[bool] = None
    # the one-launch pass with the ESS gate decided INSIDE the launch at every step (one GPU, soft
    # resampler: nfdpf_filter_pass_tiled with pass_gate = 1); None / True = wherever it applies
    # and the pass is not speculated explicitly, False = never
    pass_gate: Optional[bool] = None
    # the one-launch pass following a gate PLAN -- the last exact pass's T gates, taken in advance
    # and verified after the pass from its own partials (a differing gate reruns it exactly): no
    # batch-wide exchange inside the launch, so it also runs sharded and with more rows than the
    # device holds at once.  None = where the gated pass does not apply (a sharded batch, rows
    # beyond the resident grid), True = also on one GPU in place of the gated pass, False = never
    pass_plan: Optional[bool] = None


@dataclass
class ShardInfo:
    """Batch sharding over a torch.distributed group (rows [row_base, row_base + B))."""
    world: int = 1
    rank: int = 0
    B_global: int = 0
    row_base: int = 0
    group: Optional[object] = None

    @staticmethod
    def from_env(B_local: int, group=None) -> "ShardInfo":
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            w, r = dist.get_world_size(group), dist.get_rank(group)
            return ShardInfo(w, r, B_local * w, B_local * r, group)
        return ShardInfo(1, 0, B_local, 0, None)


def density_const(pos_noise: float, d: int = 2) -> float:
    """d*log_c - 2*log(std_pos) in float32, the op order of utils.py:30-33."""
    log_c = -0.5 * torch.log(torch.tensor(2 * np.pi))
    return float(d * log_c - 2 * torch.log(torch.tensor(pos_noise)))


class HostDraws:
    """The reference's CPU-generator draws (parity mode), optionally a recorded tape."""

    def __init__(self, gen: Optional[torch.Generator] = None):
        self.gen = gen

    def init(self, start_xy, N, width, true_state):
        B = start_xy.shape[0]
        if true_state:
            return start_xy[:, None, :].cpu().repeat(1, N, 1) + torch.randn(B, N, 2, generator=self.gen)
        x = torch.tensor(width / 2.0 + width / 2.0) * torch.rand(B, N, 2, generator=self.gen) \
            + torch.tensor(-width / 2.0)
        torch.randn(B, N, 2, generator=self.gen)  # drawn and discarded (utils.py:58)
        return x

    def offsets(self, B, N):
        return torch.empty(B).uniform_(0.0, 1.0 / N, generator=self.gen)

    def noise(self, B, N, std):
        return torch.normal(mean=0.0, std=std, size=(B, N, 2), generator=self.gen)


@dataclass
class FilterResult:
    particles: torch.Tensor
    probs: torch.Tensor
    noise: torch.Tensor
    lik: torch.Tensor
    init_logw: torch.Tensor
    index: torch.Tensor
    jac: Optional[torch.Tensor]
    prior: Optional[torch.Tensor]
    obs_likelihood: torch.Tensor
    pred: torch.Tensor = None          # (B,T,2) sum_n p x, the losses.py:21 prediction
    fired: Optional[list] = None        # per-step gate (host RNG mode only)

    def as_tuple(self):
        return (self.particles, self.probs, self.noise, self.lik, self.init_logw, self.index, self.jac,
                self.prior, self.obs_likelihood)


class FilterEngine:
    """Runs the T-step particle update with the fused HIP step kernel.

    ``models`` provides ``nf_dyn``, ``cond_model``, ``particle_encoder`` and, per measurement,
    ``cnf_measurement`` (CRNVP) or ``likelihood_est`` (NN) -- the DPF module's attributes.
    """

    def __init__(self, cfg: FilterConfig, models):
        self.cfg = cfg
        self.m = models
        self.step_events = None  # list -> nfdpf.prof.EventPair around the dominant launch of step T//2 of every pass
        self._spec_backoff = 0  # auto speculative gate: passes to run per-step after the next miss / 2
        self._spec_skip = 0     # per-step passes left before speculating again
        # auto, where the gated one-launch pass applies: after a speculative pass missed (a gate
        # fired) the next passes run gated -- the gates decided inside the launch, nothing wasted
        # when they fire -- until two gated passes in a row fired none; then speculation again
        # (the speculative pass is the faster one when no gate fires: no batch-wide decision in
        # each step's critical path)
        self._gate_mode = False
        self._gate_quiet = 0
        # OT, auto mode: did the last pass resample?  Then the next one reads its gates step by
        # step (as the reference: one host sync per step); otherwise it speculates
        self._ot_fired = False
        self.last_pass_ok = False  # the last run's shapes allow the one-launch pass
        self.last_pass = False     # the last run's pass ran as one launch (nfdpf_filter_pass_tiled)
        self.pass_launches = 0     # one-launch passes run by this engine (verified or not)
        # a one-launch pass whose row hand-offs timed out (its grid was not all resident: another
        # process or kernel held CUs) turns the pass off for this engine; the step launches rerun
        self.pass_disabled = False
        # why the last run's shapes kept a pass-family configuration off the one-launch pass
        # (N above 1024, more than 256 rows), else None; warned once per engine
        self.pass_fallback_reason = None
        self._fallback_warned = False
        self._gate_resident = False  # the last run's shapes fit the gated pass (all rows resident)
        self._hmapped = None  # ops.HostMapped slots for the speculative pass's flags (lazy)
        self._shared_device = None  # per process group: does another rank use this rank's GPU?
        self.last_gate_pass = False  # the last run was the gated one-launch pass (gates decided in the launch)
        self.last_gates = None       # one shard's one-launch pass: its T gates (decided, or verified) [T] int32
        self.last_verify = None      # finish_pending's outcome: "ok", "fired" (a gate miss) or "fault"
        # gate plans (cfg.pass_plan): the T gates the next auto pass follows (np.int32, the last exact
        # or verified pass's), their device copy (one buffer, rewritten in place: a captured pass
        # reads the current plan), plan passes run / missed
        self._plan = None
        self._plan_buf, self._plan_buf_val = None, None
        self.last_plan_pass = False
        self.plan_passes = 0
        self.plan_misses = 0
        # sharded: the cross-rank gate exchange of the gated pass (ops.GateExchange), keyed by the
        # process group, B_global and device; None inside when a rank could not set it up
        self._xg = None

    def __getstate__(self):
        # DPF keeps its engine, and main.py pickles the whole DPF (main.py:57): the last pass's
        # buffers / process group and the profiling events are per-process state
        st = dict(self.__dict__)
        st.pop("_pending", None)
        st.pop("_nfdpf_pass_ws", None)
        st["last_gates"] = None
        st["_shared_device"] = None
        st["step_events"] = None
        st["_hmapped"] = None  # (pinned host memory of this process)
        st["_plan_buf"], st["_plan_buf_val"], st["_xg"] = None, None, None
        return st

    def _decide_spec(self, shard, speculate=None, host_mode=False, teacher=False, consume=False,
                     finish=True, pass_ok=False, gate_ok=False) -> bool:
        """Does the next pass run with the speculative ESS gate (every gate taken as off, the T
        gates verified once after the pass from all steps' partials, a fired gate rerunning the
        pass step by step)?  Auto mode (``speculate`` and cfg.speculate_gate None): yes for the
        tiled pipeline when the batch is sharded (one exchange per pass instead of one per step),
        for OT at any world size (its gate is read on the host before every Sinkhorn call,
        DPFs.py:165: a device->host sync per step), and wherever the whole pass runs as ONE
        persistent launch (``pass_ok``: nfdpf_filter_pass_tiled, the C2 shape; it needs every
        gate of the pass known in advance) and the gate cannot be decided inside that launch
        (``gate_ok``: one GPU, soft resampler -- the gated pass decides every gate itself, so
        nothing is speculated while the recent passes' gates fire: the engine's gate mode) -- unless
        the previous pass resampled (OT: its gates
        are then read step by step) or a recent miss is backing off (a miss costs a whole second
        pass; the next 1, 2, 4 ... 64 passes run step by step).  Not for the step-by-step soft
        resampler on one GPU: its per-step gate is device-side already, and speculating saved
        0.33 us of the front launch per step against ~30 us of verification per pass (C2, round
        3: 2.09e9 vs 2.13e9 particle-steps/s).  ``consume``: count this pass
        against the back-off (run() only).  A pass captured into a graph (``finish`` with a
        capturing stream) cannot verify its gates on the host: auto mode does not speculate
        there (run(finish=False) does, leaving finish_pending to the caller); a gated or forced
        one-launch pass captured there leaves its fault flags in the pending state instead
        (take_pending / finish_pending after each replay)."""
        c = self.cfg
        tiled = c.kernel == "tiled"
        auto = speculate is None and c.speculate_gate is None
        if speculate is None:
            speculate = c.speculate_gate if c.speculate_gate is not None else \
                (tiled and (c.resampler == "ot" or ((shard.world > 1 or pass_ok) and not (gate_ok and self._gate_mode))))
            if auto and finish and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                speculate = False
        if auto and tiled and c.resampler == "ot" and self._ot_fired:
            speculate = False  # the last pass resampled: per-step gates, no wasted speculative pass
        elif auto and speculate and self._spec_skip > 0:
            if consume:
                self._spec_skip -= 1
            speculate = False
        return bool(speculate and tiled and c.resampler in ("soft", "ot") and not host_mode and not teacher
                    and not c.force_resample and c.measurement != "CGLOW")

    def speculates(self, shard=None, finish=True) -> bool:
        """Whether run() (auto arguments, device RNG) will speculate the gates of its next pass
        (same shapes as the last run: whether the one-launch pass applies is taken from it)."""
        shard = shard or ShardInfo()
        return self._decide_spec(shard, None, self.cfg.rng_mode == "host", finish=finish,
                                 pass_ok=self.last_pass_ok, gate_ok=self._gate_ok(shard, self.last_pass_ok))

    def _gate_ok(self, shard, pass_ok) -> bool:
        """Can the one-launch pass decide the ESS gate inside the launch (the whole batch on this
        GPU, the soft resampler)?"""
        c = self.cfg
        # (the gated mode is the C2-shaped pass's, tiled_pass_kernel; the no-flow pass -- C1 / C3
        # shapes -- only speculates)
        # (and every row resident at once: the gated pass's rows wait for the batch's decision;
        # a speculative pass of more rows runs them in resident chunks)
        # (sharded: with the cross-rank gate exchange set up for this group -- _xgate)
        xg = getattr(self, "_xg", None)
        xg_ok = shard.world == 1 or (xg is not None and xg[0] == self._xg_key(shard) and xg[1] is not None)
        return bool(pass_ok and xg_ok and c.resampler == "soft" and not c.force_resample
                    and c.pass_gate is not False and c.NF_dyn and c.NF_cond
                    and getattr(self, "_gate_resident", False))

    @staticmethod
    def _xg_key(shard):
        return (id(shard.group), shard.world, shard.rank, shard.B_global)

    def _xgate(self, shard, pass_ok, finish, dev):
        """Sharded: set up (once per group and B_global) the cross-rank gate exchange that lets the
        gated pass decide the batch-global gate inside every rank's launch (ops.GateExchange; a
        collective: every rank reaches this call with the same arguments).  Not for a pass captured
        into a graph or left unfinished (its fault and obs reductions are collectives after the
        launch), nor above 512 global rows; NFDPF_XGATE=0 turns it off."""
        c = self.cfg
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if not (shard.world > 1 and pass_ok and finish and not capturing and c.resampler == "soft"
                and not c.force_resample and c.NF_dyn and c.NF_cond and c.pass_gate is not False
                and self._gate_resident and shard.B_global <= 512 and os.environ.get("NFDPF_XGATE", "1") != "0"):
            return None
        key = self._xg_key(shard)
        if self._xg is None or self._xg[0] != key:
            self._xg = (key, ops.GateExchange.create(shard.B_global, shard.rank, shard.world, shard.group, dev))
        return self._xg[1]

    def _plan_capable(self, pass_ok) -> bool:
        """Can the one-launch pass follow a gate plan (the C2 shape's gated kernel with
        d.pass_plan: soft resampler, not forced; any world size, rows in resident chunks)?"""
        c = self.cfg
        return bool(pass_ok and c.resampler == "soft" and not c.force_resample and c.NF_dyn and c.NF_cond
                    and c.pass_gate is not False and c.pass_plan is not False
                    and os.environ.get("NFDPF_PASS_PLAN", "1") != "0")

    def _plan_wanted(self, pass_ok, gate_ok) -> bool:
        """Auto mode: do gate plans replace the other gate strategies for these shapes?  Where the
        gated pass does not apply (a sharded batch: its alternative is one exchange per step; rows
        beyond the resident grid), or everywhere with cfg.pass_plan True (or NFDPF_PASS_PLAN=1)."""
        return self._plan_capable(pass_ok) and (not gate_ok or self.cfg.pass_plan is True
                                                or os.environ.get("NFDPF_PASS_PLAN") == "1")

    def _plan_select(self, pass_ok, gate_ok, T, auto, plan, finish, dev):
        """The next pass's plan (np.int32 [T]) and its device buffer, or (None, None).  Explicit
        ``plan`` (run(plan=...)), else auto: the engine's plan when gate plans are wanted and it
        fires some gate (with none, the speculative pass is the same launch with less to do)."""
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        if plan is not None:
            if not self._plan_capable(pass_ok):
                raise L.NfdpfError("FilterEngine.run: plan= needs the C2-shaped one-launch pass (soft resampler, "
                                   "NF_dyn and NF_cond, not forced; cfg.pass_plan not False)")
            p = np.asarray(plan).astype(np.int32).reshape(-1)
            if p.shape[0] != T:
                raise L.NfdpfError(f"FilterEngine.run: plan= has {p.shape[0]} gates for T={T} steps")
        else:
            p = self._plan
            if not (auto and p is not None and p.shape[0] == T and p.any() and self._plan_wanted(pass_ok, gate_ok)):
                return None, None
            if finish and capturing:  # (nothing could verify it after the replay)
                return None, None
        buf, dev = self._plan_buf, torch.device(dev)
        if buf is None or buf.device != dev or buf.numel() != T:
            if capturing:
                return None, None
            buf = self._plan_buf = torch.empty(T, device=dev, dtype=torch.int32)
            self._plan_buf_val = None
        if self._plan_buf_val is None or not np.array_equal(self._plan_buf_val, p):
            if capturing:  # (a captured pass reads the buffer as it stands)
                return None, None
            buf.copy_(torch.from_numpy(p))  # (stream-ordered: passes already queued read the old plan)
            self._plan_buf_val = p.copy()
        return p, buf

    def plans(self, shard=None) -> bool:
        """Whether run() (auto arguments) will follow a gate plan in its next pass (same shapes as
        the last run): like a speculative pass, its gates are verified after the pass."""
        shard = shard or ShardInfo()
        p = self._plan
        return bool(self.cfg.speculate_gate is None and p is not None and p.any()
                    and self._plan_wanted(self.last_pass_ok, self._gate_ok(shard, self.last_pass_ok)))

    def _pass_supported(self, B, N, T, E, split_nets, shard) -> bool:
        """Can this configuration run its whole pass as one launch (nfdpf_filter_pass_supported:
        the configuration, and the grid resident on the current device)?"""
        c = self.cfg
        # the C2 shape (split RealNVP flows on the particle path) or the C3 shape (none: the
        # bootstrap proposal, tiled_pass_cm_kernel)
        flows_ok = split_nets or (not c.NF_dyn and not c.NF_cond)
        if not (c.kernel == "tiled" and flows_ok and c.rng_mode == "device") or self.pass_disabled:
            return False
        if c.force_resample and c.resampler != "soft":  # a forced pass resamples inside the launch
            return False
        # every workgroup of the grid must be resident at once: never on a device shared with
        # another rank (one-GPU rehearsals of a sharded run, or ranks that all picked device 0),
        # whose kernels can hold CUs.  (Other processes on the device are not detectable here:
        # a pass that times out falls back to the step launches, finish_pending.)
        # (NFDPF_PASS_SHARED_OK=1, tests only: the caller serialises the ranks' passes itself)
        if shard.world > 1 and os.environ.get("NFDPF_PASS_SHARED_OK") != "1" and self._device_shared(shard):
            return False
        d = L.FilterDesc()
        d.B, d.N, d.T, d.E, d.B_global, d.phase = B, N, T, E, shard.B_global, 0
        d.nf_dyn = (L.DYN_MAF if c.dyn_flow == "MAF" else L.DYN_REALNVP) if c.NF_dyn else L.DYN_NONE
        d.nf_cond = int(c.NF_cond)
        d.measurement = L.MEAS.get(c.measurement, L.MEAS_EXTERNAL)
        d.resampler = L.RESAMPLE[c.resampler]
        d.rng_mode, d.force_resample = L.RNG_DEVICE, int(c.force_resample)
        d.n_flows, d.hidden, d.split_nets = c.n_flows, c.hidden, int(split_nets)
        d.meas_mfma = int(self._meas_mfma())
        ok = bool(L.lib().nfdpf_filter_pass_supported(ctypes.byref(d)))
        self._gate_resident = False
        if ok and c.NF_dyn and c.NF_cond and not c.force_resample:
            d.pass_gate, d.B_global = 1, B  # (this rank's rows all resident: sharded, the exchange is per step)
            self._gate_resident = bool(L.lib().nfdpf_filter_pass_supported(ctypes.byref(d)))
        self.pass_fallback_reason = None if ok else self._shape_limit(B, N)
        warn = self.pass_fallback_reason and not getattr(self, "_fallback_warned", False)
        if warn and os.environ.get("NFDPF_PASS") != "0":
            import warnings
            warnings.warn(f"nfdpf: the one-launch pass does not cover this shape ({self.pass_fallback_reason}); "
                          f"running the step launches (about half the speed)", RuntimeWarning, stacklevel=3)
            self._fallback_warned = True
        return ok

    @staticmethod
    def _shape_limit(B, N):
        """The one-launch pass's shape limits (csrc/filter_pass.hpp pass_config_ok,
        filter_pass_cm.hpp pass_cm_config_ok): N <= 1024 (4 tiles of 256 per row), at most 256
        rows per pass (a speculative or forced pass of more rows than the device holds at once
        runs them in resident chunks; the gated pass is then not used)."""
        if not torch.cuda.is_available():
            return None
        tiles = -(-N // 256)
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        if N > 1024:
            return f"N={N} > 1024 particles per row"
        if B > 256:
            return f"B={B} > 256 rows per launch"
        if tiles > cus:
            return f"one row's {tiles} workgroups exceed the {cus} CUs"
        return None

    @staticmethod
    def device_identity(dev=None) -> str:
        """The physical GPU behind ``dev``: its UUID (or PCI location), not the process-local
        index -- two ranks with different visible-device lists can name one GPU differently."""
        idx = torch.cuda.current_device() if dev is None else torch.device(dev).index
        p = torch.cuda.get_device_properties(idx)
        uuid = getattr(p, "uuid", None)
        if uuid is not None and str(uuid).strip("0-"):
            return f"uuid:{uuid}"
        pci = tuple(getattr(p, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if any(v is not None for v in pci):
            return f"pci:{pci}"
        return f"index:{idx}"  # no identity exposed: same index = same device (conservative)

    def _device_shared(self, shard) -> bool:
        """Does another rank of the shard's group run on this rank's GPU?  One all-gather of the
        device identities per engine and process group (cached)."""
        key = id(shard.group)
        if self._shared_device is not None and self._shared_device[0] == key:
            return self._shared_device[1]
        ids = [None] * shard.world
        dist.all_gather_object(ids, self.device_identity(), group=shard.group)
        shared = len(set(ids)) < len(ids)
        self._shared_device = (key, shared)
        return shared

    def _meas_mfma(self) -> bool:
        """Does the no-flow pass (C3 shape) run the CRNVP measurement on f32 MFMA
        (csrc/crnvp_mfma.hpp; NFDPF_CM_MFMA=0 keeps the per-lane VALU measurement)?"""
        c, m = self.cfg, self.m
        if c.measurement != "CRNVP" or c.NF_dyn or c.NF_cond or os.environ.get("NFDPF_CM_MFMA", "1") == "0":
            return False
        from .pack import crnvp_mfma_ok
        return crnvp_mfma_ok(m.particle_encoder, list(m.cnf_measurement.flows))

    def _mfma_blob(self, dev):
        """The CRNVP measurement's MFMA fragment blob (nfdpf.pack.crnvp_mfma_tensors)."""
        from .pack import crnvp_mfma_tensors
        m = self.m
        return blob(m, "meas_mfma", [m.particle_encoder, m.cnf_measurement],
                    lambda: crnvp_mfma_tensors(m.particle_encoder, list(m.cnf_measurement.flows)), dev)

    def _pass_blobs(self, dev):
        """The dynamic / proposal stacks in the one-launch pass's layout (nfdpf.pack.pass_flow_tensors)."""
        m = self.m
        dyn = blob(m, "dyn_pass", m.nf_dyn.flows, lambda: pass_flow_tensors(m.nf_dyn.flows), dev)
        cond = blob(m, "cond_pass", m.cond_model.flows, lambda: pass_flow_tensors(m.cond_model.flows), dev)
        return dyn, cond

    # -- parameters -------------------------------------------------------------------------
    def _blobs(self, dev):
        c, m = self.cfg, self.m
        # the dynamic / proposal stacks carry the split suffix when every flow allows it
        dyn = blob(m, "dyn", m.nf_dyn.flows, lambda: filter_flow_tensors(m.nf_dyn.flows), dev) if c.NF_dyn else None
        cond = (blob(m, "cond", m.cond_model.flows, lambda: filter_flow_tensors(m.cond_model.flows), dev)
                if c.NF_cond else None)
        pe = blob(m, "pe", m.particle_encoder, lambda: encoder_tensors(m.particle_encoder), dev)
        meas = None
        if c.measurement == "CRNVP":
            meas = blob(m, "meas", m.cnf_measurement.flows, lambda: flows_tensors(m.cnf_measurement.flows), dev)
        elif c.measurement == "NN":
            meas = blob(m, "meas", m.likelihood_est, lambda: paired_mlp_tensors(m.likelihood_est), dev)
        elif c.measurement == "CGLOW":
            meas = blob(m, "glow", m.cglow_measurement, lambda: cglow_tensors(m.cglow_measurement), dev)
        return dyn, cond, pe, meas

    # -- main loop --------------------------------------------------------------------------
    @torch.no_grad()
    def run(self, enc: torch.Tensor, start_state: torch.Tensor, vel_input: torch.Tensor,
            shard: Optional[ShardInfo] = None, host: Optional[HostDraws] = None, init=None,
            teacher=None, finish: bool = True, speculate: Optional[bool] = None, plan=None) -> FilterResult:
        """``teacher`` (tests only): dict with the reference's own history ``x`` (B,T,N,2) and
        ``p`` (B,T,N); step t then starts from the reference's step t-1 state and its gate
        is the reference's own torch expression (one-step parity).

        Speculative-gate mode (``cfg.speculate_gate``): the pass runs with every ESS gate
        assumed off and no exchange between the shards; with ``finish`` the gates are then
        verified from all steps' gathered partials (one all-gather) and a fired gate reruns
        the pass with the per-step exchange -- the result is the reference's either way.
        ``finish=False`` leaves the verification to ``finish_pending()`` (the pass itself is
        then free of collectives and host syncs: capturable in a graph).

        Gate plans (cfg.pass_plan; ``plan``: T gates given explicitly): the one-launch pass
        follows the plan's gates, with no batch-wide exchange inside the launch, and its actual
        gates are verified after it like a speculative pass's (one shard: its epilogue; sharded:
        the gathered partials).  A differing gate reruns the pass exactly (one GPU: gated; sharded:
        once more with the corrected plan, then the per-step exchange) and the engine's plan
        becomes the actual gates."""
        c = self.cfg
        dev = enc.device
        L.require_device(enc, "FilterEngine.run")
        if c.measurement not in ("cos", "CRNVP", "NN", "gaussian", "CGLOW"):
            raise L.NfdpfError(f"measurement '{c.measurement}' has no HIP kernel in this build")
        # CGLOW runs as its own kernel between the step's two phases: phase 1 ends with the
        # proposal particles in hist_x slot t, the CGLOW kernel writes their raw likelihood,
        # phase 2 takes it from there (row-max shift, weights, normalisation)
        external = c.measurement == "CGLOW"
        enc = enc.float().contiguous()
        B, T, E = enc.shape
        N = c.N
        shard = shard or ShardInfo(1, 0, B, 0, None)
        if shard.world == 1 and shard.B_global != B:
            # without a process group nothing gathers the other rows' gate partials: the kernels
            # would index a B_global-row table that holds B rows
            raise L.NfdpfError(f"FilterEngine.run: a ShardInfo without a process group needs B_global == B "
                               f"(got B_global={shard.B_global}, B={B})")
        host_mode = c.rng_mode == "host"
        if host_mode and host is None:
            host = HostDraws()
        start_state = start_state.float()
        vel_input = vel_input.float()

        tiled = c.kernel == "tiled"
        auto = speculate is None and c.speculate_gate is None
        ot_auto = auto and tiled and c.resampler == "ot"
        split_nets = bool(tiled and c.split_nets and c.NF_dyn and splittable(self.m.nf_dyn.flows)
                          and (not c.NF_cond or splittable(self.m.cond_model.flows)))
        pass_ok = (not external and teacher is None and not host_mode
                   and self._pass_supported(B, N, T, E, split_nets, shard))
        self.last_pass_ok = pass_ok
        xg = self._xgate(shard, pass_ok, finish, dev) if shard.world > 1 else None
        gate_ok = self._gate_ok(shard, pass_ok) and (shard.world == 1 or xg is not None)
        plan_arr, plan_buf = self._plan_select(pass_ok, gate_ok, T, auto, plan, finish, dev)
        plan_pass = plan_arr is not None
        spec = False if plan_pass else \
            self._decide_spec(shard, speculate, host_mode, teacher is not None, consume=True, finish=finish,
                              pass_ok=pass_ok, gate_ok=gate_ok)
        # the one-launch pass: gates speculated (verified after it), decided inside the launch
        # (one GPU, soft resampler), following a plan (verified after it), or every step
        # resampling (--force-resample: no gate to decide, the row's resampling runs inside the launch)
        gate_pass = (gate_ok and not spec) or plan_pass
        use_pass = pass_ok and (spec or c.force_resample or gate_pass)
        self.last_gate_pass = gate_pass and not plan_pass
        self.last_plan_pass = plan_pass
        checked = spec or plan_pass  # the gates are verified after the pass
        # an exact run by the step launches where gate plans apply (sharded; rows beyond the
        # resident grid): keep every step's (gathered) input partials, so that the run's gates
        # become the engine's plan (the next passes follow it)
        record = (tiled and not checked and not use_pass and not host_mode and teacher is None
                  and self._plan_capable(pass_ok))
        hist1 = record and shard.world == 1  # (one shard: its partials history is the record)
        self.last_gates = None  # (set below by a one-shard one-launch pass; never a previous run's)

        f32 = dict(device=dev, dtype=torch.float32)
        hx = torch.empty((B, T, N, 2), **f32)
        hp = torch.empty((B, T, N), **f32)
        hn = torch.empty((B, T, N, 2), **f32)
        hl = torch.empty((B, T, N), **f32)
        hi = torch.empty((B, T, N), device=dev, dtype=torch.int64)
        hj = torch.empty((B, T, N), **f32) if c.NF_dyn else None
        hr = torch.empty((B, T, N), **f32) if c.NF_dyn else None
        scratch = torch.empty((2, B, N, 4), **f32)  # by step parity (include/nfdpf.h)
        lw_sum = torch.empty((B, T), **f32)
        pred = torch.empty((B, T, 2), **f32)
        if tiled:
            # per-(row, tile) sums of p^2 (double) feed the next step's gate
            tiles = ops.tiled_tiles(N)
            # per-(row, tile) softmax partials {max u, sum e, sum e^2, max lik} of each step:
            # the next step's gate and (deferred) normalisation derive from them
            if spec or use_pass or hist1:  # every step's partials kept for the verification
                ess_hist = torch.empty((T + 1, B, tiles, 4), device=dev, dtype=torch.float64)
                ess_bufs = [ess_hist[t] for t in range(1, T + 1)]
                ess0 = ess_hist[0]
            else:
                ess_bufs = [torch.empty((B, tiles, 4), device=dev, dtype=torch.float64) for _ in range(2)]
                ess0 = torch.empty((B, tiles, 4), device=dev, dtype=torch.float64)
        # initial particles / weights (utils.py:46-62) and p0 = normalize_log_probs (DPFs.py:153)
        # (device RNG, tiled, N <= 1024: the three and the t = 0 gate partials in one launch)
        vel_steps = None
        if init is None and not host_mode and tiled and N <= 1024:
            # (+ every step's velocity in the [T][B][2] layout: no cat / transpose launches)
            x0, logw0, p0, ie0, vel_steps = ops.filter_init(start_state.to(dev), B, N, c.width, c.init_with_true_state,
                                                            c.seed, shard.row_base, dev, ess0,
                                                            vel_input=vel_input.to(dev), T=T)
        else:
            if init is not None:
                x0, logw0 = (t.to(dev).float().contiguous() for t in init)
            elif host_mode:
                xg = host.init(self._global(start_state[:, :2], shard), N, c.width, c.init_with_true_state)
                x0 = xg[shard.row_base:shard.row_base + B].to(dev).contiguous()
                logw0 = torch.log(torch.ones([B, N], device=dev) / N)
            else:
                x0, logw0 = ops.particle_init(start_state[:, :2].to(dev), B, N, c.width, c.init_with_true_state,
                                              c.seed, shard.row_base, dev)
            p0, ie0 = ops.normalize_log_probs(logw0)
            if tiled:
                ops.tiled_init(p0, ess0)
        if tiled:
            ws = ops.tiled_workspace(B, N, T, dev)
            gather_buf = torch.empty((shard.B_global, tiles, 4), device=dev, dtype=torch.float64) \
                if shard.world > 1 and not checked else None
        else:
            ess_bufs = [torch.empty(B, **f32), torch.empty(B, **f32)]
            ess0 = ie0
            gather_buf = torch.empty(shard.B_global, **f32) if shard.world > 1 else None
        # (record: step t's gathered input partials at gather_hist[t]; one shard, its own at ess_hist[t])
        gather_hist = torch.empty((T, shard.B_global, tiles, 4), device=dev, dtype=torch.float64) \
            if record and shard.world > 1 else None
        ess_all = ess0 if checked else self._gather(ess0, shard, gather_hist[0] if gather_hist is not None else gather_buf)
        gate_buf = torch.empty(1, device=dev, dtype=torch.int32)
        # (the step launches' speculative gate word; the one-launch pass reads none)
        spec_gate = torch.zeros(1, device=dev, dtype=torch.int32) if spec and not use_pass else None
        # velocity used by each step's motion: start velocity, then vel_input[:, t-1] (DPFs.py:158,173)
        if vel_steps is None:
            vel_steps = torch.cat([start_state[:, None, 2:4].to(dev), vel_input[:, :T - 1].to(dev)], 1)
            vel_steps = vel_steps.transpose(0, 1).contiguous()  # (T, B, 2)
        dyn, cond, pe, meas = self._blobs(dev)
        lin = ops.linspace_markers(N, dev) if c.resampler == "soft" else None

        d = L.FilterDesc()
        d.B, d.N, d.T, d.E = B, N, T, E
        d.B_global, d.phase, d.row_base = shard.B_global, 0, shard.row_base
        d.nf_dyn = (L.DYN_MAF if c.dyn_flow == "MAF" else L.DYN_REALNVP) if c.NF_dyn else L.DYN_NONE
        d.nf_cond = int(c.NF_cond)
        d.measurement = L.MEAS_EXTERNAL if external else L.MEAS[c.measurement]
        d.resampler = L.RESAMPLE[c.resampler]
        lik_ext = torch.empty((B, N), **f32) if external else None
        d.lik_ext = L.ptr(lik_ext)
        d.rng_mode = L.RNG_HOST if host_mode else L.RNG_DEVICE
        d.force_resample, d.n_flows, d.hidden = int(c.force_resample), c.n_flows, c.hidden
        # tiled + soft: step t's weights are normalised inside step t+1 (one launch fewer per
        # step); not when the caller feeds p_prev itself (teacher forcing) or OT reads it first --
        # except in a speculative pass, whose gates are all taken as off (no Sinkhorn call in it)
        d.defer_norm = int(tiled and teacher is None and (c.resampler == "soft" or (c.resampler == "ot" and spec)))
        d.split_nets = int(split_nets)
        d.alpha, d.pos_noise = c.alpha, c.pos_noise
        d.dens_const, d.meas_prior_std = density_const(c.pos_noise), c.meas_prior_std
        d.seed = int(c.seed) & (2 ** 64 - 1)
        d.dyn_params, d.cond_params = L.ptr(dyn), L.ptr(cond)
        d.pe_params, d.meas_params = L.ptr(pe), L.ptr(meas)
        if tiled and self._meas_mfma():  # the C3 shape's CRNVP measurement on MFMA (pass and step launches)
            mf = self._mfma_blob(dev)
            d.meas_params, d.meas_mfma = mf.data_ptr(), 1  # (caching-allocator blocks: 512-B aligned)
        d.enc, d.lin = enc.data_ptr(), L.ptr(lin)
        d.hist_x, d.hist_p, d.hist_noise, d.hist_lik = hx.data_ptr(), hp.data_ptr(), hn.data_ptr(), hl.data_ptr()
        d.hist_jac, d.hist_prior, d.hist_idx = L.ptr(hj), L.ptr(hr), hi.data_ptr()
        d.lw_sum, d.pred, d.scratch = lw_sum.data_ptr(), pred.data_ptr(), scratch.data_ptr()
        d.ess_local = int(checked)

        fired = [] if host_mode else None
        self.last_ot_calls = 0
        ot_its = []  # the device-gated Sinkhorn calls' iteration counts (0: the gate was off)
        self.last_fused = False  # the step ran as one launch (tiled_step_fused_kernel), set at t = 0
        keep = []  # host uploads must outlive their kernels
        # per-step pointers precomputed as integers: the loop below is the launch path of every
        # time step, so it stays free of tensor slicing and per-call lookups
        hx_p, hp_p, vel_p = hx.data_ptr(), hp.data_ptr(), vel_steps.data_ptr()
        ess_out_p = [b.data_ptr() for b in ess_bufs]
        ess_in_p = [ess0.data_ptr()] + ess_out_p[:-1] if (spec or use_pass) else None
        spec_gate_p = spec_gate.data_ptr() if spec_gate is not None else None
        stream = ops.stream_ptr(dev)
        launch = L.lib().nfdpf_filter_step_tiled if tiled else L.lib().nfdpf_filter_step
        ws_p = ops._aligned_ptr(ws) if tiled else None
        d_ref = ctypes.byref(d)

        def step():
            rc = launch(d_ref, ws_p, stream) if tiled else launch(d_ref, stream)
            if rc != L.NFDPF_OK:
                L.check(rc, "nfdpf_filter_step_tiled" if tiled else "nfdpf_filter_step")

        self.last_pass = use_pass
        pass_out = None  # one shard: the pass epilogue's (gates, flags, obs)
        flags_host = None  # ... the flags mapped from host memory
        flags_lease = None  # ... and the lease of their slot when a captured graph holds it
        if use_pass:
            # the whole T-step pass as ONE persistent launch (nfdpf_filter_pass_tiled): every gate
            # taken as off, step t's softmax partials into ess_hist[t + 1] for the verification
            d.t = 0
            d.x_prev, d.p_prev, d.x_prev_rs, d.p_prev_rs = x0.data_ptr(), p0.data_ptr(), N * 2, N
            d.vel = vel_p
            d.ess_all, d.ess_out, d.gate = ess_in_p[0], ess_out_p[0], spec_gate_p
            if c.NF_dyn:  # the pass layout (tanh algebra in the weights); the C3 shape has no flows here
                pdyn, pcond = self._pass_blobs(dev)
                d.dyn_params, d.cond_params = pdyn.data_ptr(), pcond.data_ptr()
            d.pass_gate = int(gate_pass)
            d.pass_plan = plan_buf.data_ptr() if plan_pass else None
            self.plan_passes += int(plan_pass)
            xg_pass = gate_pass and not plan_pass and shard.world > 1
            if xg_pass:  # the batch-global gate through every rank's exchange buffer, per step
                d.gate_peers, d.gate_world, d.gate_rank = xg.peers.data_ptr(), shard.world, shard.rank
                i32 = dict(device=dev, dtype=torch.int32)
                xg_out = (torch.empty(T, **i32), torch.empty(3, **i32))  # the decisions; {fired, faults, done}
                self.last_gates = xg_out[0]
                d.pass_gates, d.pass_flags = xg_out[0].data_ptr(), xg_out[1].data_ptr()
            if shard.world == 1:  # the epilogue verifies the gates / reads the fault counter on the device
                i32 = dict(device=dev, dtype=torch.int32)
                pass_out = (torch.empty(T, **i32) if (spec or gate_pass) else None, torch.empty(3, **i32),
                            torch.empty((), **f32))
                self.last_gates = pass_out[0]  # the T gates: decided in the launch, or verified
                d.pass_gates, d.pass_flags, d.pass_obs = L.ptr(pass_out[0]), L.ptr(pass_out[1]), L.ptr(pass_out[2])
                capturing = torch.cuda.is_current_stream_capturing()
                if checked or capturing or not finish:
                    # the pass's {fired, faults, done} straight into pinned, device-mapped host memory
                    # (ops.HostMapped): read without a copy launch once the pass is complete -- the
                    # speculative pass's verification, and the fault check of a gated / forced pass
                    # that is captured (checked after each replay: finish_pending) or pipelined
                    if self._hmapped is None and not capturing:
                        self._hmapped = ops.HostMapped()
                    got = self._hmapped.take(reserve=capturing) if self._hmapped is not None else None
                    if got is not None:  # (None: every slot reserved -- the flags stay in device memory)
                        fdev, flags_host, flags_lease = got
                        flags_host[2] = 0  # armed: the epilogue sets it last (arm_flags before a replay)
                        d.pass_flags = fdev
            d.prof_events, d.prof_front = None, 0
            if self.step_events is not None:
                from .prof import EventPair
                ev = EventPair(2)
                self.step_events.append(ev)
                d.prof_events = ev.ptr  # rides in the pass launch's own dispatch
            pws = ops.pass_workspace(B, N, T, dev, owner=self)
            L.check(L.lib().nfdpf_filter_pass_tiled(d_ref, ops._aligned_ptr(pws), stream), "nfdpf_filter_pass_tiled")
            d.dyn_params, d.cond_params = L.ptr(dyn), L.ptr(cond)
            self.pass_launches += 1
        for t in range(0 if use_pass else T):
            if t == 0:
                d.x_prev, d.p_prev, d.x_prev_rs, d.p_prev_rs = x0.data_ptr(), p0.data_ptr(), N * 2, N
            elif teacher is not None:
                xp = teacher["x"][:, t - 1].to(dev).float().contiguous()
                pp = teacher["p"][:, t - 1].to(dev).float().contiguous()
                keep += [xp, pp]
                d.x_prev, d.p_prev, d.x_prev_rs, d.p_prev_rs = xp.data_ptr(), pp.data_ptr(), N * 2, N
            else:  # history slot t-1, rows of T*N
                d.x_prev, d.p_prev = hx_p + (t - 1) * N * 8, hp_p + (t - 1) * N * 4
                d.x_prev_rs, d.p_prev_rs = T * N * 2, T * N
            d.t = t
            d.vel = vel_p + t * B * 8
            if spec:  # this shard's own partials; the gate assumed off (verified after the pass)
                d.ess_all, d.ess_out, d.gate = ess_in_p[t], ess_out_p[t], spec_gate_p
            else:
                d.ess_all = ess_all.data_ptr()
                d.ess_out = ess_out_p[t if hist1 else t & 1]
                d.gate = None
            d.host_noise = d.host_offsets = None
            if host_mode:
                if teacher is not None and t > 0:
                    pc = teacher["p"][:, t - 1].cpu().float()
                    fire = bool(c.force_resample or torch.mean(1 / torch.sum(pc ** 2, dim=-1)) < 0.5 * N)
                elif tiled:
                    fire = self._host_gate_parts(ess_all, N, c.force_resample, t)
                else:
                    fire = self._host_gate(ess_all, N, c.force_resample)
                fired.append(fire)
                gate_buf.fill_(int(fire))
                d.gate = gate_buf.data_ptr()
                if fire and c.resampler == "soft":
                    off = host.offsets(shard.B_global, N)[shard.row_base:shard.row_base + B].to(dev)
                    keep.append(off)
                    d.host_offsets = off.data_ptr()
                nz = host.noise(shard.B_global, N, c.pos_noise)[shard.row_base:shard.row_base + B]
                nz = nz.to(dev).contiguous()
                keep.append(nz)
                d.host_noise = nz.data_ptr()
            elif c.resampler == "ot" and not spec:
                if c.force_resample:  # the gate word is constant: set once, no gate launch per step
                    if t == 0:
                        gate_buf.fill_(1)
                elif tiled:
                    ops.ess_gate_tiled(ess_all, N, t, c.force_resample, out=gate_buf)
                else:
                    ops.ess_gate(ess_all, N, c.force_resample, out=gate_buf)
                d.gate = gate_buf.data_ptr()
            if c.resampler == "ot" and spec:
                d.ot_x = x0.data_ptr()  # not read: every gate is taken as off (verified after the pass)
            elif c.resampler == "ot":
                if t == 0:
                    xin, pin = x0, p0
                elif teacher is not None:
                    xin, pin = xp, pp
                elif shard.world > 1:
                    xin, pin = hx[:, t - 1].contiguous(), hp[:, t - 1].contiguous()
                else:  # (read in place: nfdpf_ot_resample_rs)
                    xin, pin = hx[:, t - 1], hp[:, t - 1]
                # The Sinkhorn call reads the device gate itself (every launch of a call whose gate
                # is off returns at once, and the host's poll stops enqueueing iterations after the
                # first), so the host does not wait for the gate before enqueueing the call: the
                # reference's `if ESS < ...` (DPFs.py:165) is a host sync per step, which left the
                # device idle while the call's launches went out.  The steps that resampled are
                # counted from the calls' iteration counts after the pass (0: the gate was off).
                # The gate is batch-global: same on every rank.  (--force-resample: on by
                # construction; host draws / teacher forcing: the host's own decision.)
                device_gate = not host_mode and teacher is None and not c.force_resample
                fire = fired[-1] if host_mode else (True if c.force_resample else
                                                    (None if device_gate else bool(gate_buf.item())))
                if fire is None or fire:
                    if fire:
                        self.last_ot_calls += 1
                    if shard.world > 1:
                        # batch-coupled stop over every rank's rows (resamplers.py:126-129): the
                        # local loop, the MIN of the stop count, the tail at that state
                        xo, _, _, it = ops.ot_resample_sharded(xin, pin, c.eps, c.scaling, c.threshold, c.max_iter,
                                                               shard.row_base, group=shard.group, gate=gate_buf)
                    else:
                        xo, _, _, it = ops.ot_resample(xin, pin, c.eps, c.scaling, c.threshold, c.max_iter,
                                                       shard.row_base, gate=gate_buf)
                    keep.append(xo)
                    if fire is None:
                        ot_its.append(it)
                    d.ot_x = xo.data_ptr()  # (read by the step only where the gate fired)
                else:
                    d.ot_x = xin.data_ptr()  # not read: the motion stage keeps the previous particles
            if t == 0 and tiled and not external:
                self.last_fused = bool(L.lib().nfdpf_filter_tiled_fused(d_ref))
            d.prof_events = None
            d.prof_front = 0
            ev = None
            # the tiled step carries the events in the timed launch's own dispatch (no stream
            # cost): every step; elsewhere an event pair costs ~6 us of stream time: one sampled
            # step per pass
            every = c.kernel == "tiled" and not external
            if self.step_events is not None and (every or t == T // 2):
                from .prof import EventPair
                ev = EventPair(4 if every and not self.last_fused else 2)
                self.step_events.append(ev)
                if not external:
                    d.prof_events = ev.ptr  # around the step's dominant launch, inside the library
                    # and, tiled, around its front (resampling) launch -- none in the fused step
                    d.prof_front = int(every and not self.last_fused)
            if external:
                d.phase = 1
                step()
                if ev is not None:
                    ev.record_start(dev)  # the CGLOW kernel is the step's dominant launch
                ops.cglow_measurement(pe, meas, enc[:, t], hx[:, t], out=lik_ext)
                if ev is not None:
                    ev.record_end(dev)
                d.phase = 2
                step()
            else:
                step()
            if spec:
                pass
            elif shard.world > 1:
                ess_all = self._gather(ess_bufs[t & 1], shard,
                                       gather_hist[t + 1] if gather_hist is not None and t + 1 < T else gather_buf)
            else:
                ess_all = ess_bufs[t if hist1 else t & 1]
        # a wave-pair hand-off that timed out leaves stale data (csrc/split.hpp): fail loudly
        # (a stream-ordered read and a sync: deferred to finish_pending when the caller asked
        # for a pass free of host syncs)
        # (the split nets, and the CRNVP launch's cond -> flow hand-off without --NF-cond)
        # (the opt-in two-chain CRNVP launch hands off between its waves too; the default
        # one-chain launch does not, and then no check -- a host sync -- is paid)
        handoffs = d.split_nets or (d.measurement == L.MEAS["CRNVP"] and not d.nf_cond
                                    and os.environ.get("NFDPF_CM_TWO_CHAIN", "0") == "1")
        capturing = torch.cuda.is_current_stream_capturing()
        check_split = tiled and handoffs and not capturing
        if record:  # the exact run's gates: the plan of the next passes
            self._plan = ops.ess_gate_tiled_batch(gather_hist if gather_hist is not None else ess_hist[:T], N, 0,
                                                  False).cpu().numpy()
        if use_pass and not checked:
            # a forced or gated pass: one shard's epilogue read the fault counter and reduced the
            # obs-likelihood (one host read here); sharded, every rank's count is summed so that all
            # ranks fall back together.  Captured in a graph, or run(finish=False): the flags are
            # left in the pending state (take_pending / finish_pending after each replay: a replay
            # whose hand-offs timed out must not pass for a result), nothing is read here.
            check_split = False
            if pass_out is not None and (capturing or not finish):
                res = FilterResult(hx, hp, hn, hl, logw0, hi, hj, hr, pass_out[2], pred, fired)
                verify = [pass_out[1] if flags_host is None else None, pass_out[2], flags_host, flags_lease]
                self._pending = (None, None, shard, N, res, None, verify, True, True)
                return res
            if not capturing:
                if xg_pass:  # (the epilogue read and cleared this rank's fault counter)
                    n_fired, faults = xg_out[1].tolist()[:2]
                    ft = torch.tensor([faults], device=dev, dtype=torch.int64)
                    dist.all_reduce(ft, group=shard.group)  # every rank falls back together
                    faults = int(ft.item())
                    if not faults and self._plan_wanted(pass_ok, gate_ok):
                        self._plan = xg_out[0].cpu().numpy()  # the decisions: the next passes' plan
                elif pass_out is not None:
                    n_fired, faults = pass_out[1].tolist()[:2]
                    if gate_pass and not faults and self._plan_wanted(pass_ok, gate_ok):
                        self._plan = pass_out[0].cpu().numpy()  # the gates it decided: the next passes' plan
                else:
                    n_fired, faults = 0, self._faults_all(shard, dev)
                if faults:  # the grid was not all resident: the step launches instead
                    self._pass_fault(faults)
                    return self.run(enc, start_state, vel_input, shard=shard, host=host, init=init, finish=finish,
                                    speculate=speculate)
                if gate_pass and auto:  # back to speculation after two gated passes without a fired gate
                    self._gate_quiet = 0 if n_fired else self._gate_quiet + 1
                    if self._gate_quiet >= 2:
                        self._gate_mode, self._gate_quiet = False, 0
            if pass_out is not None:
                return FilterResult(hx, hp, hn, hl, logw0, hi, hj, hr, pass_out[2], pred, fired)
        # one-shard speculative pass: the gates and the fault counter are verified on the device
        # (the one-launch pass's epilogue, or ops.pass_verify after the step launches -- both
        # capturable) and read once in finish_pending
        verify_dev = checked and tiled and shard.world == 1
        if check_split and (finish or not spec) and not verify_dev and not use_pass:
            L.check_split_fault("nfdpf_filter_step_tiled", dev)
            check_split = False
        if ot_its:  # (one read for the pass: the device-gated calls that ran)
            self.last_ot_calls += int(torch.cat(ot_its).gt(0).sum())
        if c.resampler == "ot" and not spec:
            self._ot_fired = self.last_ot_calls > 0
        # obs_likelihood = sum_t mean_{b,n} logw_t (DPFs.py:191)
        tot = None if verify_dev else lw_sum.double().sum(0)  # (verified on the device: reduced there)
        if checked:
            res = FilterResult(hx, hp, hn, hl, logw0, hi, hj, hr, None, pred, fired)
            verify = None
            if verify_dev:
                verify = [pass_out[1] if flags_host is None else None, pass_out[2], flags_host, flags_lease] \
                    if pass_out is not None else list(ops.pass_verify(ess_hist[:T], lw_sum, N)[1:]) + [None, None]
                check_split = False
            # (+ the plan followed, and one shard's actual gates: a miss's new plan)
            # (+ the plan followed, one shard's actual gates, and -- sharded -- the staged verification,
            # stage_flags)
            self._pending = (ess_hist[:T], tot, shard, N, res, dev if check_split else None, verify, use_pass, False,
                             plan_arr, pass_out[0] if pass_out is not None else None, [])
            if not finish:
                return res  # the caller verifies (finish_pending, e.g. after each graph replay)
            ok = self.finish_pending()
            # verified here: a kept engine (DPF keeps one) must not pin the pass's buffers
            self._pending = None
            if ok:
                self._spec_backoff = 0
                return res
            if self.last_verify == "fault":
                # the pass's grid was not resident (not a gate miss): the one-launch pass is now off
                # for this engine and the step launches rerun it; the speculation state is left alone
                return self.run(enc, start_state, vel_input, shard=shard, host=host, init=init, speculate=speculate)
            if plan_pass:
                # a gate differed from the plan: the pass again, exactly -- one GPU with every row
                # resident, gated; else the step launches with the batch gate per step -- and the
                # gates it takes become the plan (a plan of a pass that missed is exact only up to
                # its first differing gate: following it again would fix one more gate per pass)
                self.plan_misses += 1
                return self.run(enc, start_state, vel_input, shard=shard, host=host, init=init, speculate=False)
            # a gate fired: the pass again, gated (one GPU, the one-launch pass: the gates decided in
            # the launch; the next passes stay gated while gates keep firing) or with the per-step
            # exchange
            if ot_auto:
                self._ot_fired = True  # the rerun below sets it from its own OT calls
            elif auto and gate_ok and not self.pass_disabled:
                self._gate_mode, self._gate_quiet = True, 0
            elif auto:
                self._spec_backoff = min(2 * self._spec_backoff or 1, 64)
                self._spec_skip = self._spec_backoff
            return self.run(enc, start_state, vel_input, shard=shard, host=host, init=init, speculate=False)
        if shard.world > 1:
            dist.all_reduce(tot, group=shard.group)
        obs = (tot / (shard.B_global * N)).sum().float()
        return FilterResult(hx, hp, hn, hl, logw0, hi, hj, hr, obs, pred, fired)

    @staticmethod
    def _sharded_verify(parts, tot, shard, N):
        """The verification of a sharded speculative / plan pass, enqueued on the current stream:
        ONE all-gather of each rank's summary -- its per-step log-weight sums (fp64), its rows' gate
        terms of every step (nfdpf_ess_row_terms: the per-row half of the batch gate's arithmetic,
        T x B floats instead of the T x B x tiles x 4 doubles of partials) and its hand-off fault
        counter -- then the T gates over the gathered rows (nfdpf_ess_gate_terms).  -> (int64
        [T + 1] on the device: the gates, then the faults summed over the ranks; fp64 [T]: the
        step sums summed over the ranks, in rank order)."""
        T, B = parts.shape[0], parts.shape[1]
        summ = torch.cat([tot.view(torch.float32), ops.ess_row_terms(parts, N)])  # (the fp64 words first)
        S = summ.numel()
        g = torch.empty(shard.world * S, device=summ.device, dtype=torch.float32)
        dist.all_gather_into_tensor(g, summ, group=shard.group)
        g = g.view(shard.world, S)
        terms = g[:, 2 * T:2 * T + T * B].reshape(shard.world, T, B).permute(1, 0, 2).reshape(T, shard.world * B)
        gates = ops.ess_gate_terms(terms, N)
        faults = g[:, 2 * T + T * B].view(torch.int32).to(torch.int64).sum()
        return torch.cat([gates.to(torch.int64), faults.view(1)]), g[:, :2 * T].contiguous().view(torch.float64).sum(0)

    @staticmethod
    def stage_flags(pending):
        """Enqueue (current stream) the copy of a one-shard speculative pass's device flags
        {fired, faults} into pinned host memory; after an event recorded behind it has completed,
        ``finish_pending(pending, synced=True)`` reads them with no stream operation -- so a
        later pass already queued keeps running (pipelined passes, bench.py).  Not while
        capturing a graph (the pinned allocation is not capturable): after the replay."""
        verify = pending[6]
        parts, tot, shard, N = pending[:4]
        if verify is None and shard is not None and shard.world > 1 and len(pending) > 11:
            # sharded: the all-gather and the gates enqueued now, their small result copied to
            # pinned host memory behind them (every rank stages the same sequence of collectives)
            dev_small, tot_all = FilterEngine._sharded_verify(parts, tot, shard, N)
            host = torch.empty(dev_small.shape, dtype=dev_small.dtype, pin_memory=True)
            host.copy_(dev_small, non_blocking=True)
            pending[11][:] = [host, tot_all]
            return
        if verify is None or verify[0] is None:  # (flags already mapped from host memory)
            return
        if verify[2] is None:
            verify[2] = torch.empty(verify[0].shape, dtype=verify[0].dtype, pin_memory=True)
        verify[2].copy_(verify[0], non_blocking=True)

    @staticmethod
    def arm_flags(pending):
        """Before replaying a captured speculative pass whose flags are mapped from host memory:
        clear its completion word (the epilogue sets it, last, with a system-scope release)."""
        verify = pending[6]
        if verify is not None and verify[0] is None:
            verify[2][2] = 0

    @staticmethod
    def wait_flags(pending, timeout_s: float = 60.0) -> bool:
        """Wait on the host, with no stream operation, until the pass's epilogue has written its
        flags into host memory (their completion word); False where the flags are not mapped.
        Spins with a yield for the first millisecond, then sleeps 50 us between reads; every 10 ms
        it asks whether the current stream is idle -- an idle stream with the word still unset
        means the pass never ran (a launch or stream error): raised at once, not after the bound."""
        verify = pending[6]
        if verify is None or verify[0] is not None:
            return False
        view = verify[2]
        t0 = time.perf_counter()
        last_q = t0
        while int(view[2]) == 0:
            now = time.perf_counter()
            if now - t0 > timeout_s:
                raise L.NfdpfError(f"the one-launch pass's flags did not arrive within {timeout_s} s")
            if now - t0 < 1e-3:
                os.sched_yield()
                continue
            time.sleep(50e-6)
            if now - last_q > 10e-3:
                last_q = now
                if torch.cuda.current_stream().query() and int(view[2]) == 0:
                    raise L.NfdpfError("the one-launch pass's stream is idle but its flags were never written "
                                       "(the pass or its epilogue did not run)")
        return True

    def take_pending(self):
        """The verification state of the last ``run(finish=False)``, handed to the caller (e.g.
        one per captured graph when passes are pipelined): ``finish_pending(pending)`` later."""
        p, self._pending = self._pending, None
        return p

    def finish_pending(self, pending=None, synced: bool = False) -> bool:
        """Verify the speculative pass of the last ``run`` (or the given ``take_pending()``
        state; its buffers, so also after a graph replay of it): gather every step's softmax
        partials over the shards (one all-gather), evaluate all T gates
        (nfdpf_ess_gate_tiled_batch) and, if none fired, reduce the obs-likelihood into the
        result.  False: some gate fired -- the pass is not the reference's and must be rerun
        without speculation (run(..., speculate=False)) -- or the pass's row hand-offs timed out
        (its grid was not resident; the one-launch pass is then off for this engine and a rerun
        takes the step launches).  ``self.last_verify`` tells the two apart: "ok", "fired" or
        "fault".  A gated or forced one-launch pass (its gates decided inside the launch) that was
        captured or run with finish=False only has its fault flags checked here: "ok" or "fault".
        ``synced``: the pass's flags were staged (stage_flags) and an event recorded after that
        copy has completed: they are read from pinned host memory with no stream operation, so a
        later pass already queued behind it keeps running (pipelined passes, bench.py)."""
        pend = pending if pending is not None else self._pending
        parts, tot, shard, N, res, split_dev, verify, was_pass = pend[:8]
        decided = len(pend) > 8 and pend[8]  # the gates were decided inside the launch
        # a plan pass: the plan it followed, and one shard's actual gates (its epilogue's)
        plan, gates_dev = (pend[9], pend[10]) if len(pend) > 10 else (None, None)
        self.last_verify = "ok"
        if verify is not None:  # the device verification's flags: the one host synchronisation
            if verify[0] is None:  # mapped from host memory: complete once the stream is
                if not synced:
                    torch.cuda.current_stream().synchronize()
                fired, faults = (int(v) for v in verify[2][:2])
            elif synced and verify[2] is not None:  # staged (stage_flags) and known complete
                fired, faults = verify[2].tolist()[:2]
            else:
                fired, faults = verify[0].tolist()[:2]
            if faults:
                if not was_pass:
                    raise L.NfdpfError(f"nfdpf_filter_step_tiled: {faults} wave hand-off(s) timed out on the device "
                                       f"(outputs invalid)")
                self._pass_fault(faults)  # the one-launch pass's grid was not resident: rerun step by step
                self.last_verify = "fault"
                return False
            if fired and not decided:  # (a plan pass: `fired` counts the gates that differ from the plan)
                self.last_verify = "fired"
                if plan is not None:
                    self._plan = gates_dev.cpu().numpy()  # exact up to its first differing gate
                return False
            res.obs_likelihood = verify[1]
            return True
        if shard.world > 1:
            # ONE all-gather of each rank's summary: its rows' gate terms of every step (the per-row
            # half of the batch gate's arithmetic, nfdpf_ess_row_terms: T x B floats instead of the
            # T x B x tiles x 4 doubles of partials), its hand-off fault counter and its per-step
            # log-weight sums; then the gates over the gathered rows (nfdpf_ess_gate_terms), and
            # ONE host read of {gates, faults}
            T = parts.shape[0]
            stage = pend[11] if len(pend) > 11 else []
            if stage:  # staged (stage_flags): read with no stream operation once known complete
                if not synced:
                    torch.cuda.current_stream().synchronize()
                host, tot = stage[0], stage[1]
            else:
                dev_small, tot = self._sharded_verify(parts, tot, shard, N)
                host = dev_small.cpu()
            faults = int(host[T])
            if faults:
                if not was_pass:
                    raise L.NfdpfError(f"nfdpf_filter_step_tiled: {faults} wave hand-off(s) timed out on the device "
                                       f"(outputs invalid)")
                self._pass_fault(faults)
                self.last_verify = "fault"
                return False
            gates = host[:T].to(torch.int32)
        else:
            if split_dev is not None:
                if was_pass:
                    faults = self._faults_all(shard, split_dev)
                    if faults:
                        self._pass_fault(faults)
                        self.last_verify = "fault"
                        return False
                else:
                    L.check_split_fault("nfdpf_filter_step_tiled", split_dev)
            gates = ops.ess_gate_tiled_batch(parts, N, 0, False)
        if plan is not None:  # the pass followed a plan: its actual gates must be the plan's
            g = gates.cpu().numpy()
            if not np.array_equal(g, plan):
                self.last_verify = "fired"
                self._plan = g
                return False
        elif bool(gates.any()):
            self.last_verify = "fired"
            return False
        res.obs_likelihood = (tot / (shard.B_global * N)).sum().float()
        return True

    # -- helpers ----------------------------------------------------------------------------
    def _pass_fault(self, faults: int):
        """A one-launch pass timed out waiting for its own workgroups (its grid was not all
        resident: another process or stream held CUs, or a CU mask): warn, turn the pass off
        for this engine; the caller reruns the pass with the step launches."""
        import warnings
        warnings.warn(f"nfdpf_filter_pass_tiled: {faults} row hand-off wait(s) timed out (the pass's grid was not "
                      f"resident); rerunning with the step launches, the one-launch pass is off for this engine",
                      RuntimeWarning, stacklevel=3)
        self.pass_disabled = True

    @staticmethod
    def _faults_all(shard: ShardInfo, dev) -> int:
        """The hand-off fault counter (read and cleared), summed over the shard's ranks."""
        n = int(L.lib().nfdpf_split_fault(1, L.stream_ptr(dev)))
        if n < 0:
            raise L.NfdpfError("could not read the device fault counter")
        if shard.world > 1:
            t = torch.tensor([n], device=dev, dtype=torch.int64)
            dist.all_reduce(t, group=shard.group)
            n = int(t.item())
        return n

    @staticmethod
    def _global(t: torch.Tensor, shard: ShardInfo) -> torch.Tensor:
        """Host copy of a per-row tensor over the whole (sharded) batch."""
        t = t.detach()
        if shard.world == 1:
            return t.cpu()
        out = torch.empty((shard.B_global,) + tuple(t.shape[1:]), device=t.device, dtype=t.dtype)
        dist.all_gather_into_tensor(out, t.contiguous(), group=shard.group)
        return out.cpu()

    @staticmethod
    def _gather_steps(parts: torch.Tensor, shard: ShardInfo) -> torch.Tensor:
        """[T, B, tiles, 4] per-shard step partials -> [T, B_global, tiles, 4] (rows in rank
        order = global row order), one all-gather."""
        if shard.world == 1:
            return parts
        T, B = parts.shape[0], parts.shape[1]
        # concatenated along dim 0 (the layout every backend accepts), then rank-major -> row order
        g = torch.empty((shard.world * T,) + tuple(parts.shape[1:]), device=parts.device, dtype=parts.dtype)
        dist.all_gather_into_tensor(g, parts.contiguous(), group=shard.group)
        g = g.view((shard.world, T) + tuple(parts.shape[1:]))
        return g.transpose(0, 1).reshape((T, shard.world * B) + tuple(parts.shape[2:]))

    @staticmethod
    def _gather(ie: torch.Tensor, shard: ShardInfo, buf=None) -> torch.Tensor:
        if shard.world == 1:
            return ie
        out = buf if buf is not None else torch.empty(shard.B_global, device=ie.device, dtype=ie.dtype)
        dist.all_gather_into_tensor(out, ie, group=shard.group)
        return out

    @staticmethod
    def _host_gate_parts(parts: torch.Tensor, N: int, force: bool, t: int) -> bool:
        """Tiled-mode gate of step t on the host, from the [B, tiles, 4] softmax partials of
        step t-1 (csrc/filter_tiled.hip row_inv_ess): sum p^2 = sum e^2 / S^2 (+ the +1e-12
        terms after a filter step), 1/sum in float32, then torch.mean over rows."""
        if force:
            return True
        inv = []
        for row in parts.double().cpu().numpy():
            M = row[:, 0].max()
            f = np.exp((row[:, 0] - M).astype(np.float32)).astype(np.float64)  # f32 factors, as the kernel
            S = float(np.sum(row[:, 1] * f))
            Q = float(np.sum(row[:, 2] * f * f))
            sp2 = Q / (S * S) + ((2e-12 + N * 1e-24) if t > 0 else 0.0)
            inv.append(np.float32(1.0) / np.float32(sp2))
        return bool(torch.from_numpy(np.array(inv, dtype=np.float32)).mean() < np.float32(0.5 * N))

    @staticmethod
    def _host_gate(ess_all: torch.Tensor, N: int, force: bool) -> bool:
        """The kernel's gate rule evaluated on the host (parity mode syncs here, as the
        reference does at DPFs.py:165): torch.mean of 1/sum(p^2) < 0.5 N."""
        if force:
            return True
        return bool(ess_all.float().cpu().mean() < np.float32(0.5 * N))
