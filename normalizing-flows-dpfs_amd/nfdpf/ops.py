"""torch-facing wrappers of the C ABI (one function per nfdpf_* entry point).

Every wrapper takes device tensors, allocates its outputs with torch (the library never
allocates), launches on torch's current HIP stream and raises on error.  No host copies,
no synchronisation.
"""
from __future__ import annotations

import functools
from typing import Optional

import torch

from . import _lib as L
from ._lib import check, lib, ptr, require_device, stream_ptr

f32 = torch.float32


def _c(t: torch.Tensor, dtype=f32) -> torch.Tensor:
    return t.to(dtype=dtype).contiguous()


def cond_stack(blob, n_flows, dim, obser_dim, hidden, x, cond, cond_group=1, inverse=False,
               prior_mean=0.0, prior_std=1.0, want_prior=False):
    """NormalizingFlowModel_cond.forward/.inverse (nf/models.py:45-61) -> (out, logdet, prior_lp)."""
    require_device(x, "cond_stack")
    x = _c(x)
    rows = x.shape[0]
    cond = _c(cond) if cond is not None and obser_dim > 0 else None
    out = torch.empty_like(x)
    ld = torch.empty(rows, device=x.device, dtype=f32)
    lp = torch.empty(rows, device=x.device, dtype=f32) if (want_prior and not inverse) else None
    check(lib().nfdpf_cond_stack(ptr(blob), n_flows, dim, obser_dim, hidden, ptr(x), ptr(cond), rows,
                                 max(1, int(cond_group)), int(bool(inverse)), float(prior_mean), float(prior_std),
                                 ptr(out), ptr(ld), ptr(lp), stream_ptr(x.device)), "nfdpf_cond_stack")
    return out, ld, lp


def cond_stack_backward(blob, n_flows, dim, obser_dim, hidden, x, cond, inverse, g_out, g_logdet,
                        g_prior=None, prior_mean=0.0, prior_std=1.0):
    """Backward of cond_stack with a per-row condition -> (g_x, g_cond or None, g_blob)
    (include/nfdpf.h nfdpf_cond_stack_backward)."""
    require_device(x, "cond_stack_backward")
    x, g_out, g_logdet = _c(x), _c(g_out), _c(g_logdet)
    rows = x.shape[0]
    cond = _c(cond) if cond is not None and obser_dim > 0 else None
    if cond is not None and cond.shape[0] != rows:
        raise ValueError(f"cond_stack_backward: cond has {cond.shape[0]} rows, x has {rows} (per-row condition only)")
    g_prior = _c(g_prior) if g_prior is not None and not inverse else None
    gx = torch.empty_like(x)
    gc = torch.empty_like(cond) if cond is not None else None
    gb = torch.empty_like(blob)
    nbytes = lib().nfdpf_cond_stack_backward_workspace(n_flows, dim, obser_dim, hidden, rows)
    if nbytes < 0:
        raise L.NfdpfError(f"cond_stack_backward: bad sizes (n_flows={n_flows}, dim={dim}, hidden={hidden})")
    ws = torch.empty(max(1, nbytes // 4), device=x.device, dtype=f32)
    check(lib().nfdpf_cond_stack_backward(ptr(blob), n_flows, dim, obser_dim, hidden, ptr(x), ptr(cond), rows,
                                          int(bool(inverse)), float(prior_mean), float(prior_std), ptr(g_out),
                                          ptr(g_logdet), ptr(g_prior), ptr(gx), ptr(gc), ptr(gb), ptr(ws),
                                          stream_ptr(x.device)), "nfdpf_cond_stack_backward")
    return gx, gc, gb


def maf_stack(blob, n_flows, dim, hidden, x, inverse=False):
    """NormalizingFlowModel over MAF flows (nf/models.py:13-30, nf/flows.py:259-284)."""
    require_device(x, "maf_stack")
    x = _c(x)
    out = torch.empty_like(x)
    ld = torch.empty(x.shape[0], device=x.device, dtype=f32)
    check(lib().nfdpf_maf_stack(ptr(blob), n_flows, dim, hidden, ptr(x), x.shape[0], int(bool(inverse)),
                                ptr(out), ptr(ld), stream_ptr(x.device)), "nfdpf_maf_stack")
    return out, ld


def maf_stack_backward(blob, n_flows, dim, hidden, x, inverse, g_out, g_logdet):
    """Backward of maf_stack -> (g_x, g_blob), or None when the kernel does not cover the sizes
    (include/nfdpf.h nfdpf_maf_stack_backward)."""
    require_device(x, "maf_stack_backward")
    x = _c(x)
    rows = x.shape[0]
    nbytes = int(lib().nfdpf_maf_stack_backward_workspace(n_flows, dim, hidden, rows))
    if nbytes < 0 or (dim == 4 and n_flows > 2):
        return None
    gx = torch.empty_like(x)
    gb = torch.empty_like(blob)
    ws = torch.empty(max(1, nbytes // 4), device=x.device, dtype=f32)
    go = _c(g_out) if g_out is not None else None
    gl = _c(g_logdet) if g_logdet is not None else None
    check(lib().nfdpf_maf_stack_backward(ptr(blob), n_flows, dim, hidden, ptr(x), rows, int(bool(inverse)), ptr(go),
                                         ptr(gl), ptr(gx), ptr(gb), ptr(ws), stream_ptr(x.device)),
          "nfdpf_maf_stack_backward")
    return gx, gb


def pseudo_lik_forward(w, lik, prior, index, block_len):
    """compute_block_density_nf (losses.py:37-68) -> Q [B] fp64 (nfdpf_pseudo_lik_forward)."""
    require_device(w, "pseudo_lik_forward")
    B, T, N = w.shape
    w, lik, prior = _c(w), _c(lik), _c(prior)
    index = index.to(torch.int64).contiguous()
    Q = torch.empty(B, device=w.device, dtype=torch.float64)
    check(lib().nfdpf_pseudo_lik_forward(ptr(w), ptr(lik), ptr(prior), ptr(index), B, T, N, int(block_len), ptr(Q),
                                         stream_ptr(w.device)), "nfdpf_pseudo_lik_forward")
    return Q


def pseudo_lik_monotone(index) -> bool:
    """True when every step's ancestor map is non-decreasing over the flattened batch (one
    device flag read: a host sync)."""
    B, T, N = index.shape
    ok = torch.ones(1, device=index.device, dtype=torch.int32)
    check(lib().nfdpf_pseudo_lik_check(ptr(index), B, T, N, ptr(ok), stream_ptr(index.device)),
          "nfdpf_pseudo_lik_check")
    return bool(ok.item())


def pseudo_lik_backward(w, lik, prior, index, block_len, g_Q):
    """-> (g_w, g_lik, g_prior) [B, T, N] (nfdpf_pseudo_lik_backward)."""
    require_device(w, "pseudo_lik_backward")
    B, T, N = w.shape
    w, lik, prior, g_Q = _c(w), _c(lik), _c(prior), _c(g_Q)
    index = index.to(torch.int64).contiguous()
    gw, gl, gp = torch.empty_like(w), torch.empty_like(lik), torch.empty_like(prior)
    nbytes = int(lib().nfdpf_pseudo_lik_workspace(B, T, N, int(block_len)))
    ws = torch.empty(max(1, nbytes // 4), device=w.device, dtype=f32)
    check(lib().nfdpf_pseudo_lik_backward(ptr(w), ptr(lik), ptr(prior), ptr(index), B, T, N, int(block_len),
                                          ptr(g_Q), ptr(gw), ptr(gl), ptr(gp), ptr(ws), stream_ptr(w.device)),
          "nfdpf_pseudo_lik_backward")
    return gw, gl, gp


@functools.lru_cache(maxsize=64)
def _lin_cpu(N: int) -> torch.Tensor:
    # the reference's marker base, torch.linspace on CPU (resamplers.py:42); a per-N constant
    return torch.linspace(0.0, (N - 1.0) / N, N)


_lin_dev = {}


def linspace_markers(N: int, device) -> torch.Tensor:
    key = (N, str(device))
    t = _lin_dev.get(key)
    if t is None:
        t = _lin_dev[key] = _lin_cpu(N).to(device)
    return t


def soft_resample(x, p, alpha, offsets, row_base=0):
    """soft_resampler (resamplers.py:20-60) -> (x', w', flat idx int64)."""
    require_device(x, "soft_resample")
    B, N = p.shape
    x, p = _c(x), _c(p)
    D = x.shape[-1]
    xo = torch.empty_like(x)
    wo = torch.empty_like(p)
    idx = torch.empty((B, N), device=x.device, dtype=torch.int64)
    off = _c(offsets.to(x.device))
    check(lib().nfdpf_soft_resample(ptr(x), ptr(p), ptr(linspace_markers(N, x.device)), ptr(off), B, N, D,
                                    float(alpha), int(row_base), ptr(xo), ptr(wo), ptr(idx),
                                    stream_ptr(x.device)), "nfdpf_soft_resample")
    return xo, wo, idx


def soft_resample_backward(p, idx, w_out, g_x_out, g_w_out, alpha, D, row_base=0):
    """Backward of soft_resample -> (g_x [B, N, D], g_p [B, N]) (include/nfdpf.h)."""
    require_device(p, "soft_resample_backward")
    B, N = p.shape
    p, w_out = _c(p), _c(w_out)
    idx = idx.to(torch.int64).contiguous()
    gxo = _c(g_x_out) if g_x_out is not None else None
    gwo = _c(g_w_out) if g_w_out is not None else None
    gx = torch.empty((B, N, D), device=p.device, dtype=f32)
    gp = torch.empty((B, N), device=p.device, dtype=f32)
    ws = torch.empty(max(1, int(lib().nfdpf_soft_resample_backward_workspace(B, N))), device=p.device,
                     dtype=torch.uint8)
    check(lib().nfdpf_soft_resample_backward(ptr(p), ptr(idx), ptr(w_out), ptr(gxo), ptr(gwo), B, N, D,
                                             float(alpha), int(row_base), ptr(gx), ptr(gp), ptr(ws),
                                             stream_ptr(p.device)), "nfdpf_soft_resample_backward")
    return gx, gp


def cos_measurement_backward(pe_blob, enc, x, g_lik):
    """Backward of the cosine measurement -> (g_enc [B, E], g_x [B, N, 2], g_params [1648] in
    nn.Linear order W1 b1 W2 b2 W3 b3) (include/nfdpf.h nfdpf_cos_measurement_backward)."""
    require_device(x, "cos_measurement_backward")
    B, N, _ = x.shape
    enc, x, g_lik = _c(enc), _c(x), _c(g_lik)
    E = enc.shape[-1]
    g_enc = torch.empty_like(enc)
    gx = torch.empty_like(x)
    gp = torch.empty(1648, device=x.device, dtype=f32)
    nb = int(lib().nfdpf_cos_measurement_backward_workspace(B, N))
    ws = torch.empty(max(1, nb // 4), device=x.device, dtype=f32)
    check(lib().nfdpf_cos_measurement_backward(ptr(pe_blob), ptr(enc), ptr(x), ptr(g_lik), B, N, E, ptr(g_enc),
                                               ptr(gx), ptr(gp), ptr(ws), stream_ptr(x.device)),
          "nfdpf_cos_measurement_backward")
    return g_enc, gx, gp


def particle_encoder_forward(pe_blob, x):
    """PE(x) -> [B*N, 32] (nfdpf_particle_encoder mode 0)."""
    require_device(x, "particle_encoder_forward")
    B, N, _ = x.shape
    x = _c(x)
    e = torch.empty((B * N, 32), device=x.device, dtype=f32)
    check(lib().nfdpf_particle_encoder(0, ptr(pe_blob), ptr(x), B, N, None, ptr(e), None, None, None,
                                       stream_ptr(x.device)), "nfdpf_particle_encoder")
    return e


def particle_encoder_backward(pe_blob, x, g_e):
    """-> (g_x [B, N, 2], g_params [1648] nn.Linear order) (nfdpf_particle_encoder mode 1)."""
    require_device(x, "particle_encoder_backward")
    B, N, _ = x.shape
    x, g_e = _c(x), _c(g_e)
    gx = torch.empty_like(x)
    gp = torch.empty(1648, device=x.device, dtype=f32)
    nb = int(lib().nfdpf_cos_measurement_backward_workspace(B, N))
    ws = torch.empty(max(1, nb // 4), device=x.device, dtype=f32)
    check(lib().nfdpf_particle_encoder(1, ptr(pe_blob), ptr(x), B, N, ptr(g_e), None, ptr(gx), ptr(gp), ptr(ws),
                                       stream_ptr(x.device)), "nfdpf_particle_encoder")
    return gx, gp


def nn_measurement_backward(meas_blob, enc, es, g_lik):
    """Backward of the NN likelihood head -> (g_e [B*N, 32], g_enc [B, 32], g_params [8385] in
    nn.Linear order) for encodings es = PE(x) [B*N, 32] (nfdpf_nn_measurement_backward)."""
    require_device(es, "nn_measurement_backward")
    B, N = g_lik.shape
    enc, es, g_lik = _c(enc), _c(es), _c(g_lik)
    g_e = torch.empty_like(es)
    g_enc = torch.empty_like(enc)
    gp = torch.empty(8385, device=es.device, dtype=f32)
    nb = int(lib().nfdpf_nn_measurement_backward_workspace(B, N))
    ws = torch.empty(max(1, nb // 4), device=es.device, dtype=f32)
    check(lib().nfdpf_nn_measurement_backward(ptr(meas_blob), ptr(enc), ptr(es), ptr(g_lik), B, N, enc.shape[-1],
                                              ptr(g_e), ptr(g_enc), ptr(gp), ptr(ws), stream_ptr(es.device)),
          "nfdpf_nn_measurement_backward")
    return g_e, g_enc, gp


_ws = {}


def workspace(nbytes: int, device, tag="ot") -> torch.Tensor:
    key = (tag, str(device))
    t = _ws.get(key)
    if t is None or t.numel() < nbytes:
        t = _ws[key] = torch.empty(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
    return t


def _aligned_ptr(t: torch.Tensor) -> int:
    p = t.data_ptr()
    return (p + 255) // 256 * 256


def ot_resample(x, w, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, row_base=0, gate=None,
                stop_at=None, poll=None, keep=None):
    """resampler_ot (resamplers.py:62-70) -> (x', w', flat idx, iterations int32[1]).

    ``stop_at`` (device int32[1], iterations encoding): run exactly that many Sinkhorn
    iterations instead of the batch-coupled stop rule (include/nfdpf.h) -- the second pass
    of a batch sharded over ranks.  ``poll`` (default: unless the stream is being captured
    into a graph): follow the loop's progress from the host and stop enqueueing iteration
    launches once it has stopped.  ``keep``: a private workspace (ot_workspace) to run in
    instead of the shared one -- it then holds the state ot_transport_backward needs."""
    require_device(x, "ot_resample")
    B, N, D = x.shape
    if D != 2:
        raise L.NfdpfError("ot_resample: the HIP Sinkhorn is built for 2-D particles (state_dim = 2)")
    # rows read in place when each row is contiguous (one step of a [B, T, N, 2] history:
    # nfdpf_ot_resample_rs), else a contiguous copy
    if not (x.dtype == torch.float32 and x.stride(2) == 1 and x.stride(1) == 2 and x.stride(0) >= 2 * N):
        x = _c(x)
    if not (w.dtype == torch.float32 and w.stride(1) == 1 and w.stride(0) >= N):
        w = _c(w)
    xo = torch.empty((B, N, 2), device=x.device, dtype=torch.float32)
    wo = torch.empty((B, N), device=x.device, dtype=torch.float32)
    idx = torch.empty((B, N), device=x.device, dtype=torch.int64)
    it = torch.empty(1, device=x.device, dtype=torch.int32)  # (the apply launch writes it, gate off included)
    if poll is None:
        poll = not torch.cuda.is_current_stream_capturing()
    nb = int(lib().nfdpf_ot_workspace_bytes(B, N))
    ws = workspace(nb, x.device) if keep is None else keep
    check(lib().nfdpf_ot_resample_rs(ptr(x), int(x.stride(0)), ptr(w), int(w.stride(0)), B, N, float(eps),
                                     float(scaling), float(threshold), int(max_iter), int(row_base), ptr(xo),
                                     ptr(wo), ptr(idx), ptr(it), _aligned_ptr(ws), ptr(gate), ptr(stop_at),
                                     int(bool(poll)), stream_ptr(x.device)),
          "nfdpf_ot_resample")
    return xo, wo, idx, it


def ot_history(B, N, max_iter, device) -> torch.Tensor:
    """A private potential history for ot_sinkhorn_local / ot_sinkhorn_finish."""
    nb = int(lib().nfdpf_ot_history_bytes(B, N, int(max_iter)))
    return torch.empty(max(nb, 256) + 256, dtype=torch.uint8, device=device)


def ot_sinkhorn_local(x, w, eps, scaling, threshold, max_iter, ws, hist, gate=None, poll=None):
    """Phase 1 of a sharded Sinkhorn call (include/nfdpf.h): the loop with this rank's stop
    rule, every state's potentials kept in ``hist`` -> the local count (int32[1])."""
    require_device(x, "ot_sinkhorn_local")
    B, N, D = x.shape
    if D != 2:
        raise L.NfdpfError("ot_sinkhorn_local: the HIP Sinkhorn is built for 2-D particles (state_dim = 2)")
    it = torch.zeros(1, device=x.device, dtype=torch.int32)
    if poll is None:
        poll = not torch.cuda.is_current_stream_capturing()
    check(lib().nfdpf_ot_sinkhorn_local(ptr(x), ptr(w), B, N, float(eps), float(scaling), float(threshold),
                                        int(max_iter), ptr(it), _aligned_ptr(ws), _aligned_ptr(hist), ptr(gate),
                                        int(bool(poll)), stream_ptr(x.device)), "nfdpf_ot_sinkhorn_local")
    return it


def ot_sinkhorn_finish(x, eps, scaling, threshold, max_iter, row_base, ws, hist, stop_at, gate=None):
    """Phase 2: the tail of the call at state ``stop_at`` (the MIN over ranks of phase 1's
    counts) -> (x', w', flat idx)."""
    B, N, _ = x.shape
    xo = torch.empty_like(x)
    wo = torch.empty((B, N), device=x.device, dtype=f32)
    idx = torch.empty((B, N), device=x.device, dtype=torch.int64)
    check(lib().nfdpf_ot_sinkhorn_finish(ptr(x), B, N, float(eps), float(scaling), float(threshold), int(max_iter),
                                         int(row_base), ptr(xo), ptr(wo), ptr(idx), None, _aligned_ptr(ws),
                                         _aligned_ptr(hist), ptr(gate), ptr(stop_at), stream_ptr(x.device)),
          "nfdpf_ot_sinkhorn_finish")
    return xo, wo, idx


def ot_resample_sharded(x, w, eps=0.1, scaling=0.75, threshold=1e-3, max_iter=100, row_base=0, group=None,
                        gate=None, poll=None, keep=None):
    """ot_resample for this rank's rows of a batch sharded over ``group`` -- the unsharded
    call's result bit for bit, no Sinkhorn iteration run twice (include/nfdpf.h): the loop
    with the local stop rule keeping every state's potentials, the MIN of the stop count over
    the ranks (one int32 all-reduce on the stream, resamplers.py:126-129: the first row to
    converge anywhere ends the loop), then the tail at that state."""
    import torch.distributed as dist
    B, N, _ = x.shape
    x, w = _c(x), _c(w)
    ws = workspace(int(lib().nfdpf_ot_workspace_bytes(B, N)), x.device) if keep is None else keep
    hist = workspace(int(lib().nfdpf_ot_history_bytes(B, N, int(max_iter))), x.device, tag="ot_hist")
    it = ot_sinkhorn_local(x, w, eps, scaling, threshold, max_iter, ws, hist, gate, poll)
    dist.all_reduce(it, op=dist.ReduceOp.MIN, group=group)
    xo, wo, idx = ot_sinkhorn_finish(x, eps, scaling, threshold, max_iter, row_base, ws, hist, it, gate)
    return xo, wo, idx, it


def ot_workspace(B, N, device) -> torch.Tensor:
    """A private OT workspace (the forward state of one call, for its backward)."""
    nb = int(lib().nfdpf_ot_workspace_bytes(B, N))
    return torch.empty(max(nb, 256) + 256, dtype=torch.uint8, device=device)


def ot_transport_backward(ws, g_out, eps, gate=None):
    """dL/dx of ot_resample's x' = T x with T constant (resamplers.py:234-264): T^T g_out,
    from the state the forward left in ``ws`` (include/nfdpf.h nfdpf_ot_transport_backward)."""
    require_device(g_out, "ot_transport_backward")
    B, N, D = g_out.shape
    g_out = _c(g_out)
    gx = torch.empty_like(g_out)
    check(lib().nfdpf_ot_transport_backward(ptr(g_out), B, N, float(eps), ptr(gx), _aligned_ptr(ws), ptr(gate),
                                            stream_ptr(g_out.device)), "nfdpf_ot_transport_backward")
    return gx


def ot_stats(device=None):
    """(iterations or -1, exact-fallback count) of the last ot_resample on ``device``
    (synchronous; diagnostics for tests and benchmarks)."""
    import ctypes
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    ws = _ws.get(("ot", str(dev)))
    if ws is None:
        raise L.NfdpfError("ot_stats: no ot_resample has run on this device")
    out = (ctypes.c_int32 * 2)()
    torch.cuda.synchronize(dev)
    check(lib().nfdpf_ot_stats(_aligned_ptr(ws), ctypes.addressof(out)), "nfdpf_ot_stats")
    return int(out[0]), int(out[1])


def ess_gate(inv_ess, N, force=False, out=None):
    """DPFs.py:163-165 gate as a device int32[1] (no host sync)."""
    B = inv_ess.shape[0]
    g = out if out is not None else torch.empty(1, device=inv_ess.device, dtype=torch.int32)
    check(lib().nfdpf_ess_gate(ptr(inv_ess), B, N, int(bool(force)), ptr(g), stream_ptr(inv_ess.device)),
          "nfdpf_ess_gate")
    return g


def normalize_log_probs(logw, add=0.0):
    """normalize_log_probs (utils.py:39-44) + add -> (p, 1/sum p^2)."""
    require_device(logw, "normalize_log_probs")
    lw = _c(logw)
    B, N = lw.shape
    p = torch.empty_like(lw)
    ie = torch.empty(B, device=lw.device, dtype=f32)
    check(lib().nfdpf_normalize_log_probs(ptr(lw), B, N, float(add), ptr(p), ptr(ie), stream_ptr(lw.device)),
          "nfdpf_normalize_log_probs")
    return p, ie


def measurement(kind: str, pe_blob, meas_blob, n_flows, enc, x, prior_std=2.5):
    """measurement models (model/models.py:206-278) -> lik [B,N]."""
    require_device(x, "measurement")
    enc, x = _c(enc), _c(x)
    B, N, _ = x.shape
    lik = torch.empty((B, N), device=x.device, dtype=f32)
    check(lib().nfdpf_measurement(L.MEAS[kind], ptr(pe_blob), ptr(meas_blob), int(n_flows), ptr(enc), ptr(x),
                                  B, N, enc.shape[-1], float(prior_std), ptr(lik), stream_ptr(x.device)),
          "nfdpf_measurement")
    return lik


def cglow_measurement(pe_blob, glow_blob, enc, x, K=1, out=None):
    """Conditional-GLOW likelihood (model/models.py:280-303) WITHOUT the row-max shift:
    enc [B, 192] (or rows of a strided [B, T, 192] view), x [B, N, 2] (rows may be strided)
    -> raw lik [B, N]."""
    require_device(x, "cglow_measurement")
    B, N, _ = x.shape
    if x.stride(2) != 1 or x.stride(1) != 2:
        x = x.contiguous()
    if enc.stride(-1) != 1:
        enc = enc.contiguous()
    if enc.shape[-1] != 192:
        raise L.NfdpfError("cglow_measurement: frame encodings must be 192 wide (--hiddensize 192)")
    if int(glow_blob.numel()) != int(lib().nfdpf_cglow_params_size(int(K))):
        raise L.NfdpfError("cglow_measurement: parameter blob does not match flow_depth K")
    lik = out if out is not None else torch.empty((B, N), device=x.device, dtype=f32)
    check(lib().nfdpf_cglow_measurement(ptr(pe_blob), ptr(glow_blob), int(K), ptr(enc), enc.stride(0), ptr(x),
                                        x.stride(0), B, N, ptr(lik), lik.stride(0), stream_ptr(x.device)),
          "nfdpf_cglow_measurement")
    return lik


def cglow_measurement_backward(pe_blob, glow_blob, enc, x, g_lik, K=1):
    """Backward of cglow_measurement (raw lik, no row-max shift): enc [B, 192], x [B, N, 2],
    g_lik [B, N] -> (g_enc [B, 192], g_x [B, N, 2], g_glow [blob], g_pe [blob])
    (nfdpf_cglow_measurement_backward: per-particle dL/dy summed over each row's N here)."""
    require_device(x, "cglow_measurement_backward")
    B, N, _ = x.shape
    x, enc, g_lik = _c(x), _c(enc), _c(g_lik)
    if enc.shape[-1] != 192:
        raise L.NfdpfError("cglow_measurement_backward: frame encodings must be 192 wide (--hiddensize 192)")
    if int(glow_blob.numel()) != int(lib().nfdpf_cglow_params_size(int(K))):
        raise L.NfdpfError("cglow_measurement_backward: parameter blob does not match flow_depth K")
    gx = torch.empty_like(x)
    gy = torch.empty((B * N, 192), device=x.device, dtype=f32)
    g_glow = torch.empty_like(glow_blob)
    g_pe = torch.empty_like(pe_blob)
    nb = int(lib().nfdpf_cglow_backward_workspace(B * N))
    ws = torch.empty(max(1, nb // 4), device=x.device, dtype=f32)
    check(lib().nfdpf_cglow_measurement_backward(ptr(pe_blob), ptr(glow_blob), int(K), ptr(enc), enc.stride(0), ptr(x),
                                                 x.stride(0), B, N, ptr(g_lik), g_lik.stride(0), ptr(gx), ptr(gy),
                                                 ptr(g_glow), ptr(g_pe), ptr(ws), stream_ptr(x.device)),
          "nfdpf_cglow_measurement_backward")
    return gy.view(B, N, 192).sum(1), gx, g_glow, g_pe


def cglow_flow_backward(glow_blob, x, y, g_z, g_nll, K=1):
    """Backward of cglow_flow: x, y [M,3,8,8], g_z [M,12,4,4] (or None), g_nll [M] -> (g_x, g_y
    [M,3,8,8], g_glow [blob]) (nfdpf_cglow_flow_backward)."""
    require_device(x, "cglow_flow_backward")
    M = x.shape[0]
    x, y = _c(x), _c(y)
    g_nll = _c(g_nll) if g_nll is not None else torch.zeros((M,), device=x.device, dtype=f32)
    g_z = _c(g_z) if g_z is not None else None
    gx = torch.empty_like(x)
    gy = torch.empty_like(y)
    g_glow = torch.empty_like(glow_blob)
    nb = int(lib().nfdpf_cglow_backward_workspace(M))
    ws = torch.empty(max(1, nb // 4), device=x.device, dtype=f32)
    check(lib().nfdpf_cglow_flow_backward(ptr(_c(glow_blob)), int(K), ptr(x), ptr(y), int(M),
                                          ptr(g_z) if g_z is not None else None, ptr(g_nll), ptr(gx), ptr(gy),
                                          ptr(g_glow), ptr(ws), stream_ptr(x.device)), "nfdpf_cglow_flow_backward")
    return gx, gy, g_glow


def cglow_flow(glow_blob, x, y, K=1):
    """CondGlowModel.forward(x, y) (nf/cglow/CGlowModel.py:167-176) -> (z [M,12,4,4], nll [M]);
    x, y [M,3,8,8] (the condition and the flow input, per sample)."""
    require_device(x, "cglow_flow")
    M = x.shape[0]
    if tuple(x.shape[1:]) != (3, 8, 8) or tuple(y.shape) != tuple(x.shape):
        raise L.NfdpfError(f"cglow_flow: x and y must both be [M, 3, 8, 8] (got {tuple(x.shape)}, {tuple(y.shape)})")
    x, y = _c(x), _c(y)
    z = torch.empty((M, 12, 4, 4), device=x.device, dtype=f32)
    nll = torch.empty((M,), device=x.device, dtype=f32)
    check(lib().nfdpf_cglow_flow(ptr(_c(glow_blob)), int(K), ptr(x), ptr(y), int(M), ptr(z), ptr(nll),
                                 stream_ptr(x.device)), "nfdpf_cglow_flow")
    return z, nll


def particle_init(start_xy, B, N, width, true_state, seed, row_base=0, device=None):
    """particle_initialization (utils.py:46-62), device RNG -> (x [B,N,2], logw [B,N])."""
    device = device if device is not None else start_xy.device
    x = torch.empty((B, N, 2), device=device, dtype=f32)
    lw = torch.empty((B, N), device=device, dtype=f32)
    s = _c(start_xy) if start_xy is not None else None
    check(lib().nfdpf_particle_init(ptr(s), B, N, float(width), int(bool(true_state)), int(seed) & (2**64 - 1),
                                    int(row_base), ptr(x), ptr(lw), stream_ptr(device)), "nfdpf_particle_init")
    return x, lw


def rqs(x, W, H, D, inverse=False, left=-1.0, right=1.0, bottom=-1.0, top=1.0, tails=True, min_bin_width=1e-3,
        min_bin_height=1e-3, min_derivative=1e-3):
    """The rational-quadratic spline (include/nfdpf.h nfdpf_rqs) -> (y, logdet), shapes of
    ``x``.  W, H: x.shape + (K,); D: x.shape + (K - 1,) (unconstrained_RQS, nf/utils.py:23-53,
    tails pass through) or x.shape + (K + 1,) (RQS, :55-147)."""
    require_device(x, "rqs")
    shape = x.shape
    K = W.shape[-1]
    x, W, H, D = _c(x), _c(W), _c(H), _c(D)
    M = x.numel()
    full = D.shape[-1] == K + 1
    if W.numel() != M * K or H.numel() != M * K or D.numel() != M * (K + 1 if full else K - 1):
        raise ValueError(f"rqs: parameter shapes {tuple(W.shape)}, {tuple(H.shape)}, {tuple(D.shape)} do not match "
                         f"{M} inputs x {K} bins")
    y = torch.empty_like(x)
    ld = torch.empty_like(x)
    check(lib().nfdpf_rqs(ptr(x), ptr(W), ptr(H), ptr(D), M, K, int(full), int(bool(inverse)), float(left),
                          float(right), float(bottom), float(top), int(bool(tails)), float(min_bin_width),
                          float(min_bin_height), float(min_derivative), ptr(y), ptr(ld), stream_ptr(x.device)),
          "nfdpf_rqs")
    return y.reshape(shape), ld.reshape(shape)


def filter_step(desc: L.FilterDesc, device):
    check(lib().nfdpf_filter_step(desc, stream_ptr(device)), "nfdpf_filter_step")


def tiled_tiles(N: int) -> int:
    return int(lib().nfdpf_filter_tiled_tiles(N))


def tiled_workspace(B: int, N: int, T: int, device) -> torch.Tensor:
    return workspace(int(lib().nfdpf_filter_tiled_workspace_bytes(B, N, T)), device, tag="tiled")


def pass_workspace(B: int, N: int, T: int, device, owner=None) -> torch.Tensor:
    """Workspace of the one-launch pass (nfdpf_filter_pass_tiled): a header (the granule tags'
    epoch, the abort word), the row exchanges' granules and the per-wave prediction /
    obs-likelihood partials.  Kept on ``owner`` (one per FilterEngine: passes of two engines --
    e.g. on two streams -- never share granules or an abort word; module-level without one) and
    zeroed, stream-ordered, when it is new or its (B, N, T) layout changed (include/nfdpf.h):
    stale granules of another layout must not carry a live tag."""
    store = owner.__dict__ if owner is not None else _ws
    nbytes = int(lib().nfdpf_filter_pass_workspace_bytes(B, N, T))
    t, layout = store.get("_nfdpf_pass_ws", (None, None))
    if t is None or t.device != torch.device(device) or t.numel() < nbytes + 256:
        t = torch.zeros(max(nbytes, 256) + 256, dtype=torch.uint8, device=device)
    elif layout != (B, N, T):
        t.zero_()
    store["_nfdpf_pass_ws"] = (t, (B, N, T))
    return t


def filter_init(start_state, B, N, width, true_state, seed, row_base, device, ess_out, vel_input=None, T=0):
    """particle_init + normalize_log_probs + tiled_init in one launch (nfdpf_filter_init, N <= 1024)
    -> (x [B,N,2], logw [B,N], p0 [B,N], inv_ess [B], vel_steps [T,B,2] or None); the t = 0 gate
    partials into ``ess_out`` ([B, tiles, 4] float64).  ``start_state`` [B, >= 4] (x, y, vx, vy);
    with ``vel_input`` [B, >= T - 1, 2] also every step's velocity (the start velocity, then
    vel_input[:, t - 1]) in the descriptor's [T][B][2] layout."""
    x = torch.empty((B, N, 2), device=device, dtype=f32)
    lw = torch.empty((B, N), device=device, dtype=f32)
    p = torch.empty((B, N), device=device, dtype=f32)
    ie = torch.empty(B, device=device, dtype=f32)
    st = _c(start_state)
    vel = vi = None
    if vel_input is not None:
        vi = _c(vel_input)
        vel = torch.empty((T, B, 2), device=device, dtype=f32)
    check(lib().nfdpf_filter_init(ptr(st), st.shape[1], ptr(vi), vi.shape[1] * 2 if vi is not None else 2, int(T), B,
                                  N, float(width), int(bool(true_state)), int(seed) & (2**64 - 1), int(row_base),
                                  ptr(x), ptr(lw), ptr(p), ptr(ie), ptr(ess_out), ptr(vel), stream_ptr(device)),
          "nfdpf_filter_init")
    return x, lw, p, ie, vel


class HostMapped:
    """Slots of pinned, device-mapped, coherent host memory (nfdpf_host_mapped_alloc): a kernel
    writes a slot through its device address, the host reads it (numpy view) once an event
    behind that kernel has completed -- no copy launch.  ``take()`` hands out slots round robin;
    ``take(reserve=True)`` (a slot baked into a captured graph) is never handed out again.
    Allocated on construction: not while a stream is being captured."""

    def __init__(self, slots: int = 64, slot_bytes: int = 64):
        import ctypes
        import numpy as np
        self.slot_bytes, self.slots = slot_bytes, slots
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().nfdpf_host_mapped_alloc(slots * slot_bytes, ctypes.byref(h), ctypes.byref(d)),
              "nfdpf_host_mapped_alloc")
        self._host, self._dev = h.value, d.value
        buf = (ctypes.c_int32 * (slots * slot_bytes // 4)).from_address(self._host)
        self._view = np.frombuffer(buf, dtype=np.int32).reshape(slots, slot_bytes // 4)
        self._free = list(range(slots))
        self._next = 0

    def take(self, reserve: bool = False):
        """-> (device address, int32 numpy view of the slot, lease).  ``reserve``: the slot stays
        out of the round robin until the returned lease is released (``lease.release()``, or
        when the lease object is dropped -- e.g. with the pending state of the captured pass that
        holds it); lease is None for an unreserved slot.  None when every slot is reserved (the
        caller then keeps its flags in device memory)."""
        if not self._free:
            return None
        k = self._free[self._next % len(self._free)]
        lease = None
        if reserve:
            self._free.remove(k)
            lease = _SlotLease(self, k)
        else:
            self._next += 1
        return self._dev + k * self.slot_bytes, self._view[k], lease

    def _release(self, k: int):
        if k not in self._free:
            self._free.append(k)

    def __del__(self):
        try:
            if getattr(self, "_host", None):
                lib().nfdpf_host_mapped_free(self._host)
                self._host = None
        except Exception:  # interpreter shutdown
            pass


class GateExchange:
    """The sharded gated pass's cross-rank gate exchange (include/nfdpf.h nfdpf_gate_xchg_*): this
    rank's buffer of uncached device memory and every peer's, mapped from its IPC handle --
    ``peers`` (int64 [world] on the device) is the pass's d.gate_peers.  Set up collectively over
    the shard's process group (every rank allocates and exports, then maps the others); ``create``
    returns None on EVERY rank when any rank could not (the caller then keeps the exchange-free
    modes).  Unmapped / freed when dropped."""

    def __init__(self, own, opened, peers):
        self._own, self._opened, self.peers = own, opened, peers

    @staticmethod
    def create(B_global: int, rank: int, world: int, group, device) -> "Optional[GateExchange]":
        import ctypes
        import torch.distributed as dist
        lb = lib()
        own, h = ctypes.c_void_p(), ctypes.create_string_buffer(64)
        ok = lb.nfdpf_gate_xchg_alloc(int(lb.nfdpf_gate_xchg_bytes(B_global)), ctypes.byref(own),
                                      ctypes.cast(h, ctypes.c_void_p)) == L.NFDPF_OK
        hs = [None] * world
        dist.all_gather_object(hs, h.raw if ok else None, group=group)
        ptrs, opened = [], []
        ok = ok and all(x is not None for x in hs)
        if ok:
            for r, hb in enumerate(hs):
                if r == rank:
                    ptrs.append(own.value)
                    continue
                p = ctypes.c_void_p()
                hbuf = ctypes.create_string_buffer(hb, 64)
                if lb.nfdpf_gate_xchg_open(ctypes.cast(hbuf, ctypes.c_void_p), ctypes.byref(p)) != L.NFDPF_OK:
                    ok = False
                    break
                ptrs.append(p.value)
                opened.append(p.value)
        oks = [None] * world
        dist.all_gather_object(oks, bool(ok), group=group)
        if not all(oks):
            for p in opened:
                lb.nfdpf_gate_xchg_close(p)
            if own.value:
                lb.nfdpf_gate_xchg_free(own.value)
            return None
        return GateExchange(own.value, opened, torch.tensor(ptrs, dtype=torch.int64, device=device))

    def __del__(self):
        try:
            lb = lib()
            for p in self._opened:
                lb.nfdpf_gate_xchg_close(p)
            lb.nfdpf_gate_xchg_free(self._own)
        except Exception:  # interpreter shutdown
            pass


class _SlotLease:
    """A reserved HostMapped slot; returned to its pool on release() or when dropped."""

    def __init__(self, pool: HostMapped, k: int):
        self._pool, self.k = pool, k

    def release(self):
        pool, self._pool = self._pool, None
        if pool is not None:
            pool._release(self.k)

    def __del__(self):
        try:
            self.release()
        except Exception:  # interpreter shutdown
            pass


def tiled_init(p0: torch.Tensor, out: torch.Tensor):
    B, N = p0.shape
    check(lib().nfdpf_filter_tiled_init(ptr(p0), B, N, ptr(out), stream_ptr(p0.device)), "nfdpf_filter_tiled_init")
    return out


def ess_gate_tiled(parts, N, t, force=False, out=None):
    """Gate of step ``t`` from the [B, tiles, 4] softmax partials of step t-1 (include/nfdpf.h)."""
    B = parts.shape[0]
    g = out if out is not None else torch.empty(1, device=parts.device, dtype=torch.int32)
    check(lib().nfdpf_ess_gate_tiled(ptr(parts), B, N, int(t), int(bool(force)), ptr(g),
                                     stream_ptr(parts.device)), "nfdpf_ess_gate_tiled")
    return g


def ess_gate_tiled_batch(parts, N, t0=0, force=False, out=None):
    """Gates of T consecutive steps from [T, B_global, tiles, 4] input partials -> int32 [T]
    (the verification of a speculative sharded pass, include/nfdpf.h)."""
    T, B = parts.shape[0], parts.shape[1]
    g = out if out is not None else torch.empty(T, device=parts.device, dtype=torch.int32)
    parts = parts.to(torch.float64).contiguous()
    check(lib().nfdpf_ess_gate_tiled_batch(ptr(parts), T, B, N, int(t0), int(bool(force)), ptr(g),
                                           stream_ptr(parts.device)), "nfdpf_ess_gate_tiled_batch")
    return g


def ess_row_terms(parts, N, t0=0, out=None):
    """[T, B, tiles, 4] step partials -> float32 [T * B + 1]: the rows' gate terms (1 / sum p^2,
    t-major), then this device's hand-off fault counter (read and cleared) as int32 bits
    (include/nfdpf.h nfdpf_ess_row_terms)."""
    T, B = parts.shape[0], parts.shape[1]
    parts = parts.to(torch.float64).contiguous()
    terms = out if out is not None else torch.empty(T * B + 1, device=parts.device, dtype=torch.float32)
    check(lib().nfdpf_ess_row_terms(ptr(parts), T, B, N, int(t0), ptr(terms), stream_ptr(parts.device)),
          "nfdpf_ess_row_terms")
    return terms


def ess_gate_terms(terms, N, force=False, out=None):
    """float32 [T, B_global] gathered gate terms -> the T batch-global gates int32 [T]
    (nfdpf_ess_gate_terms: ATen's cascade mean over the rows, as nfdpf_ess_gate_tiled_batch)."""
    T, B = terms.shape
    terms = terms.contiguous()
    g = out if out is not None else torch.empty(T, device=terms.device, dtype=torch.int32)
    check(lib().nfdpf_ess_gate_terms(ptr(terms), T, B, N, int(bool(force)), ptr(g), stream_ptr(terms.device)),
          "nfdpf_ess_gate_terms")
    return g


def pass_verify(parts, lw_sum, N, t0=0):
    """[T, B, tiles, 4] step partials and [B, T] lw_sum of a one-shard speculative pass ->
    (gates int32 [T], flags int32 [2] = {gates fired, hand-off faults since the last read},
    obs float32 [] = the obs-likelihood), no host sync (include/nfdpf.h nfdpf_pass_verify)."""
    T, B = parts.shape[0], parts.shape[1]
    parts = parts.to(torch.float64).contiguous()
    lw_sum = lw_sum.to(torch.float32).contiguous()
    assert tuple(lw_sum.shape) == (B, T)
    g = torch.empty(T, device=parts.device, dtype=torch.int32)
    flags = torch.empty(2, device=parts.device, dtype=torch.int32)
    obs = torch.empty((), device=parts.device, dtype=torch.float32)
    check(lib().nfdpf_pass_verify(ptr(parts), ptr(lw_sum), T, B, N, int(t0), ptr(g), ptr(flags), ptr(obs),
                                  stream_ptr(parts.device)), "nfdpf_pass_verify")
    return g, flags, obs


def filter_step_tiled(desc: L.FilterDesc, ws: torch.Tensor, device):
    check(lib().nfdpf_filter_step_tiled(desc, _aligned_ptr(ws), stream_ptr(device)), "nfdpf_filter_step_tiled")
