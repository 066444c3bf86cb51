"""Pack nn.Module parameters into the flat fp32 blobs the kernels read (include/nfdpf.h).

Blobs are cached per module and rebuilt only when a parameter changes (tensor version
counter or storage), so an optimizer step is picked up and an unchanged model pays nothing.
"""
from __future__ import annotations

import torch
import torch.nn as nn


def _linears(seq: nn.Module):
    return [m for m in seq.modules() if isinstance(m, nn.Linear)]


def _same(p):
    return p


def fcnn_tensors(fcnn: nn.Module, get=_same):
    """FCNN(in, out, H): W1 b1 W2 b2 W3 b3 (nf/flows.py:101-114)."""
    out = []
    for lin in _linears(fcnn.network):
        out += [get(lin.weight), get(lin.bias)]
    return out


def pair(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Interleave two equally shaped tensors elementwise: out[..., 0] = a, out[..., 1] = b.
    The kernels read such pairs as one 8-byte float2 and update both with one v_pk_fma_f32."""
    return torch.stack([a, b], -1)


def row_pairs(w: torch.Tensor) -> torch.Tensor:
    """nn.Linear weight [out, in] -> [out/2][in][2]: output rows 2m and 2m+1 interleaved, so
    two outputs of a layer advance together in one packed FMA per input."""
    o, i = w.shape
    return w.reshape(o // 2, 2, i).transpose(1, 2)


def col_pairs(w: torch.Tensor) -> torch.Tensor:
    """nn.Linear weight [out, in] -> [in][out/2][2]: for each input, the weights of output
    rows 2m and 2m+1 adjacent, all output pairs contiguous -- an input-major layer reads one
    contiguous run per input (csrc/flows.hpp, particle encoder)."""
    o, i = w.shape
    return w.t().reshape(i, o // 2, 2)


def encoder_tensors(seq: nn.Module, get=_same):
    """Particle encoder Linear(2,16) Linear(16,32) Linear(32,E) (model/models.py:130-150) in
    the kernel layout: W1 row_pairs, W2 and W3 col_pairs, biases as they are."""
    l1, l2, l3 = _linears(seq)
    return [row_pairs(get(l1.weight)), get(l1.bias), col_pairs(get(l2.weight)), get(l2.bias),
            col_pairs(get(l3.weight)), get(l3.bias)]


def coupling_pair_tensors(t_net: nn.Module, s_net: nn.Module, half: int, get=_same):
    """Nets t and s of one coupling half, FCNN(half + O, half, H) each (nf/flows.py:101-114,
    183-190), interleaved t/s elementwise (csrc/flows.hpp ts_pair): core
    [W1[:, :half], W2, b2, W3, b3] then context [W1[:, half:], b1]."""
    (tw1, tb1), (tw2, tb2), (tw3, tb3) = [(get(m.weight), get(m.bias)) for m in _linears(t_net.network)]
    (sw1, sb1), (sw2, sb2), (sw3, sb3) = [(get(m.weight), get(m.bias)) for m in _linears(s_net.network)]
    return [pair(tw1[:, :half], sw1[:, :half]), pair(tw2, sw2), pair(tb2, sb2), pair(tw3, sw3),
            pair(tb3, sb3), pair(tw1[:, half:], sw1[:, half:]), pair(tb1, sb1)]


def realnvp_tensors(flow: nn.Module, get=_same):
    """RealNVP / RealNVP_cond flow (nf/flows.py:123-129, 183-190): pair (t1, s1), pair (t2, s2)."""
    half = flow.dim // 2
    return (coupling_pair_tensors(flow.t1, flow.s1, half, get) +
            coupling_pair_tensors(flow.t2, flow.s2, half, get))


def maf_tensors(flow: nn.Module, get=_same):
    """MAF flow: initial_param[2] then FCNN(i, 2, H) for i = 1..dim-1 (nf/flows.py:247-254)."""
    out = [get(flow.initial_param)]
    for layer in flow.layers:
        out += fcnn_tensors(layer, get)
    return out


def mlp_tensors(seq: nn.Module):
    """nn.Sequential of Linear layers (+activations): W, b per Linear, plain row-major."""
    out = []
    for lin in _linears(seq):
        out += [lin.weight, lin.bias]
    return out


def paired_mlp_tensors(seq: nn.Module):
    """likelihood_est MLP (model/models.py:119-128): W in row_pairs
    layout wherever the layer has an even number of outputs, biases as they are."""
    out = []
    for lin in _linears(seq):
        w = lin.weight
        out += [row_pairs(w) if w.shape[0] % 2 == 0 else w, lin.bias]
    return out


def _taps_last(w: torch.Tensor) -> torch.Tensor:
    """Conv weight [out][in][kh][kw] -> [kh][kw][in][out]: one tap's input channel feeds a
    contiguous run of output channels (csrc/cglow.hip)."""
    return w.permute(2, 3, 1, 0)


def _cond_net_tensors(m: nn.Module, get=_same):
    """CondActNorm / Cond1x1Conv conditioning net (nf/cglow/modules.py:84-101, 145-162):
    x_Con conv 0 as [k][out] (k = in, kh, kw), convs 2, 4 and the x_Linear layers as stored."""
    c0, c2, c4 = [l for l in m.x_Con if isinstance(l, nn.Conv2d)]
    l0, l2, l4 = _linears(m.x_Linear)
    w0 = get(c0.weight)
    return [w0.reshape(w0.shape[0], -1).t()] + [get(t) for t in (c0.bias, c2.weight, c2.bias, c4.weight, c4.bias,
                                                                   l0.weight, l0.bias, l2.weight, l2.bias,
                                                                   l4.weight, l4.bias)]


def cglow_tensors(glow: nn.Module, get=_same):
    """CondGlowModel (nf/cglow/CGlowModel.py) with K = 1, L = 1: the CondGlowStep's actnorm
    net, 1x1-conv net, then the affine coupling (modules.py:258-303) in the kernel layout of
    csrc/cglow.hip (Aff): resize_x / f convolutions tap-major, output channel fastest."""
    steps = [l for l in glow.flow.layers if hasattr(l, "affine")]
    if len(steps) != 1:
        raise ValueError(f"the CGLOW kernel is built for flow_depth K = 1 (got {len(steps)} steps)")
    st = steps[0]
    a = st.affine
    r0, r2, r4 = [l for l in a.resize_x if isinstance(l, nn.Conv2d)]
    f0, f2, f4 = [l for l in a.f if isinstance(l, nn.Conv2d)]
    w2 = get(f2.weight)
    return (_cond_net_tensors(st.actnorm, get) + _cond_net_tensors(st.invconv, get) +
            [_taps_last(get(r0.weight)), get(r0.bias), _taps_last(get(r2.weight)), get(r2.bias),
             _taps_last(get(r4.weight)), get(r4.bias),
             _taps_last(get(f0.weight)), get(f0.actnorm.bias), get(f0.actnorm.logs),
             w2.reshape(w2.shape[0], -1).t(), get(f2.actnorm.bias), get(f2.actnorm.logs),
             _taps_last(get(f4.weight)), get(f4.bias), get(f4.logs), get(f4.newbias)])


def flows_tensors(flows, get=_same):
    """``get`` maps each parameter to the tensor packed in its place (default: itself)."""
    out = []
    for f in flows:
        if hasattr(f, "initial_param"):
            out += maf_tensors(f, get)
        else:
            out += realnvp_tensors(f, get)
    return out


def blob_source_index(params, build) -> torch.Tensor:
    """For every entry of the blob ``build(get)`` packs, the index of its source element in the
    concatenation of ``params`` (flattened, in order).  The packing is a gather, so a blob
    gradient maps back to the parameters by one scatter with this index."""
    ids, off = {}, 0
    for p in params:
        ids[id(p)] = torch.arange(off, off + p.numel(), dtype=torch.int64).view(p.shape)
        off += p.numel()
    return torch.cat([t.reshape(-1) for t in build(lambda p: ids[id(p)])])


def blob_grad_to_params(owner: nn.Module, name: str, params, build, g_blob: torch.Tensor):
    """Scatter a gradient in blob layout back to per-parameter gradients (cached index)."""
    caches = owner.__dict__.setdefault("_nfdpf_blob_index", {})
    key = (name, str(g_blob.device)) + tuple(id(p) for p in params)
    idx = caches.get(key)
    if idx is None:
        idx = caches[key] = blob_source_index(params, build).to(g_blob.device)
    flat = torch.empty(sum(p.numel() for p in params), device=g_blob.device, dtype=g_blob.dtype)
    flat[idx] = g_blob
    out, off = [], 0
    for p in params:
        out.append(flat[off:off + p.numel()].view(p.shape).to(p.dtype))
        off += p.numel()
    return out


def blob_param_grads(owner: nn.Module, name: str, params, build, g_blob: torch.Tensor):
    """blob_grad_to_params for a parameter list of which the blob may pack only a subset:
    gradients of the packed parameters, None for the others (a parameter the forward does not
    read gets no gradient under autograd either, e.g. CondGlowModel's new_mean / new_logs with
    learn_top off)."""
    seen = {}

    def rec(p):
        seen[id(p)] = p
        return p
    build(rec)
    used = [p for p in params if id(p) in seen]
    grads = dict(zip([id(p) for p in used], blob_grad_to_params(owner, name, used, build, g_blob)))
    return [grads.get(id(p)) for p in params]


def splittable(flows) -> bool:
    """True when every flow is a RealNVP(_cond) on 2-D particles with hidden width 8: the
    layout of the split suffix (csrc/split.hpp)."""
    for f in flows:
        if hasattr(f, "initial_param") or getattr(f, "dim", None) != 2:
            return False
        if _linears(f.t1.network)[1].weight.shape != (8, 8):
            return False
    return True


def split_net_tensors(net: nn.Module):
    """One coupling net FCNN(1 + O, 1, 8) in the split layout (csrc/split.hpp): W1[:, 0],
    W2 and b2 with hidden units 2m, 2m+1 adjacent, W3 likewise, then {b3, 0} -- 90 floats."""
    (w1, _), (w2, b2), (w3, b3) = [(m.weight, m.bias) for m in _linears(net.network)]
    h = w2.shape[0]
    return [row_pairs(w1[:, :1]), row_pairs(w2), b2.reshape(h // 2, 2), w3.reshape(h // 2, 2),
            torch.cat([b3.reshape(1), b3.new_zeros(1)])]


def split_flow_tensors(flows):
    """The split suffix of a flow stack: per flow the nets t1, s1, t2, s2."""
    out = []
    for f in flows:
        for net in (f.t1, f.s1, f.t2, f.s2):
            out += split_net_tensors(net)
    return out


def filter_flow_tensors(flows):
    """The filter's dynamic / proposal stack: the pair layout (flows_tensors), then the
    split suffix when the stack allows it (include/nfdpf.h)."""
    return flows_tensors(flows) + (split_flow_tensors(flows) if splittable(flows) else [])


# 2 log2(e): tanh(a) = 1 - 2 / (1 + 2^(c a))
TANH_C = 2.0 / 0.6931471805599453


def pass_coupling_tensors(t_net: nn.Module, s_net: nn.Module, half: int):
    """One coupling half of the one-launch pass (csrc/filter_pass.hpp ts_half) in the pair
    layout of coupling_pair_tensors with the tanh algebra folded into the weights: with
    r = 1 / (1 + 2^y) a hidden unit's tanh is 1 - 2 r, so a layer that reads tanh outputs h
    reads r instead as W h + b = (b + sum_k W[:, k]) - 2 W r, and the next tanh's scale c =
    2 log2(e) goes into the layer producing its argument:
      W1' = c W1 (core and context columns), b1' = c b1,
      W2' = -2 c W2, b2' = c (b2 + rowsum W2),  W3' = -2 W3, b3' = b3 + rowsum W3
    (computed in float64, rounded once).  Each hidden unit then costs exp2 + add + rcp:
    the multiply by c and the 1 - 2 r fma of the plain layout are gone (nf/flows.py:101-114
    computes the same function; the rounding differs at the 1e-7 level)."""
    c = TANH_C
    nets = []
    for net in (t_net, s_net):
        (w1, b1), (w2, b2), (w3, b3) = [(m.weight.detach().double(), m.bias.detach().double())
                                        for m in _linears(net.network)]
        nets.append(dict(w1=c * w1[:, :half], w2=-2.0 * c * w2, b2=c * (b2 + w2.sum(1)), w3=-2.0 * w3,
                         b3=b3 + w3.sum(1), w1c=c * w1[:, half:], b1=c * b1))
    t, s = nets
    return [pair(t[k], s[k]).float() for k in ("w1", "w2", "b2", "w3", "b3", "w1c", "b1")]


def pass_flow_tensors(flows):
    """The one-launch pass's dynamic / proposal stack (nfdpf_filter_pass_tiled, include/nfdpf.h):
    per RealNVP(_cond) flow the halves (t1, s1), (t2, s2) as pass_coupling_tensors."""
    out = []
    for f in flows:
        half = f.dim // 2
        out += pass_coupling_tensors(f.t1, f.s1, half) + pass_coupling_tensors(f.t2, f.s2, half)
    return out


def mfma_frag(w: torch.Tensor) -> torch.Tensor:
    """A matrix W [M, K] (M a multiple of 16, K of 4) as the A operands of a chain of
    v_mfma_f32_16x16x4_f32 with features as rows and particles as columns (csrc/crnvp_mfma.hpp):
    [M / 16][lane 64][K / 4] with entry (MT, l, s) = W[16 MT + (l & 15)][16 (s >> 2) + 4 (l >> 4) +
    (s & 3)] -- K-step s reads, in lane group g, register s & 3 of the previous layer's M tile
    s >> 2, so chained layers exchange no data."""
    M, K = w.shape
    lane = torch.arange(64)
    s = torch.arange(K // 4)
    rows = (16 * torch.arange(M // 16))[:, None, None] + (lane & 15)[None, :, None]
    cols = 16 * (s >> 2)[None, None, :] + 4 * (lane >> 4)[None, :, None] + (s & 3)[None, None, :]
    return w[rows, cols]


def crnvp_mfma_tensors(encoder: nn.Module, flows):
    """The CRNVP measurement (model/models.py:256-278: particle encoder Linear(2,16) ReLU
    Linear(16,32) ReLU Linear(32,E), then RealNVP_cond flows of dim E with condition E) as the
    fragment blob of csrc/crnvp_mfma.hpp (offsets kCmf*): the encoder's layer 1 plain (it runs on
    VALU), layers 2 and 3 as mfma_frag; per flow and coupling half the nets t and s stacked as 16
    hidden rows (t 0-7, s 8-15) -- the fold over the condition columns W1[:, HALF:], layer 1 over
    u = W1[:, :HALF], layers 2 and 3 block-diagonal -- with the tanh algebra of
    pass_coupling_tensors folded in (float64, rounded once)."""
    l1, l2, l3 = _linears(encoder)
    f64 = lambda t: t.detach().double().cpu()  # noqa: E731
    out = [f64(l1.weight).reshape(-1), f64(l1.bias), mfma_frag(f64(l2.weight)).reshape(-1), f64(l2.bias),
           mfma_frag(f64(l3.weight)).reshape(-1), f64(l3.bias)]
    c = TANH_C
    for f in flows:
        half = f.dim // 2
        for t_net, s_net in ((f.t1, f.s1), (f.t2, f.s2)):
            nets = []
            for net in (t_net, s_net):
                (w1, b1), (w2, b2), (w3, b3) = [(f64(m.weight), f64(m.bias)) for m in _linears(net.network)]
                nets.append(dict(w1u=c * w1[:, :half], w1c=c * w1[:, half:], b1=c * b1, w2=-2.0 * c * w2,
                                 b2=c * (b2 + w2.sum(1)), w3=-2.0 * w3, b3=b3 + w3.sum(1)))
            t, s_ = nets
            H, O = t["w2"].shape[0], t["w3"].shape[0]
            # hidden row p of the 16: t-net unit j at 4 (j >> 1) + (j & 1), s-net unit j at
            # 4 (j >> 1) + 2 + (j & 1) -- the t units in registers 0-1 of every lane group, the s
            # units in registers 2-3, so layer 3's t outputs read K-steps 0-1 only and its s
            # outputs K-steps 2-3 (half of the block-diagonal layer's MFMAs skipped)
            j = torch.arange(H)
            pt, ps = 4 * (j >> 1) + (j & 1), 4 * (j >> 1) + 2 + (j & 1)

            def rows(a, b):
                o = torch.zeros((2 * H,) + tuple(a.shape[1:]), dtype=torch.float64)
                o[pt], o[ps] = a, b
                return o
            w2 = torch.zeros(2 * H, 2 * H, dtype=torch.float64)
            w2[pt[:, None], pt[None, :]] = t["w2"]
            w2[ps[:, None], ps[None, :]] = s_["w2"]
            w3 = torch.zeros(2 * O, 2 * H, dtype=torch.float64)
            w3[:O, pt] = t["w3"]
            w3[O:, ps] = s_["w3"]
            out += [mfma_frag(rows(t["w1c"], s_["w1c"])).reshape(-1),
                    mfma_frag(rows(t["w1u"], s_["w1u"])).reshape(-1),
                    mfma_frag(w2).reshape(-1), mfma_frag(w3).reshape(-1),
                    rows(t["b1"], s_["b1"]), rows(t["b2"], s_["b2"]), torch.cat([t["b3"], s_["b3"]])]
    return [x.float() for x in out]


def crnvp_mfma_ok(encoder: nn.Module, flows) -> bool:
    """The shapes csrc/crnvp_mfma.hpp is written for: encoder 2 -> 16 -> 32 -> 32, one or two
    RealNVP_cond flows of dim 32, condition 32, hidden 8."""
    try:
        l1, l2, l3 = _linears(encoder)
    except ValueError:
        return False
    if (l1.weight.shape, l2.weight.shape, l3.weight.shape) != ((16, 2), (32, 16), (32, 32)):
        return False
    if not 1 <= len(flows) <= 2:
        return False
    for f in flows:
        if hasattr(f, "initial_param") or getattr(f, "dim", None) != 32 or getattr(f, "obser_dim", None) != 32:
            return False
        if [tuple(m.weight.shape) for m in _linears(f.t1.network)] != [(8, 48), (8, 8), (16, 8)]:
            return False
    return True


class BlobCache:
    """Flat fp32 copy of a parameter set on one device in a kernel layout, rebuilt only when
    a source parameter changes (storage, version counter)."""

    def __init__(self):
        self._key = None
        self._blob = None

    def get(self, sources, build, device) -> torch.Tensor:
        key = (str(device),) + tuple((t.data_ptr(), t._version, t.numel()) for t in sources)
        if key != self._key:
            with torch.no_grad():
                flat = [t.detach().reshape(-1).to(device=device, dtype=torch.float32) for t in build()]
                self._blob = torch.cat(flat).contiguous() if flat else torch.zeros(1, device=device)
            self._key = key
        return self._blob


def blob(owner: nn.Module, name: str, source, build, device) -> torch.Tensor:
    """Cached blob stored on ``owner`` under ``name`` (not a registered buffer).  ``source``
    (a module, or a list of modules / tensors) keys the cache; ``build()`` returns the tensors to pack."""
    if isinstance(source, nn.Module):
        sources = list(source.parameters())
    else:
        sources = []
        for x in source:
            sources += list(x.parameters()) if isinstance(x, nn.Module) else [x]
    caches = owner.__dict__.setdefault("_nfdpf_blobs", {})
    cache = caches.get(name)
    if cache is None:
        cache = caches[name] = BlobCache()
    return cache.get(sources, build, device)
