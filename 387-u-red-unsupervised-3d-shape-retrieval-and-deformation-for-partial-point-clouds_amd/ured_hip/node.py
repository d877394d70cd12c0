"""Graph-node layers of DeformNet_MatchingNet on libured_hip.so (csrc/node.hip), as autograd
Functions over node-major [rows, C] tensors (rows = B x nodes).

NodeLinearFn   one Conv1d(k=1) over nodes: y = x W^T + b (+ residual); forward and both
               backward GEMMs on ured_node_gemm (out_proj; attention_graph/attention_gnn.py:20-32).
NodeProjFn     row-stacked projections (in_proj q|k|v of a self-attention, q and k|v of a
               cross-attention) over the parameters' own back-to-back memory (FlatAdam chains).
NodeFFNFn      ResidualAttentionMessagePropagation's update (attention_gnn.py:50-54):
               out = x + conv2(BN(relu(conv1(cat([first, message]))))) with
               FeedForwardNet_norm [2C, 2C, C] (attention_utils.py:62-86); the concatenation is
               read in place (two A sources), BatchNorm1d per node set (ured_node_bn_*).
ParamDecoderFn param_decoder (network/deformation_net.py:61,90): Conv 3C->256 -> ReLU ->
               Conv 256->6 on cat([global pair broadcast to the parts, part nodes]); the global
               half is a per-sample row bias (never broadcast).
Parameter gradients go straight into FlatAdam's flat gradient (ured_hip.optim.grad_slot):
written by the first use of a parameter in a backward, accumulated in the kernels by a second
use (the cross-attention module updates both node sets with the same weights), so autograd has
no gradient to copy or add.
Reference semantics: Conv1d over [B, C, nodes] == a linear map of each node row; BatchNorm1d
on [B, C, n] == per-channel statistics over the B*n node rows of one call.
"""
import ctypes

import torch
from torch.autograd import Function

from . import _lib, syncbn
from . import kernels as K
from .optim import grad_buffer, grad_slot

_P, _I, _LL, _F = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
MAX_SETS = 4


class NodeGemmDesc(ctypes.Structure):
    _fields_ = [("M", _I), ("N", _I), ("K", _I),
                ("A", _P), ("sam", _LL), ("sak", _LL),
                ("A2", _P), ("sam2", _LL), ("sak2", _LL), ("k1", _I),
                ("B", _P), ("sbk", _LL), ("sbn", _LL),
                ("B2", _P), ("sbk2", _LL), ("sbn2", _LL), ("n1", _I),
                ("C", _P), ("ldc", _LL), ("accumulate", _I),
                ("bias", _P),
                ("rowbias", _P), ("ldrb", _LL), ("rdiv", _I),
                ("relu_out", _I),
                ("gate", _P), ("ldgate", _LL),
                ("R", _P), ("ldR", _LL), ("R_ncols", _I),
                ("kind", _I)]


class NodeBNDesc(ctypes.Structure):
    _fields_ = [("N", _I), ("nsets", _I), ("off", _I * (MAX_SETS + 1)),
                ("Y", _P), ("ldy", _LL), ("relu_in", _I), ("training", _I),
                ("gamma", _P), ("beta", _P),
                ("running_mean", _P), ("running_var", _P), ("num_batches_tracked", _P),
                ("momentum", _F), ("eps", _F),
                ("mean", _P), ("invstd", _P),
                ("act", _P), ("ld_act", _LL),
                ("stats_out", _P), ("stats_in", _P)]


class NodeBNBwdDesc(ctypes.Structure):
    _fields_ = [("N", _I), ("nsets", _I), ("off", _I * (MAX_SETS + 1)),
                ("G", _P), ("ldg", _LL),
                ("Y", _P), ("ldy", _LL), ("relu_in", _I), ("training", _I),
                ("gamma", _P), ("mean", _P), ("invstd", _P),
                ("dY", _P), ("lddy", _LL),
                ("dgamma", _P), ("dbeta", _P), ("accumulate", _I),
                ("sums_out", _P), ("sums_in", _P)]


MAX_JOBS = 6
KIND_GEMM, KIND_COLSUM = 0, 1
_lib.register({"ured_node_gemm": [ctypes.POINTER(NodeGemmDesc), _P],
               "ured_node_gemm_batch": [ctypes.POINTER(ctypes.POINTER(NodeGemmDesc)), _I, _P],
               "ured_node_bn_fwd": [ctypes.POINTER(NodeBNDesc), _P],
               "ured_node_bn_bwd": [ctypes.POINTER(NodeBNBwdDesc), _P]})


def _ptr(t, off=0):
    return None if t is None else t.data_ptr() + 4 * off


def _mat(t):
    """(pointer, row stride) of a row-major 2-D view with unit column stride."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"node op: expected a 2-D view with unit column stride, got {tuple(t.shape)} {t.stride()}")
    return t.data_ptr(), t.stride(0)


def _rows(g):
    """g as a row-major 2-D view the node kernels read in place (any row stride >= its width,
    unit column stride: e.g. a column slice of NodeFFNFn's [d first | d message]), else a copy."""
    if g.dim() == 2 and g.stride(1) == 1 and g.stride(0) >= g.shape[1]:
        return g
    return g.contiguous()


def node_gemm_desc(M, N, K, A, sam, sak, B, sbk, sbn, C, ldc, *, A2=None, sam2=0, sak2=0, k1=None, accumulate=False,
                   bias=None, rowbias=None, ldrb=0, rdiv=1, relu_out=False, gate=None, ldgate=0, R=None, ldR=0,
                   R_ncols=None, B2=None, sbk2=0, sbn2=0, n1=None):
    """A ured_node_gemm descriptor; A / A2 / B / B2 / C / rowbias / gate / R are device addresses
    (int) or tensors (their data_ptr)."""
    def addr(x):
        return None if x is None else (x if isinstance(x, int) else x.data_ptr())
    d = NodeGemmDesc()
    d.M, d.N, d.K = int(M), int(N), int(K)
    d.A, d.sam, d.sak = addr(A), int(sam), int(sak)
    d.A2, d.sam2, d.sak2, d.k1 = addr(A2), int(sam2), int(sak2), int(K if k1 is None else k1)
    d.B, d.sbk, d.sbn = addr(B), int(sbk), int(sbn)
    d.B2, d.sbk2, d.sbn2, d.n1 = addr(B2), int(sbk2), int(sbn2), int(N if n1 is None else n1)
    d.C, d.ldc, d.accumulate = addr(C), int(ldc), int(bool(accumulate))
    d.bias = addr(bias)
    d.rowbias, d.ldrb, d.rdiv = addr(rowbias), int(ldrb), int(rdiv)
    d.relu_out = int(bool(relu_out))
    d.gate, d.ldgate = addr(gate), int(ldgate)
    d.R, d.ldR, d.R_ncols = addr(R), int(ldR), int(N if R_ncols is None else R_ncols)
    d.kind = KIND_GEMM
    return d


def colsum_desc(g, out, accumulate=False):
    """out [N] (+)= column sums of g [M, N] (a bias gradient), as a job of a batched launch."""
    ga, gs = _mat(g)
    M, N = g.shape
    d = node_gemm_desc(M, N, 0, ga, gs, 1, ga, 0, 0, out, 0, accumulate=accumulate)
    d.kind = KIND_COLSUM
    return d


def launch(*descs):
    """Run independent node GEMMs (up to 4 per launch) on the current stream."""
    stream = _lib.current_stream()
    for i in range(0, len(descs), MAX_JOBS):
        part = descs[i:i + MAX_JOBS]
        arr = (ctypes.POINTER(NodeGemmDesc) * len(part))(*[ctypes.pointer(d) for d in part])
        _lib.call("ured_node_gemm_batch", arr, len(part), stream)


def node_gemm(*args, **kw):
    launch(node_gemm_desc(*args, **kw))


def linear_desc(x, W, C, *, bias=None, R=None, accumulate=False, relu_out=False, rowbias=None, rdiv=1, gate=None):
    """C [M, N] (+)= x [M, K] W[N, K]^T (+ bias, rowbias[m // rdiv], relu, gate, R); x and W may
    be column slices (unit column stride)."""
    xa, xs = _mat(x)
    wa, ws = _mat(W)
    ca, cs = _mat(C)
    M, Kd = x.shape
    N = W.shape[0]
    return node_gemm_desc(M, N, Kd, xa, xs, 1, wa, 1, ws, ca, cs, accumulate=accumulate, bias=bias,
                          rowbias=rowbias, ldrb=0 if rowbias is None else rowbias.stride(0), rdiv=rdiv,
                          relu_out=relu_out, gate=gate, ldgate=0 if gate is None else gate.stride(0), R=R,
                          ldR=0 if R is None else R.stride(0))


def linear(x, W, C, **kw):
    launch(linear_desc(x, W, C, **kw))


def dgrad_desc(g, W, C, *, R=None, R_ncols=None, accumulate=False, gate=None):
    """C [M, K] (+)= g [M, N] W [N, K] (+ R on the first R_ncols columns), optionally masked by
    gate > 0."""
    ga, gs = _mat(g)
    wa, ws = _mat(W)
    ca, cs = _mat(C)
    M, N = g.shape
    Kd = W.shape[1]
    return node_gemm_desc(M, Kd, N, ga, gs, 1, wa, ws, 1, ca, cs, accumulate=accumulate, R=R,
                          ldR=0 if R is None else R.stride(0), R_ncols=R_ncols, gate=gate,
                          ldgate=0 if gate is None else gate.stride(0))


def dgrad(g, W, C, **kw):
    launch(dgrad_desc(g, W, C, **kw))


def wgrad_desc(g, x, C, accumulate=False, x2=None):
    """C [N, K] (+)= g [M, N]^T x [M, K] (the weight gradient of linear()); with x2, the input
    is cat([x, x2], -1) read in place."""
    ga, gs = _mat(g)
    xa, xs = _mat(x)
    ca, cs = _mat(C)
    M, N = g.shape
    Kd = x.shape[1]
    kw = {}
    if x2 is not None:
        x2a, x2s = _mat(x2)
        kw = dict(B2=x2a, sbk2=x2s, sbn2=1, n1=Kd)
        Kd += x2.shape[1]
    return node_gemm_desc(N, Kd, M, ga, 1, gs, xa, xs, 1, ca, cs, accumulate=accumulate, **kw)


def wgrad(g, x, C, **kw):
    launch(wgrad_desc(g, x, C, **kw))


def colsum(g):
    return K.colsum(g.contiguous())


def _sets(off):
    off = [int(o) for o in off]
    if not 2 <= len(off) <= MAX_SETS + 1:
        raise ValueError("node BN: 1 to 4 node sets")
    arr = (_I * (MAX_SETS + 1))(*(off + [off[-1]] * (MAX_SETS + 1 - len(off))))
    return len(off) - 1, arr


def bn_fwd(Y, bnm, off, training, relu_in=True):
    """BatchNorm1d `bnm` applied to relu(Y) per node set -> (act, mean [S, N], invstd [S, N])."""
    R, N = Y.shape
    nsets, arr = _sets(off)
    act = torch.empty_like(Y)
    mean = torch.empty(nsets, N, device=Y.device)
    invstd = torch.empty(nsets, N, device=Y.device)
    d = NodeBNDesc()
    d.N, d.nsets, d.off = N, nsets, arr
    d.Y, d.ldy = Y.data_ptr(), Y.stride(0)
    d.relu_in, d.training = int(relu_in), int(bool(training))
    d.gamma, d.beta = bnm.weight.data_ptr(), bnm.bias.data_ptr()
    d.running_mean, d.running_var = bnm.running_mean.data_ptr(), bnm.running_var.data_ptr()
    nbt = bnm.num_batches_tracked
    d.num_batches_tracked = nbt.data_ptr() if (training and nbt is not None) else None
    d.momentum = bnm.momentum if bnm.momentum is not None else 0.0
    d.eps = bnm.eps
    d.mean, d.invstd = mean.data_ptr(), invstd.data_ptr()
    d.act, d.ld_act = act.data_ptr(), act.stride(0)
    stream = _lib.stream_of(Y)
    if training and syncbn.active():
        # SyncBN: this rank's per-set (count, mean, M2) -> merged over the ranks -> normalise
        local = torch.empty(nsets, 3, N, dtype=torch.float64, device=Y.device)
        d.stats_out = local.data_ptr()
        _lib.call("ured_node_bn_fwd", ctypes.byref(d), stream)
        glob = syncbn.merge_stats(local)
        d.stats_out, d.stats_in = None, glob.data_ptr()
    _lib.call("ured_node_bn_fwd", ctypes.byref(d), stream)
    return act, mean, invstd


def bn_bwd(G, Y, gamma, mean, invstd, off, training, relu_in=True, dgamma=None, dbeta=None, accumulate=False):
    R, N = Y.shape
    nsets, arr = _sets(off)
    dY = torch.empty_like(Y)
    dgamma = torch.empty(N, device=Y.device) if dgamma is None else dgamma
    dbeta = torch.empty(N, device=Y.device) if dbeta is None else dbeta
    d = NodeBNBwdDesc()
    d.N, d.nsets, d.off = N, nsets, arr
    d.G, d.ldg = G.data_ptr(), G.stride(0)
    d.Y, d.ldy = Y.data_ptr(), Y.stride(0)
    d.relu_in, d.training = int(relu_in), int(bool(training))
    d.gamma, d.mean, d.invstd = gamma.data_ptr(), mean.data_ptr(), invstd.data_ptr()
    d.dY, d.lddy = dY.data_ptr(), dY.stride(0)
    d.dgamma, d.dbeta, d.accumulate = dgamma.data_ptr(), dbeta.data_ptr(), int(bool(accumulate))
    stream = _lib.stream_of(Y)
    if training and syncbn.active():
        # SyncBN: the input gradient from the ranks' summed (sum g, sum g*xhat, count)
        local = torch.empty(nsets, 3, N, dtype=torch.float64, device=Y.device)
        d.sums_out = local.data_ptr()
        _lib.call("ured_node_bn_bwd", ctypes.byref(d), stream)
        glob = syncbn.sum_over_ranks(local)
        d.sums_out, d.sums_in = None, glob.data_ptr()
    _lib.call("ured_node_bn_bwd", ctypes.byref(d), stream)
    return dY, dgamma, dbeta


def _w2(conv):
    return conv.weight.view(conv.weight.shape[0], -1)


class NodeLinearFn(Function):
    """y = x W^T + b (+ R). x [M, K] (any row stride, unit column stride), W [N, K]."""

    @staticmethod
    def forward(ctx, x, W, b, R):
        _lib.require_device(x, W)
        M = x.shape[0]
        y = torch.empty(M, W.shape[0], device=x.device)
        linear(x, W, y, bias=b, R=R)
        ctx.save_for_backward(x, W, b)
        ctx.has_b, ctx.has_r = b is not None, R is not None
        return y

    @staticmethod
    def backward(ctx, g):
        x, W, b = ctx.saved_tensors
        g = _rows(g)
        dx = dW = db = None
        jobs = []
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x.shape, device=x.device)
            jobs.append(dgrad_desc(g, W, dx))
        accW = accb = False
        if ctx.needs_input_grad[1]:
            dW, accW = grad_slot(W)
            jobs.append(wgrad_desc(g, x, dW, accumulate=accW))
        if ctx.has_b and ctx.needs_input_grad[2]:
            db, accb = grad_slot(b)
            jobs.append(colsum_desc(g, db, accumulate=accb))
        if jobs:
            launch(*jobs)
        return dx, (None if accW else dW), (None if accb else db), (g if ctx.has_r else None)


def node_linear(x, W, b=None, R=None):
    return NodeLinearFn.apply(x, W, b, R)


def fused_rows(ts):
    """ONE [sum of rows, ...] view over tensors that lie back to back in memory (FlatAdam lays out
    chained parameters that way: an attention's in_proj q/k/v weights and biases), else None."""
    t0 = ts[0]
    if not t0.is_contiguous():
        return None
    if len(ts) == 1:
        return t0.detach()
    end = t0.data_ptr() + t0.numel() * t0.element_size()
    base = t0.untyped_storage().data_ptr()     # one allocation: separate tensors may abut by chance
    for t in ts[1:]:
        if (not t.is_contiguous() or t.shape[1:] != t0.shape[1:] or t.data_ptr() != end or t.dtype != t0.dtype
                or t.untyped_storage().data_ptr() != base):
            return None
        end += t.numel() * t.element_size()
    return t0.detach().as_strided((sum(t.shape[0] for t in ts),) + tuple(t0.shape[1:]), t0.stride())


def _stack_rows(ts):
    f = fused_rows(ts)
    return f if f is not None else torch.cat([t.detach() for t in ts])


def _grad_rows(ts):
    """Gradient storage of row-stacked parameters `ts` for one kernel job:
    (buffer [sum of rows, ...], accumulate, finish) where finish() returns the per-part gradients
    to hand to autograd (None for a part accumulated in place, grad_slot)."""
    slots = [grad_slot(t) for t in ts]
    bufs, accs = [b for b, _ in slots], [a for _, a in slots]
    if all(a == accs[0] for a in accs):
        f = fused_rows(bufs)
        if f is not None:                     # the flat views are adjacent: write them in place
            return f, accs[0], lambda: [None if accs[0] else b for b in bufs]
    buf = torch.empty((sum(t.shape[0] for t in ts),) + tuple(ts[0].shape[1:]), device=ts[0].device)

    def finish():
        out, o = [], 0
        for b, acc, t in zip(bufs, accs, ts):
            part = buf[o:o + t.shape[0]]
            o += t.shape[0]
            if b._base is None:               # a fresh tensor (no flat slot): hand over the slice
                out.append(part)
            else:                             # a claimed flat view must receive the gradient
                (b.add_ if acc else b.copy_)(part)
                out.append(None if acc else b)
        return out
    return buf, False, finish


class NodeProjFn(Function):
    """Row-stacked projections of node sets: for input i, y_i = x_i W_i^T + b_i where W_i / b_i
    stack the weights / biases of group i along rows — the q|k|v projections of a self-attention
    (one input), the q and the k|v projections of a cross-attention (two inputs). When FlatAdam
    has laid the chained parameters out back to back (MultiheadAttention declares the chain) the
    stack is the parameters' own memory: no concatenation forward, and the weight / bias
    gradients are written (or, for a second use of the layer, accumulated) straight into the flat
    gradient. All GEMMs of one direction run in one launch.

    apply(groups, aliases, x_0, .., x_{n-1}, then per input: its weights, then its biases).
    aliases[i]: also return x_i itself (after the projections) for a second consumer of the node
    features (DeformNet's FFN reads the query nodes, the next call the key / value nodes); its
    gradient then arrives in this backward and is added inside the dgrad's epilogue (R) instead of
    in a separate autograd add (the pattern of ops.PartRowsFn's alias output)."""

    @staticmethod
    def forward(ctx, groups, aliases, *tensors):
        n = len(groups)
        xs, rest = tensors[:n], tensors[n:]
        _lib.require_device(*xs)
        Ws, bs, o = [], [], 0
        for gsz in groups:
            Ws.append(rest[o:o + gsz])
            bs.append(rest[o + gsz:o + 2 * gsz])
            o += 2 * gsz
        ys, jobs = [], []
        for x, w, b in zip(xs, Ws, bs):
            Wf, bf = _stack_rows(w), _stack_rows(b)
            y = torch.empty(x.shape[0], Wf.shape[0], device=x.device)
            jobs.append(linear_desc(x, Wf, y, bias=bf))
            ys.append(y)
        launch(*jobs)
        ctx.groups, ctx.aliases = groups, aliases
        ctx.save_for_backward(*xs, *rest)
        outs = tuple(ys) + tuple(x for x, a in zip(xs, aliases) if a)
        return outs if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, *gs):
        groups, aliases = ctx.groups, ctx.aliases
        n = len(groups)
        saved = ctx.saved_tensors
        xs, rest = saved[:n], saved[n:]
        galias, q = [None] * n, n
        for i, a in enumerate(aliases):
            if a:
                galias[i] = gs[q]
                q += 1
        jobs, dxs, fins, o = [], [], [], 0
        for i, gsz in enumerate(groups):
            w, b = rest[o:o + gsz], rest[o + gsz:o + 2 * gsz]
            o += 2 * gsz
            g = _rows(gs[i])
            x = xs[i]
            dx = torch.empty(x.shape, device=x.device)
            R = None if galias[i] is None else _rows(galias[i])
            dW, aW, fW = _grad_rows(w)
            db, ab, fb = _grad_rows(b)
            jobs += [dgrad_desc(g, _stack_rows(w), dx, R=R), wgrad_desc(g, x, dW, accumulate=aW),
                     colsum_desc(g, db, accumulate=ab)]
            dxs.append(dx)
            fins.append((fW, fb))
        launch(*jobs)
        out = [None, None] + dxs
        for fW, fb in fins:
            out += fW() + fb()
        return tuple(out)


def node_proj(xs, groups_w, groups_b, aliases=None):
    """NodeProjFn over inputs xs with weight groups groups_w[i] (tuples of [N_j, K] tensors) and
    bias groups groups_b[i]; aliases[i] (optional): also return xs[i] (see NodeProjFn)."""
    args = list(xs)
    for w, b in zip(groups_w, groups_b):
        args += list(w) + list(b)
    aliases = tuple(bool(a) for a in aliases) if aliases is not None else (False,) * len(xs)
    return NodeProjFn.apply(tuple(len(w) for w in groups_w), aliases, *args)


class NodeFFNFn(Function):
    """out = R + conv2(bn(relu(conv1(cat([x, msg], -1))))) over node rows; `off` delimits the
    node sets that are separate calls of the BatchNorm (statistics per set, running stats
    updated per set in order). Inputs: x, msg [M, C]; R [M, C] the residual (None: x itself,
    whose two gradient paths are then summed inside the dgrad epilogue); W1 [2C', 2C], b1,
    W2 [C, 2C'], b2; bn module via spec."""

    @staticmethod
    def forward(ctx, spec, x, msg, R, W1, b1, gamma, beta, W2, b2):
        bnm, off, training = spec[:3]
        ctx.res_is_x = R is None
        R = x if R is None else R
        M, C = x.shape
        N1 = W1.shape[0]
        dev = x.device
        Y1 = torch.empty(M, N1, device=dev)
        xa, xs = _mat(x)
        ma, ms = _mat(msg)
        node_gemm(M, N1, 2 * C, xa, xs, 1, W1.data_ptr(), 1, W1.stride(0), Y1, N1, A2=ma, sam2=ms, sak2=1, k1=C,
                  bias=b1)
        act, mean, invstd = bn_fwd(Y1, bnm, off, training)
        out = torch.empty(M, W2.shape[0], device=dev)
        linear(act, W2, out, bias=b2, R=R)
        ctx.spec = spec
        ctx.save_for_backward(x, msg, W1, gamma, W2, Y1, act, mean, invstd, b1, beta, b2)
        return out

    @staticmethod
    def backward(ctx, g):
        bnm, off, training = ctx.spec[:3]
        x, msg, W1, gamma, W2, Y1, act, mean, invstd, b1, beta, b2 = ctx.saved_tensors
        g = _rows(g)
        M, C = x.shape
        dev = x.device
        dact = torch.empty(act.shape, device=dev)
        (dW2, aW2), (db2, ab2) = grad_slot(W2), grad_slot(b2)
        launch(dgrad_desc(g, W2, dact), wgrad_desc(g, act, dW2, accumulate=aW2), colsum_desc(g, db2, accumulate=ab2))
        (dgamma, ag), (dbeta, abe) = grad_slot(gamma), grad_slot(beta)
        if ag == abe:
            dY1, dgamma, dbeta = bn_bwd(dact, Y1, gamma, mean, invstd, off, training, dgamma=dgamma, dbeta=dbeta,
                                        accumulate=ag)
        else:                  # the BN kernel accumulates both or neither: settle each one after it
            dY1, tg, tb = bn_bwd(dact, Y1, gamma, mean, invstd, off, training)
            for buf, acc, tmp in ((dgamma, ag, tg), (dbeta, abe, tb)):
                (buf.add_ if acc else buf.copy_)(tmp)
        (dW1, aW1), (db1, ab1) = grad_slot(W1), grad_slot(b1)
        R = g if ctx.res_is_x else None
        dxm = torch.empty(M, 2 * C, device=dev)               # [d first | d message] in one GEMM
        launch(wgrad_desc(dY1, x, dW1, accumulate=aW1, x2=msg),
               dgrad_desc(dY1, W1, dxm, R=R, R_ncols=C), colsum_desc(dY1, db1, accumulate=ab1))
        dx, dmsg = dxm[:, :C], dxm[:, C:]
        return (None, dx, dmsg, (None if ctx.res_is_x else g),
                *(None if acc else t for t, acc in ((dW1, aW1), (db1, ab1), (dgamma, ag), (dbeta, abe), (dW2, aW2),
                                                    (db2, ab2))))


def node_ffn(fc, x, msg, R, off):
    """FeedForwardNet_norm([2C, 2C, C], use_bn) `fc` on cat([x, msg]) + R (None: + x), node
    sets `off`."""
    conv1, bnm, conv2 = fc[0], fc[2], fc[3]
    spec = (bnm, tuple(int(o) for o in off), bnm.training)
    return NodeFFNFn.apply(spec, x, msg, R, _w2(conv1), conv1.bias, bnm.weight, bnm.bias, _w2(conv2), conv2.bias)


class ParamDecoderFn(Function):
    """param_decoder on cat([glob [B, 2C] broadcast to P parts, parts [B*P, C]]):
    h = relu(parts W1p^T + (glob W1g^T)[b] + b1), out = h W2^T + b2 -> [B*P, 6]."""

    @staticmethod
    def forward(ctx, P, glob, parts, W1, b1, W2, b2):
        B, Cg = glob.shape
        BP, C = parts.shape
        dev = parts.device
        N1 = W1.shape[0]
        rb = torch.empty(B, N1, device=dev)
        linear(glob, W1[:, :Cg], rb)
        h = torch.empty(BP, N1, device=dev)
        linear(parts, W1[:, Cg:], h, bias=b1, rowbias=rb, rdiv=P, relu_out=True)
        out = torch.empty(BP, W2.shape[0], device=dev)
        linear(h, W2, out, bias=b2)
        ctx.P = P
        ctx.save_for_backward(glob, parts, W1, W2, h, b1, b2)
        return out

    @staticmethod
    def backward(ctx, g):
        glob, parts, W1, W2, h, b1, b2 = ctx.saved_tensors
        P = ctx.P
        B, Cg = glob.shape
        g = _rows(g)
        dev = g.device
        dW2 = grad_buffer(W2)
        db2 = grad_buffer(b2)
        dh = torch.empty(h.shape, device=dev)
        launch(wgrad_desc(g, h, dW2), dgrad_desc(g, W2, dh, gate=h), colsum_desc(g, db2))   # dh through the ReLU
        S = K.group_colsum(dh, dh.shape[1], B, group_rows=P)  # per-sample sums of the broadcast half
        dW1 = grad_buffer(W1)
        db1 = grad_buffer(b1)
        dparts = torch.empty(parts.shape, device=dev)
        dglob = torch.empty(glob.shape, device=dev)
        launch(wgrad_desc(S, glob, dW1[:, :Cg]), wgrad_desc(dh, parts, dW1[:, Cg:]),
               dgrad_desc(dh, W1[:, Cg:], dparts), dgrad_desc(S, W1[:, :Cg], dglob), colsum_desc(dh, db1))
        return None, dglob, dparts, dW1, db1, dW2, db2


def param_decoder(dec, glob, parts, P):
    c1, c2 = dec[0], dec[2]
    return ParamDecoderFn.apply(P, glob, parts, _w2(c1), c1.bias, _w2(c2), c2.bias)
