"""Fused per-point MLP chains on libured_hip.so, as torch autograd Functions.

PointEncoderFn : TargetEncoder.forward (network/simple_encoder.py:88-107) —
                 conv 3->64->64 (mlp1), 64->64->128->1024 (mlp2), fuse_sem
                 (1024+S)->1024, per_point_out 1024->C->C, max-pool + fc —
                 every Conv1d+BatchNorm1d(train)+ReLU fused into ured_gemm
                 launches (prologue = previous BN+ReLU, epilogue = stats / pool).
ResidualNetFn  : re_residual_net.forward (network/deformation_net.py:96-107) with
                 FeedForwardNet_norm [in,256,256,32,3] (Conv->ReLU->BN), whose
                 input is cat(per-point features, per-group code): the group half
                 is folded into a per-group row bias (W_code @ code), so it is
                 never broadcast to every point.
Both run forward and backward entirely on HIP kernels; only the tiny
per-call index bookkeeping is Python.
"""
import torch
from torch.autograd import Function

from . import _lib
from . import kernels as K
from . import node
from .optim import grad_buffer

BN_EPS = 1e-5


class EncoderSpec:
    """Static description of one TargetEncoder call.

    mode "src": x [G*group_rows, 3] with per-group semantics sem [G, S] (row bias)
    mode "tgt": x [M, 3] with per-point semantics sem [M, S] (extra K columns)
    bn_modules: the 7 BatchNorm1d modules (running stats updated in place when training)
    rw: optional K.RowWeights — group g of the call stands for rw.w[g] identical groups of
        the full batch (unique-row training: batch statistics and BN backward are those of
        the expanded batch; the caller expands outputs and sums duplicate gradients)
    record: optional dict; the forward stores the max-pool winners there ("pool_rows": int32
        [G, 1024], the row of the call each pooled channel came from)
    """

    def __init__(self, mode, group_rows, training, bn_modules, momentum=0.1, eps=BN_EPS, rw=None, record=None):
        assert mode in ("src", "tgt")
        self.mode, self.group_rows, self.training = mode, group_rows, training
        self.bn_modules, self.momentum, self.eps = bn_modules, momentum, eps
        self.rw = rw
        self.record = record


def _nbt(bnm):
    """The module's int64 num_batches_tracked (incremented inside the finalize launch)."""
    t = bnm.num_batches_tracked
    if t is None:
        return None
    if t.dtype != torch.int64 or not t.is_cuda or not t.is_contiguous():
        raise TypeError("num_batches_tracked must be a contiguous int64 device tensor")
    return t


def _bn_state(spec, i, Yws, M, N, gamma, beta):
    bnm = spec.bn_modules[i]
    if spec.training:
        mom = bnm.momentum if bnm.momentum is not None else 0.0
        return K.bn_fwd_finalize(Yws, M, N, gamma, beta, spec.eps, mom, bnm.running_mean, bnm.running_var, rw=spec.rw,
                                 num_batches_tracked=_nbt(bnm))
    return K.bn_eval_state(gamma, beta, bnm.running_mean, bnm.running_var, spec.eps)


class PointEncoderFn(Function):
    """params: W1,b1,g1,be1, ..., W7,b7,g7,be7, W8,b8, fcW, fcb  (32 tensors)."""

    @staticmethod
    def forward(ctx, spec, x, sem, *params):
        x = x.contiguous()
        sem = sem.contiguous()
        M = x.shape[0]
        GR = spec.group_rows
        G = M // GR
        dev = x.device
        Ws = [params[4 * i].reshape(params[4 * i].shape[0], -1) for i in range(7)]
        bs = [params[4 * i + 1] for i in range(7)]
        gs = [params[4 * i + 2] for i in range(7)]
        bes = [params[4 * i + 3] for i in range(7)]
        W8, b8, fcW, fcb = params[28].reshape(params[28].shape[0], -1), params[29], params[30], params[31]
        Ys, states = [], []
        h, kin, pro, st = x, 3, K.PRO_NONE, None
        pool_ws = None
        for i in range(7):
            W = Ws[i]
            N = W.shape[0]
            Y = torch.empty(M, N, device=dev)
            sws = torch.empty(K.nblocks(M), 2, N, device=dev)
            kw = {}
            if i == 5:   # fuse_sem: (1024 + S) -> 1024, then max-pool over each group
                if GR % K.BM == 0:   # pooling partials fused into the GEMM epilogue
                    pool_ws = torch.empty(K.nblocks(M), 4, N, device=dev)
                    kw.update(pool_ws=pool_ws)
                kw.update(group_rows=GR)
                S = sem.shape[1]
                if spec.mode == "src":
                    rb = torch.empty(G, N, device=dev)
                    K.gemm(G, N, S, sem, S, W, W.shape[1], rb, N, B_off=kin)
                    kw.update(rowbias=rb, ldr=N)
                    Kdim = kin
                else:
                    kw.update(A2=sem, lda2=S, k1=kin)
                    Kdim = kin + S
            else:
                Kdim = kin
            K.gemm(M, N, Kdim, h, h.shape[1], W, W.shape[1], Y, N, pro_a=pro,
                   pro_s=None if st is None else st.scale, pro_t=None if st is None else st.shift,
                   bias=bs[i], epi=K.EPI_FWD, stat_ws=sws, **kw)
            st = _bn_state(spec, i, sws, M, N, gs[i], bes[i])
            Ys.append(Y)
            states.append(st)
            h, kin, pro = Y, N, K.PRO_ENC
        C = W8.shape[0]
        pp = torch.empty(M, C, device=dev)
        K.gemm(M, C, kin, h, kin, W8, W8.shape[1], pp, C, pro_a=K.PRO_ENC, pro_s=st.scale, pro_t=st.shift, bias=b8)
        if pool_ws is not None:
            pooled, argidx = K.pool_finalize(pool_ws, M, Ws[5].shape[0], GR, states[5].scale, states[5].shift)
        else:
            pooled, argidx = K.pool_rows(Ys[5], GR, states[5].scale, states[5].shift)
        code = torch.empty(G, C, device=dev)
        K.gemm(G, C, pooled.shape[1], pooled, pooled.shape[1], fcW, fcW.shape[1], code, C, bias=fcb)
        ctx.spec = spec
        ctx.states = states
        if spec.record is not None:      # diagnostics / parity tests: the max-pool winners and the
            spec.record["pool_rows"] = argidx        # values they were chosen from (relu(Y*scale+shift))
            spec.record["pool_y"], spec.record["pool_scale"], spec.record["pool_shift"] = \
                Ys[5], states[5].scale, states[5].shift
        ctx.save_for_backward(x, sem, pooled, argidx, *Ys, *params)
        return code, pp

    @staticmethod
    def backward(ctx, dcode, dpp):
        spec, states = ctx.spec, ctx.states
        saved = ctx.saved_tensors
        x, sem, pooled, argidx = saved[:4]
        Ys = list(saved[4:11])
        params = saved[11:]
        M = x.shape[0]
        GR = spec.group_rows
        G = M // GR
        dev = x.device
        Ws = [params[4 * i].reshape(params[4 * i].shape[0], -1) for i in range(7)]
        gs = [params[4 * i + 2] for i in range(7)]
        W8, fcW = params[28].reshape(params[28].shape[0], -1), params[30]
        C = W8.shape[0]
        grads = [None] * 32
        bias = _BiasSums()
        dcode = torch.zeros(G, C, device=dev) if dcode is None else dcode.contiguous()
        dpp = torch.zeros(M, C, device=dev) if dpp is None else dpp.contiguous()
        # fc: code = pooled @ fcW^T + fcb
        NP = pooled.shape[1]
        dpool = torch.empty(G, NP, device=dev)
        K.gemm(G, NP, C, dcode, C, fcW, NP, dpool, NP, b_kmajor=True)
        dfcW, dfcb = grad_buffer(fcW), grad_buffer(params[31])
        K.wgrad(dcode, C, pooled, NP, C, NP, G, dfcW, NP)
        K.colsum(dcode, out=dfcb)
        grads[30], grads[31] = dfcW, dfcb
        # per_point_out.3 (no BN): dW8 = dpp^T @ H7
        dW8, db8 = grad_buffer(params[28]).view(W8.shape), grad_buffer(params[29])
        K.wgrad(dpp, C, Ys[6], Ys[6].shape[1], C, W8.shape[1], M, dW8, W8.shape[1],
                pro=K.PRO_ENC, pro_s=states[6].scale, pro_t=states[6].shift)
        K.colsum(dpp, out=db8)
        grads[28], grads[29] = dW8.view(params[28].shape), db8
        dY, Wn = dpp, W8   # gradient at the output of the layer above, and that layer's weight
        for i in range(6, -1, -1):
            Y, st = Ys[i], states[i]
            N = Y.shape[1]
            Cn = dY.shape[1]
            G_ = torch.empty(M, N, device=dev)
            bws = torch.empty(K.nblocks(M), 2, N, device=dev)
            kw = {}
            if i == 5:
                kw.update(pool_idx=argidx, pool_grad=dpool, pool_group_rows=GR)
            # dH_i = dY_{i+1} @ W_{i+1}[:, :N]; fused ReLU mask + BN-backward partials of layer i
            K.gemm(M, N, Cn, dY, Cn, Wn, Wn.shape[1], G_, N, b_kmajor=True, epi=K.EPI_BNBWD,
                   Yp=Y, ldy=N, bn=st, bwd_res=False, bwd_ws=bws, **kw)
            dgamma, dbeta = grad_buffer(gs[i]), grad_buffer(params[4 * i + 3])
            coefs = K.bn_bwd_finalize(bws, M, N, gs[i], st.invstd, dgamma, dbeta, rw=spec.rw)
            dYi, cs = K.bn_bwd_apply(G_, Y, False, st.mean, coefs, rw=spec.rw)
            W = Ws[i]
            dW, db = grad_buffer(params[4 * i]).view(W.shape), grad_buffer(params[4 * i + 1])
            _enc_layer_wgrad(spec, i, N, M, G, GR, x, sem, Ys, states, dYi, cs, W, dW)
            bias.add(cs, db)
            grads[4 * i] = dW.view(params[4 * i].shape)
            grads[4 * i + 1] = db
            grads[4 * i + 2], grads[4 * i + 3] = dgamma, dbeta
            dY, Wn = dYi, W
        bias.flush()
        return (None, None, None) + tuple(grads)


class _BiasSums:
    """Conv-bias gradients of a chain backward: the column sums of each BN layer's per-128-row
    partials of dY (cs [M/128, N], from the BN-backward apply), collected and issued at the end of
    the backward as column-sum jobs of batched node-GEMM launches (csrc/node.hip, up to 6 per
    launch) instead of one launch per layer. Nothing reads them before the optimizer."""

    def __init__(self):
        self.jobs = []

    def add(self, cs, out):
        self.jobs.append((cs, out))
        return out

    def flush(self):
        if self.jobs:
            node.launch(*[node.colsum_desc(cs, out) for cs, out in self.jobs])
        self.jobs = []


def _enc_layer_wgrad(spec, i, N, M, G, GR, x, sem, Ys, states, dYi, cs, W, dW):
    """Weight gradient of TargetEncoder layer i from its dY."""
    if i == 0:
        K.wgrad(dYi, N, x, 3, N, 3, M, dW, 3)
    else:
        Xp, stp = Ys[i - 1], states[i - 1]
        kin = Xp.shape[1]
        K.wgrad(dYi, N, Xp, kin, N, kin, M, dW, W.shape[1], pro=K.PRO_ENC, pro_s=stp.scale, pro_t=stp.shift)
        if i == 5:   # semantic columns of fuse_sem
            S = sem.shape[1]
            if spec.mode == "src":
                # G-row GEMM on the per-group sums: short work
                K.wgrad(_group_sums(dYi, cs, N, G, GR), N, sem, S, N, S, G, dW, W.shape[1], out_off=kin)
            else:
                K.wgrad(dYi, N, sem, S, N, S, M, dW, W.shape[1], out_off=kin)


def _group_sums(dY, cs, N, G, group_rows):
    """Per-group column sums of dY [G*group_rows, N]. When groups are whole 128-row blocks they
    come from the BN-backward apply's per-block partials cs [M/128, N] (8 MB instead of
    re-reading the 1 GB gradient)."""
    if group_rows % K.BM == 0:
        return K.group_colsum(cs, N, G, group_rows=group_rows // K.BM)
    return K.group_colsum(dY, N, G, group_rows=group_rows)


class ResidualNetFn(Function):
    """re_residual_net on cat(per-point pp [M,Cp], group code [G,Cc]).

    params: W1,b1,g1,be1, W2,b2,g2,be2, W3,b3,g3,be3, W4,b4 (14 tensors).
    code_first: True when the input is cat(code, pp) (recon_decoder_src).
    grouping: gidx int32 [M] (row -> group) + off int32 [G+1], or fixed group_rows.
    rw: optional K.RowWeights (fixed group_rows only), as in EncoderSpec.
    """

    @staticmethod
    def forward(ctx, spec, pp, code, *params):
        code_first, gidx, off, group_rows, training, bn_modules, rw = spec[:7]
        pp = pp.contiguous()
        code = code.contiguous()
        M, Cp = pp.shape
        G, Cc = code.shape
        dev = pp.device
        W1 = params[0].reshape(params[0].shape[0], -1)
        ld1 = W1.shape[1]
        assert ld1 == Cp + Cc
        pp_off, code_off = (Cc, 0) if code_first else (0, Cp)
        N1 = W1.shape[0]
        rb = None
        if Cc > 0:   # the group half of the concatenated input becomes a per-group row bias
            rb = torch.empty(G, N1, device=dev)
            K.gemm(G, N1, Cc, code, Cc, W1, ld1, rb, N1, B_off=code_off)
        Ys, states = [], []
        h, kin, pro, st = pp, Cp, K.PRO_NONE, None
        for i in range(3):
            W = params[4 * i].reshape(params[4 * i].shape[0], -1)
            N = W.shape[0]
            Y = torch.empty(M, N, device=dev)
            sws = torch.empty(K.nblocks(M), 2, N, device=dev)
            kw = {}
            if i == 0:
                kw = dict(B_off=pp_off)
                if rb is not None:
                    kw.update(rowbias=rb, ldr=N1, gidx=gidx, group_rows=group_rows)
            K.gemm(M, N, kin, h, h.shape[1], W, W.shape[1], Y, N, pro_a=pro,
                   pro_s=None if st is None else st.scale, pro_t=None if st is None else st.shift,
                   bias=params[4 * i + 1], epi=K.EPI_FWD, stat_ws=sws, stat_relu=True, **kw)
            bnm = bn_modules[i]
            if training:
                st = K.bn_fwd_finalize(sws, M, N, params[4 * i + 2], params[4 * i + 3], BN_EPS,
                                       bnm.momentum if bnm.momentum is not None else 0.0,
                                       bnm.running_mean, bnm.running_var, rw=rw, num_batches_tracked=_nbt(bnm))
            else:
                st = K.bn_eval_state(params[4 * i + 2], params[4 * i + 3], bnm.running_mean, bnm.running_var, BN_EPS)
            Ys.append(Y)
            states.append(st)
            h, kin, pro = Y, N, K.PRO_RES
        W4 = params[12].reshape(params[12].shape[0], -1)
        out = torch.empty(M, W4.shape[0], device=dev)
        K.gemm(M, W4.shape[0], kin, h, kin, W4, W4.shape[1], out, W4.shape[0], pro_a=K.PRO_RES,
               pro_s=st.scale, pro_t=st.shift, bias=params[13])
        ctx.spec, ctx.states = spec, states
        ctx.save_for_backward(pp, code, *Ys, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        code_first, gidx, off, group_rows, training, bn_modules, rw = ctx.spec[:7]
        states = ctx.states
        saved = ctx.saved_tensors
        pp, code = saved[:2]
        Ys = list(saved[2:5])
        params = saved[5:]
        M, Cp = pp.shape
        G, Cc = code.shape
        dev = pp.device
        grads = [None] * 14
        bias = _BiasSums()
        dout = dout.contiguous()
        W4 = params[12].reshape(params[12].shape[0], -1)
        No = W4.shape[0]
        dW4, db4 = grad_buffer(params[12]).view(W4.shape), grad_buffer(params[13])
        K.wgrad(dout, No, Ys[2], Ys[2].shape[1], No, W4.shape[1], M, dW4, W4.shape[1],
                pro=K.PRO_RES, pro_s=states[2].scale, pro_t=states[2].shift)
        K.colsum(dout, out=db4)
        grads[12], grads[13] = dW4.view(params[12].shape), db4
        dY, Wn = dout, W4
        W1 = params[0].reshape(params[0].shape[0], -1)
        ld1 = W1.shape[1]
        pp_off, code_off = (Cc, 0) if code_first else (0, Cp)
        dcode = torch.zeros(G, Cc, device=dev)
        for i in range(2, -1, -1):
            Y, st = Ys[i], states[i]
            N = Y.shape[1]
            Cn = dY.shape[1]
            G_ = torch.empty(M, N, device=dev)
            bws = torch.empty(K.nblocks(M), 2, N, device=dev)
            K.gemm(M, N, Cn, dY, Cn, Wn, Wn.shape[1], G_, N, b_kmajor=True, epi=K.EPI_BNBWD,
                   Yp=Y, ldy=N, bn=st, bwd_res=True, bwd_ws=bws)
            dgamma, dbeta = grad_buffer(params[4 * i + 2]), grad_buffer(params[4 * i + 3])
            coefs = K.bn_bwd_finalize(bws, M, N, params[4 * i + 2], st.invstd, dgamma, dbeta, rw=rw)
            dYi, cs = K.bn_bwd_apply(G_, Y, True, st.mean, coefs, rw=rw)
            W = params[4 * i].reshape(params[4 * i].shape[0], -1)
            dW, db = grad_buffer(params[4 * i]).view(W.shape), grad_buffer(params[4 * i + 1])
            if i == 0:
                K.wgrad(dYi, N, pp, Cp, N, Cp, M, dW, ld1, out_off=pp_off)
                if Cc > 0:                     # G-row work on the per-group sums: short kernels
                    if off is not None:
                        D = K.group_colsum(dYi, N, G, off=off)
                    else:
                        D = _group_sums(dYi, cs, N, G, group_rows)
                    K.wgrad(D, N, code, Cc, N, Cc, G, dW, ld1, out_off=code_off)
                    # dcode = D @ W1[:, code cols]
                    K.gemm(G, Cc, N, D, N, W1, ld1, dcode, Cc, b_kmajor=True, B_off=code_off)
            else:
                Xp, stp = Ys[i - 1], states[i - 1]
                K.wgrad(dYi, N, Xp, Xp.shape[1], N, Xp.shape[1], M, dW, W.shape[1],
                        pro=K.PRO_RES, pro_s=stp.scale, pro_t=stp.shift)
            bias.add(cs, db)
            grads[4 * i] = dW.view(params[4 * i].shape)
            grads[4 * i + 1] = db
            grads[4 * i + 2], grads[4 * i + 3] = dgamma, dbeta
            dY, Wn = dYi, W
        bias.flush()
        # input gradient dpp = dY1 @ W1[:, pp cols]
        dpp = torch.empty(M, Cp, device=dev)
        K.gemm(M, Cp, W1.shape[0], dY, W1.shape[0], W1, ld1, dpp, Cp, b_kmajor=True, B_off=pp_off)
        return (None, dpp, dcode) + tuple(grads)


class ChainSpec:
    """Static description of one PointChainFn call (a PointNet conv chain).

    acts: per layer K.ACT_ENC (Conv->BN->ReLU) or K.ACT_BN (Conv->BN; last layer only)
    group_rows: points per cloud (the max-pool groups)
    pool: max-pool the last layer's activation over each group -> pooled [G, N_L]
    want_act: also return the last layer's activation materialised [M, N_L]
    bn_modules: the BatchNorm1d modules (running stats updated in place when training)
    """

    def __init__(self, acts, group_rows, training, bn_modules, pool=True, want_act=False):
        assert all(a == K.ACT_ENC for a in acts[:-1]), "inner layers feed a GEMM prologue: Conv->BN->ReLU only"
        self.acts, self.group_rows, self.training = list(acts), int(group_rows), training
        self.bn_modules, self.pool, self.want_act = bn_modules, pool, want_act


class PointChainFn(Function):
    """Conv1d(k=1)+BatchNorm1d(+ReLU) x L on point-major x [M, Cin], then max-pool over groups of
    spec.group_rows points and/or the last activation (PointNet STN3d / STNkd / PointNetEncoder
    conv stacks, network/pointnet/pointnet_utils.py:27-33,62-68,109-127).

    params: W1,b1,g1,be1, ..., WL,bL,gL,beL. Returns (pooled [G, N_L], act [M, N_L]); an output
    not asked for is an empty tensor. Backward: the last layer's gradient (scattered pool
    gradient + act gradient) enters through a K = 0 BN-backward epilogue; every layer below is
    the fused dgrad + BN-backward GEMM of PointEncoderFn; dx = dY1 @ W1.
    """

    @staticmethod
    def forward(ctx, spec, x, *params):
        _lib.require_device(x, *params)
        x = x.contiguous()
        M = x.shape[0]
        GR = spec.group_rows
        L = len(spec.acts)
        dev = x.device
        Ys, states = [], []
        h, pro, st = x, K.PRO_NONE, None
        pool_ws = None
        for i in range(L):
            W = params[4 * i].reshape(params[4 * i].shape[0], -1)
            N = W.shape[0]
            Y = torch.empty(M, N, device=dev)
            sws = torch.empty(K.nblocks(M), 2, N, device=dev)
            kw = {}
            if i == L - 1 and spec.pool and GR % K.BM == 0:
                pool_ws = torch.empty(K.nblocks(M), 4, N, device=dev)
                kw.update(pool_ws=pool_ws, group_rows=GR)
            K.gemm(M, N, W.shape[1], h, h.shape[1], W, W.shape[1], Y, N, pro_a=pro,
                   pro_s=None if st is None else st.scale, pro_t=None if st is None else st.shift,
                   bias=params[4 * i + 1], epi=K.EPI_FWD, stat_ws=sws, **kw)
            spec_i = _LayerBN(spec, i)
            st = _bn_state(spec_i, 0, sws, M, N, params[4 * i + 2], params[4 * i + 3])
            Ys.append(Y)
            states.append(st)
            h, pro = Y, K.PRO_ENC
        relu_last = spec.acts[-1] == K.ACT_ENC
        NL = Ys[-1].shape[1]
        pooled = argidx = None
        if spec.pool:
            if pool_ws is not None:
                pooled, argidx = K.pool_finalize(pool_ws, M, NL, GR, st.scale, st.shift, relu=relu_last)
            else:
                pooled, argidx = K.pool_rows(Ys[-1], GR, st.scale, st.shift, relu=relu_last)
        act = K.bn_act(Ys[-1], st, relu=relu_last) if spec.want_act else None
        ctx.spec, ctx.states = spec, states
        ctx.save_for_backward(x, argidx, *Ys, *params)
        empty = x.new_empty(0)
        out_p = pooled if pooled is not None else empty
        out_a = act if act is not None else x.new_empty(0)
        if pooled is None:
            ctx.mark_non_differentiable(out_p)
        if act is None:
            ctx.mark_non_differentiable(out_a)
        return out_p, out_a

    @staticmethod
    def backward(ctx, dpooled, dact):
        spec, states = ctx.spec, ctx.states
        saved = ctx.saved_tensors
        L = len(spec.acts)
        x, argidx = saved[0], saved[1]
        Ys = list(saved[2:2 + L])
        params = saved[2 + L:]
        M, Cin = x.shape
        GR = spec.group_rows
        dev = x.device
        grads = [None] * (4 * L)
        use_pool = spec.pool and dpooled is not None and dpooled.numel() > 0
        use_act = spec.want_act and dact is not None and dact.numel() > 0
        dY, Wn = None, None
        bias = _BiasSums()
        for i in range(L - 1, -1, -1):
            Y, st = Ys[i], states[i]
            N = Y.shape[1]
            G_ = torch.empty(M, N, device=dev)
            bws = torch.empty(K.nblocks(M), 2, N, device=dev)
            if i == L - 1:
                # no GEMM feeds the last layer: K = 0, the epilogue adds the pooled gradient at
                # the winning rows and the activation's own gradient, masks, and reduces
                kw = {}
                if use_pool:
                    kw.update(pool_idx=argidx, pool_grad=dpooled.contiguous(), pool_group_rows=GR)
                if use_act:
                    dact = dact.contiguous()
                    kw.update(gadd=dact, ldg=N)
                K.gemm(M, N, 0, Y, N, Y, N, G_, N, b_kmajor=True, epi=K.EPI_BNBWD, Yp=Y, ldy=N, bn=st,
                       bwd_res=spec.acts[i], bwd_ws=bws, **kw)
            else:
                Cn = dY.shape[1]
                K.gemm(M, N, Cn, dY, Cn, Wn, Wn.shape[1], G_, N, b_kmajor=True, epi=K.EPI_BNBWD,
                       Yp=Y, ldy=N, bn=st, bwd_res=spec.acts[i], bwd_ws=bws)
            gamma = params[4 * i + 2]
            dgamma, dbeta = grad_buffer(gamma), grad_buffer(params[4 * i + 3])
            coefs = K.bn_bwd_finalize(bws, M, N, gamma, st.invstd, dgamma, dbeta)
            dYi, cs = K.bn_bwd_apply(G_, Y, False, st.mean, coefs)
            W = params[4 * i].reshape(params[4 * i].shape[0], -1)
            dW = grad_buffer(params[4 * i]).view(W.shape)
            if i == 0:
                K.wgrad(dYi, N, x, Cin, N, Cin, M, dW, Cin)
            else:
                Xp, stp = Ys[i - 1], states[i - 1]
                kin = Xp.shape[1]
                K.wgrad(dYi, N, Xp, kin, N, kin, M, dW, kin, pro=K.PRO_ENC, pro_s=stp.scale, pro_t=stp.shift)
            grads[4 * i] = dW.view(params[4 * i].shape)
            grads[4 * i + 1] = bias.add(cs, grad_buffer(params[4 * i + 1]))
            grads[4 * i + 2], grads[4 * i + 3] = dgamma, dbeta
            dY, Wn = dYi, W
        bias.flush()
        dx = None
        if ctx.needs_input_grad[1]:
            dx = torch.empty(M, Cin, device=dev)
            K.gemm(M, Cin, dY.shape[1], dY, dY.shape[1], Wn, Wn.shape[1], dx, Cin, b_kmajor=True)
        return (None, dx) + tuple(grads)


class _LayerBN:
    """Adapter: the BN bookkeeping of layer i of a ChainSpec in _bn_state's form."""
    __slots__ = ("bn_modules", "training", "eps", "rw")

    def __init__(self, spec, i):
        self.bn_modules, self.training, self.eps, self.rw = [spec.bn_modules[i]], spec.training, BN_EPS, None
