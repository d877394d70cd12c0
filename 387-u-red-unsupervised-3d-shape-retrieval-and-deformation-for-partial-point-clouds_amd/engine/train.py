"""Drop-in for the reference engine/train.py: U-RED training on the MI355X hot path.

  python engine/train.py [config.json]          (the reference ignores argv and
                                                  hard-codes config/config_train_test.json,
                                                  engine/train.py:362-364; argv is honoured here)
  torchrun --nproc-per-node N engine/train.py [config.json]
                                                 data-parallel: one process per GPU, bs per GPU,
                                                 gradients all-reduced over RCCL during backward
                                                 (engine/dp.py); rank 0 logs and saves

One iteration (engine/train.py:196-345) = source/target encoders, part pooling,
three residual nets, DeformNet, get_shape, the chamfer / contrast / symmetry /
residual / reconstruction losses, backward, per-module clip_grad_norm_(5.0) and
Adam. Differences that do not change results:
  * the per-sample / per-part Python loops (get_part, compute_cm_loss,
    residual_retrieval_loss) are device-side ragged ops — no host syncs;
  * the concatenated residual-net inputs are never materialised (row-bias form);
  * the embedding layer's gradient is not computed: the reference excludes it from
    the optimizer (train_utils/optimizer_dm.py:83) and never reads it;
  * per-step scalar logging (which forces .item() host syncs) is optional (cfg["log_every"]).
Data: cfg["synthetic"] (default) generates SURVEY §8(d) targets; the source labels come from
the reference's pseudo-label selection (get_labels, dataset/dataset_utils.py:1101-1143) over a
target-part x source calc_dcd table computed once on the GPU and the sources_connect matrix
(PseudoLabelLoader; cfg["pseudo_labels"]: false draws them uniformly instead). The reference's
on-disk PartNet h5 readers are out of scope (h5py is not in this image).
"""
import datetime
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
if os.path.dirname(_HERE) not in sys.path:
    sys.path.insert(0, os.path.dirname(_HERE))

from dataset import synthetic  # noqa: E402
from engine.config import check_config  # noqa: E402
from dataset.dataset_utils import (get_shape, get_shape_src, get_source_info, get_source_points,  # noqa: E402
                                   get_symmetric)
from loss.basic_consistency_loss import compute_pc_consistency, compute_pc_consistency_weighted  # noqa: E402
from loss.basic_loss import residual_retrieval_loss  # noqa: E402
from loss.chamfer_loss import compute_cm_loss, compute_cm_loss_pair  # noqa: E402
from loss.contrast_loss import compute_contrast_loss_loss  # noqa: E402
from loss.regularization_loss import regularization_param  # noqa: E402
from network.deformation_net import DeformNet_MatchingNet as DM_decoder  # noqa: E402
from network.deformation_net import re_residual_net  # noqa: E402
from network.simple_encoder import TargetEncoder as simple_encoder  # noqa: E402
from train_utils.load_sources import load_sources  # noqa: E402
from train_utils.optimizer_dm import define_optimizer_dm_re_recon  # noqa: E402
from ured_hip.kernels import RowWeights  # noqa: E402
from ured_hip.ops import PartBounds, UniqueRows, build_parts, part_aabb, part_rows, upload  # noqa: E402

_SHAPE_SRC = os.environ.get("URED_SHAPE_SRC", "1") == "1"     # A/B knob (tools/gpu_py_ab.sh)

MODULE_NAMES = ("target_encoder_full", "param_decoder_full", "recon_decoder_full", "re_residual_net_full",
                "src_encoder_all", "recon_decoder_src", "embedding_layer")
CLIPPED = ("target_encoder_full", "param_decoder_full", "re_residual_net_full", "recon_decoder_full",
           "recon_decoder_src", "src_encoder_all")           # engine/train.py:339-344 order


def get_models(cfg, device=None):
    """engine/train.py:39-101: the seven modules (+ checkpoint init), Adam and StepLR."""
    device = device or cfg["device"]
    m = {
        "src_encoder_all": simple_encoder(cfg["source_latent_dim"], is_src=True, sem_size=cfg["sem_latent_dim"]),
        "recon_decoder_src": re_residual_net(cfg["source_latent_dim"] * 2),
        "target_encoder_full": simple_encoder(cfg["target_latent_dim"], sem_size=cfg["sem_latent_dim"]),
        "recon_decoder_full": re_residual_net(cfg["target_latent_dim"] * 2),
        "param_decoder_full": DM_decoder(cfg["source_latent_dim"] * 3, graph_dim=cfg["source_latent_dim"],
                                         max_num_parts=cfg["MAX_NUM_PARTS"], matching=False),
        "embedding_layer": nn.Embedding(42, cfg["sem_latent_dim"]),
        "re_residual_net_full": re_residual_net(cfg["target_latent_dim"] * 2),
    }
    if cfg.get("init_dm"):
        sd = torch.load(cfg["dm_model_path"], map_location="cpu", weights_only=True)
        for k in ("target_encoder_full", "param_decoder_full", "recon_decoder_full", "src_encoder_all",
                  "recon_decoder_src", "embedding_layer"):
            m[k].load_state_dict(sd[k])
    if cfg.get("init_re"):
        sd = torch.load(cfg["re_model_path"], map_location="cpu", weights_only=True)
        m["re_residual_net_full"].load_state_dict(sd["re_residual_net_full"])
    for v in m.values():
        v.to(device, dtype=torch.float).train()
    opt, sched = define_optimizer_dm_re_recon(m["target_encoder_full"], m["param_decoder_full"],
                                              m["recon_decoder_full"], m["re_residual_net_full"],
                                              m["src_encoder_all"], m["recon_decoder_src"],
                                              m["embedding_layer"], cfg)
    return m, opt, sched


class ReInput:
    """Lazy re_input_codes_full: cat(per-point features sorted by part, part mean) (engine/train.py:125)."""

    def __init__(self, pp_sorted, part_mean, gid, off):
        self.pp_sorted, self.part_mean, self.gid, self.off = pp_sorted, part_mean, gid, off


def get_part(cfg, per_point_full, target_labels, x, alias=False):
    """engine/train.py:103-136 without host syncs. per_point_full [B, N, C].

    Returns (target_part_f [B,P,C], None (the unused per-part feature lists), ReInput,
    mask_part [B,P], PartBatch (the part_x lists), param_def [B,P,6]); alias=True appends
    per_point_full as an output of the regrouping (ured_hip.ops.PartRowsFn) for another consumer,
    whose gradient is then added inside the regrouping's backward pass.
    """
    B, N, C = per_point_full.shape
    P = cfg["MAX_NUM_PARTS"]
    parts = build_parts(target_labels, x, P)
    pp_sorted, sums, *pp_alias = part_rows(per_point_full, parts, alias=alias)
    part_mean = sums / parts.counts.reshape(-1, 1).clamp(min=1).float()
    param_def = getattr(parts, "param_def", None)                      # indexed by label value (train.py:120)
    if param_def is None:
        aabb = part_aabb(parts)                                        # by part slot (rank)
        param_def = torch.gather(aabb, 1, parts.rank_of_label.clamp(min=0).unsqueeze(-1).expand(-1, -1, 6))
        param_def = param_def * parts.present.unsqueeze(-1).float()
    return (part_mean.view(B, P, C), None, ReInput(pp_sorted, part_mean, parts.gid, parts.off),
            parts.mask, parts, param_def) + tuple(pp_alias)


class TrainStep:
    """One U-RED iteration on device-resident inputs (no host sync unless logging)."""

    def __init__(self, cfg, db, device=None):
        self.cfg = cfg
        self.db = db
        self.models, self.optimizer, self.scheduler = get_models(cfg, device)
        self.np_per_part = db.points.shape[1]
        dev = torch.device(device or cfg["device"])
        self._zflip = torch.tensor([1.0, 1.0, -1.0], device=dev)
        # the fused HIP loss head (ured_hip/losshead.py); False: the composed torch + NN-launch form
        self.loss_head = dev.type == "cuda" and cfg.get("loss_head", True)
        self.force_gather = False    # engine/dp.py: gather the contrastive codes even at world size 1
        # optional SyncBN (ured_hip/syncbn.py): global-batch BN statistics over the ranks
        import torch.distributed as dist
        self.sync_bn = bool(cfg.get("sync_bn", False)) and dist.is_initialized() and dist.get_world_size() > 1
        if self.sync_bn:
            if dev.type != "cuda":
                raise NotImplementedError("sync_bn: the HIP BatchNorm path only (a CUDA device)")
        if dev.type == "cuda":       # process-wide: the last step constructed decides
            from ured_hip import syncbn
            if self.sync_bn:
                syncbn.enable()
            else:
                syncbn.disable()

    def _source_branch(self, uq, src_points, src_sem_f, B, P, expand_rec=True):
        """src_encoder_all + recon_decoder_src (engine/train.py:210-216) -> codes [B*P, C],
        recon_src_p [B, P, NP, 3] — or, with expand_rec=False, (codes, recon per encoded part
        [U, NP, 3], that part's points [U, NP, 3], slot -> part index [B*P]) for the loss head."""
        M = self.models
        if uq is not None:
            # unique source encoding: the slots' inputs are functions of their source part
            # only, so the encoder and recon_decoder_src run once per distinct part with row
            # multiplicities (BN statistics / backward of the full batch), then expand
            rw = RowWeights(uq.w, self.np_per_part)
            with torch.no_grad():
                sem_u = M["embedding_layer"](self.db.sem[uq.uniq])
            pts_u = self.db.points[uq.uniq]
            code_u, pp_u = M["src_encoder_all"].forward_pointmajor(pts_u.unsqueeze(0), sem_u.unsqueeze(0), rw=rw)
            rec_u = M["recon_decoder_src"].forward_split(pp_u, code_u, code_first=True,
                                                         group_rows=self.np_per_part, rw=rw)
            if not expand_rec:
                return uq.expand(code_u), rec_u.view(uq.U, -1, 3), pts_u, uq.inverse
            return uq.expand(code_u), uq.expand(rec_u.view(uq.U, -1)).view(B, P, -1, 3)
        codes, src_pp = M["src_encoder_all"].forward_pointmajor(src_points, src_sem_f)
        recon_src_p = M["recon_decoder_src"].forward_split(src_pp, codes, code_first=True,
                                                           group_rows=self.np_per_part).view(B, P, -1, 3)
        if not expand_rec:
            return (codes, recon_src_p.view(B * P, -1, 3), src_points.reshape(B * P, -1, 3),
                    self._arange(B * P, codes.device))
        return codes, recon_src_p

    def _arange(self, n, dev):
        a = getattr(self, "_ar", None)
        if a is None or a.shape[0] != n:
            a = self._ar = torch.arange(n, device=dev)
        return a

    def _deform_losses(self, T, tcode, codes, mats, param_def, x, part_x, mask_part, target_part_f, src_labels):
        """param_decoder_full -> get_shape -> chamfer (full, part), contrast and symmetry terms
        (engine/train.py:253-302) -> (their weighted sum, out, params, the x -> out NN indices of
        the chamfer full family or None)."""
        cfg, M = self.cfg, self.models
        B = x.shape[0]
        params_full = M["param_decoder_full"](tcode, codes, None)
        out = get_shape(mats, params_full, param_def, cfg["alpha"]).reshape(B, -1, 3)
        contrast_labels = torch.where(src_labels >= 0, torch.ones_like(src_labels), src_labels)
        loss = out.new_zeros(())
        if cfg.get("use_param_loss", 0.0) > 0.0:     # engine/train.py:281-283 (first term, as there)
            T["param_loss"] = regularization_param(params_full, mask_part)
            loss = loss + T["param_loss"] * cfg["use_param_loss"]
        pair = cfg["use_chamfer_loss"] > 0.0 and cfg["use_symmetry_loss"] > 0.0
        knn_idx = None
        if pair:        # both chamfer families of out and of its mirror image in one launch each
            (T["cd_loss_full"], T["cd_loss_part"]), (T["ref_cd_loss_full"], T["ref_cd_loss_part"]), knn_idx = \
                compute_cm_loss_pair(out, get_symmetric(out), x, part_x, mask_part, np_per_part=self.np_per_part,
                                     return_idx=True)
        if cfg["use_chamfer_loss"] > 0.0:
            if not pair:
                T["cd_loss_full"], T["cd_loss_part"] = compute_cm_loss(out, x, part_x, mask_part,
                                                                       np_per_part=self.np_per_part)
            loss = loss + T["cd_loss_full"] * cfg["use_chamfer_loss"] + T["cd_loss_part"] * cfg["use_chamfer_part_loss"]
        if cfg["use_contrast_loss"] > 0.0:
            T["contrast_loss"] = compute_contrast_loss_loss(target_part_f, codes, contrast_labels,
                                                            cfg.get("differentiable_gather", False),
                                                            self.force_gather)
            loss = loss + T["contrast_loss"] * cfg["use_contrast_loss"]
        if cfg["use_symmetry_loss"] > 0.0:
            if not pair:
                T["ref_cd_loss_full"], T["ref_cd_loss_part"] = compute_cm_loss(get_symmetric(out), x, part_x,
                                                                               mask_part, np_per_part=self.np_per_part)
            loss = loss + T["ref_cd_loss_full"] * cfg["use_symmetry_loss"]
        return loss, out, params_full, knn_idx

    def forward(self, batch, epoch=0):
        if self.loss_head:
            return self._forward_head(batch, epoch)
        return self._forward_composed(batch, epoch)

    def _forward_head(self, batch, epoch=0):
        """The step with the loss head as one HIP autograd Function (ured_hip/losshead.py): the
        chamfer, contrastive, residual and reconstruction losses and their weighted sum in ~10
        launches forward and ~7 backward (the composed form, _forward_composed, is the same
        arithmetic as ~150 small torch kernels)."""
        from loss.contrast_loss import gathers
        from ured_hip.losshead import HeadInputs, loss_head
        cfg, M = self.cfg, self.models
        P = cfg["MAX_NUM_PARTS"]
        x = batch["x"]
        if cfg.get("complementme", False):      # engine/train.py:192-194 (out of place, see _forward_composed)
            x = x * self._zflip
        B, N, _ = x.shape
        src_labels = batch["src_labels"]
        uq = batch.get("src_unique") if cfg.get("unique_sources", True) else None
        # the unique-source path embeds the distinct parts' semantics itself (_source_branch); the
        # source matrices are read in place by get_shape_src
        mats, _, src_sem_idx = get_source_info(src_labels, self.db, want=(not _SHAPE_SRC, False, uq is None))
        emb = M["embedding_layer"]
        with torch.no_grad():          # the embedding is not trained (optimizer_dm.py:83)
            src_sem_f = emb(src_sem_idx) if uq is None else None
            tgt_sem_f = emb(batch["tgt_sem"])
        # every slot's points only when every slot is encoded (the unique path reads the distinct parts)
        src_points = get_source_points(src_labels, self.db) if uq is None else None
        codes, rec_u, pts_u, inv = self._source_branch(uq, src_points, src_sem_f, B, P, expand_rec=False)
        tcode, pp = M["target_encoder_full"].forward_pointmajor(x, tgt_sem_f)
        # the per-point features feed get_part's regrouping and the reconstruction decoder: the
        # decoder reads them through the regrouping's alias output, so their two gradients are
        # summed in the regrouping's backward pass
        target_part_f, _, re_in, mask_part, parts, param_def, pp_alias = get_part(cfg, pp.view(B, N, -1),
                                                                                 batch["labels"], x, alias=True)
        codes = codes.view(B, P, -1)
        params_full = M["param_decoder_full"](tcode, codes, None)
        out = (get_shape_src(self.db, src_labels, params_full, param_def, cfg["alpha"]) if _SHAPE_SRC else
               get_shape(mats, params_full, param_def, cfg["alpha"])).reshape(B, -1, 3)
        recon_full_p = M["recon_decoder_full"].forward_split(pp_alias.view(B * N, -1), tcode,
                                                             group_rows=N).view(B, N, 3)
        re_res = M["re_residual_net_full"].forward_split(re_in.pp_sorted, re_in.part_mean, gidx=re_in.gid,
                                                         off=re_in.off).view(B, N, 3)
        param = regularization_param(params_full, mask_part) if cfg.get("use_param_loss", 0.0) > 0.0 else None
        contrast_ext = None
        if gathers(self.force_gather) and cfg.get("use_contrast_loss", 0.0) > 0.0:
            # the reference gathers the source codes of every rank (contrast_loss.py:35-58)
            contrast_labels = torch.where(src_labels >= 0, torch.ones_like(src_labels), src_labels)
            contrast_ext = compute_contrast_loss_loss(target_part_f, codes, contrast_labels,
                                                      cfg.get("differentiable_gather", False), self.force_gather)
        hi = HeadInputs(x, parts, self.np_per_part, src_labels, pts_u, inv, cfg,
                        gate=cfg.get("use_residuals_reg", 0.0) > 0.0 and epoch > cfg["init_p_m_loss"],
                        bounds=batch.get("part_bounds"))
        loss, T, _ = loss_head(hi, out, re_res, recon_full_p, rec_u, target_part_f, codes, param, contrast_ext)
        T["all_loss"] = loss
        T["_out"] = out
        T["_params"] = params_full
        return loss, T

    def _forward_composed(self, batch, epoch=0):
        cfg, M = self.cfg, self.models
        P = cfg["MAX_NUM_PARTS"]
        x = batch["x"]
        if cfg.get("complementme", False):
            # engine/train.py:192-194: ComplementMe targets are z-flipped (the reference negates the
            # batch tensor in place; the batch here may be replayed, so the flip is out of place)
            x = x * self._zflip
        B, N, _ = x.shape
        src_labels = batch["src_labels"]
        mats, _, src_sem_idx = get_source_info(src_labels, self.db)
        emb = M["embedding_layer"]
        with torch.no_grad():          # the embedding is not trained (optimizer_dm.py:83)
            src_sem_f = emb(src_sem_idx)
            tgt_sem_f = emb(batch["tgt_sem"])
        src_points = get_source_points(src_labels, self.db)
        uq = batch.get("src_unique") if cfg.get("unique_sources", True) else None
        codes, recon_src_p = self._source_branch(uq, src_points, src_sem_f, B, P)
        tcode, pp = M["target_encoder_full"].forward_pointmajor(x, tgt_sem_f)
        target_part_f, _, re_in, mask_part, part_x, param_def = get_part(cfg, pp.view(B, N, -1), batch["labels"], x)
        codes = codes.view(B, P, -1)
        T = {}
        loss_d, out, params_full, knn_idx = self._deform_losses(T, tcode, codes, mats, param_def, x, part_x,
                                                                mask_part, target_part_f, src_labels)
        recon_full_p = M["recon_decoder_full"].forward_split(pp, tcode, group_rows=N).view(B, N, 3)
        re_res = M["re_residual_net_full"].forward_split(re_in.pp_sorted, re_in.part_mean, gidx=re_in.gid,
                                                         off=re_in.off).view(B, N, 3)
        loss = loss_d
        if cfg["use_residuals_reg"] > 0.0 and epoch > cfg["init_p_m_loss"]:
            # the x -> out NN query of the residual loss is the chamfer full family's second direction
            T["re_reg_loss_full"], T["reg_loss_full"] = residual_retrieval_loss(x, out.detach(), re_res, mask_part,
                                                                                np_per_part=self.np_per_part,
                                                                                nn_idx=knn_idx)
            loss = loss + T["re_reg_loss_full"] * cfg["use_residuals_reg"] + T["reg_loss_full"] * cfg["use_residuals_reg"] * 0.01
        if cfg["use_recon"] > 0.0:
            T["recon_loss_full"] = compute_pc_consistency(recon_full_p, x)
            T["recon_loss_src"] = compute_pc_consistency_weighted(recon_src_p, src_points, mask_part)
            loss = loss + T["recon_loss_full"] * cfg["use_recon"] + T["recon_loss_src"] * cfg["use_recon"]
        T["all_loss"] = loss
        T["_out"] = out
        T["_params"] = params_full
        return loss, T

    def clip_and_step(self, max_norm=5.0):
        """clip_grad_norm_(module.parameters(), 5.0) for each of the six modules
        (engine/train.py:331-336) with the per-tensor norms of all six in one multi-tensor
        launch and the six totals / clip factors as one small vector (deterministic: fixed-order
        row sums, no atomics); then Adam."""
        if hasattr(self.optimizer, "flat_grad"):      # FlatAdam (ured_hip/optim.py): one fused tail
            self.optimizer.step(max_norm=max_norm)
            return
        groups = [[p.grad for p in self.models[name].parameters() if p.grad is not None] for name in CLIPPED]
        grads = [g for grp in groups for g in grp]
        if grads:
            counts = tuple(len(grp) for grp in groups)
            key = (counts, grads[0].device)
            if getattr(self, "_clip_key", None) != key:
                L, n = max(counts), len(grads)
                idx = torch.full((len(counts), L), n, dtype=torch.long)
                o = 0
                for g, c in enumerate(counts):
                    idx[g, :c] = torch.arange(o, o + c)
                    o += c
                self._clip_idx, self._clip_key = idx.to(grads[0].device), key
            norms = torch.stack(torch._foreach_norm(grads, 2.0))
            sq = torch.cat([norms * norms, norms.new_zeros(1)])
            total = sq[self._clip_idx].sum(1).sqrt()                       # [6] module norms
            coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
            for g, grp in enumerate(groups):
                if grp:
                    torch._foreach_mul_(grp, coef[g])
        self.optimizer.step()

    def step(self, batch, epoch=0):
        self.optimizer.zero_grad(set_to_none=True)
        loss, T = self.forward(batch, epoch)
        self.begin_backward()
        self.backward_loss(loss)
        self.reduce_gradients()
        self.clip_and_step()
        return T

    def backward_loss(self, loss):
        """loss.backward() seeded with a persistent 1.0 (no fill kernel per step; a HIP-graph
        capture reads the same tensor)."""
        seed = getattr(self, "_seed", None)
        if seed is None or seed.device != loss.device or seed.dtype != loss.dtype:
            seed = self._seed = torch.ones((), device=loss.device, dtype=loss.dtype)
        loss.backward(seed)

    def begin_backward(self):
        """Data-parallel hook before loss.backward() (engine/dp.py: arms the bucket all-reduce)."""

    def reduce_gradients(self):
        """Data-parallel hook (engine/dp.py overrides); single process: nothing to do."""

    def state_dict(self):
        m = self.models
        return {"target_encoder_full": m["target_encoder_full"].state_dict(),
                "param_decoder_full": m["param_decoder_full"].state_dict(),
                "re_residual_net_full": m["re_residual_net_full"].state_dict(),
                "recon_decoder_full": m["recon_decoder_full"].state_dict(),
                "src_encoder_all": m["src_encoder_all"].state_dict(),
                "recon_decoder_src": m["recon_decoder_src"].state_dict(),
                "embedding_layer": m["embedding_layer"].state_dict()}


def batch_to_device(b, device, num_sources=None, bucket=None):
    """Host batch -> device tensors (pinned-memory staged, asynchronous on the current stream:
    the reference's per-iteration .to(cfg["device"]) copies, engine/train.py:223-232). With num_sources (the source DB size) the distinct source
    parts of the batch are also computed here, on the host labels (UniqueRows; used by
    TrainStep unless cfg["unique_sources"] is False); `bucket` pads their count for HIP-graph
    replay (engine/graph.py keeps one graph per padded count)."""
    out = {k: upload(b[k], device) for k in ("x", "labels", "tgt_sem", "src_labels")}
    out["part_bounds"] = PartBounds(b["labels"])
    if num_sources is not None:
        out["src_unique"] = UniqueRows(b["src_labels"], num_sources, device, bucket=bucket)
    return out


def loader_batching(cfg):
    """(batch size, shuffle) of the training loader: cfg["batch_size"] and a shuffled order in
    "train" mode, else 2 and the dataset order (engine/train.py:160-165,174)."""
    if cfg.get("mode", "train") == "train":
        return int(cfg["batch_size"]), True
    return 2, False


def make_loader(cfg, db, device, seed=0, dist_src=None):
    if cfg.get("pseudo_labels", True) and dist_src is not None and torch.device(device).type == "cuda":
        return PseudoLabelLoader(cfg, db, device, dist_src, seed=seed)
    return SyntheticLoader(cfg, db.num_sources, device, seed=seed)


def resample_parts(x, labels, k, n=1024, seed=0):
    """[k, n, 3] part clouds of one target (each part's points drawn with replacement and
    normalised, like the reference's 1024-point part h5 clouds, generate_pair.py:87-122)."""
    from engine.generate_pair import normalize_pts
    rng = np.random.Generator(np.random.PCG64(seed))
    out = np.zeros((k, n, 3), np.float32)
    for i in range(k):
        pts = x[labels == i]
        out[i] = normalize_pts(pts[rng.integers(0, pts.shape[0], size=n)])
    return out


class PseudoLabelLoader:
    """DataLoader(partnet_dataset) + get_labels (engine/train.py:167-197,
    dataset/dataset_utils.py:1101-1143) on a fixed synthetic target set: cfg["num_targets"]
    targets (cfg["synthetic_targets"]: "sources" (default) assembles each from distinct source
    parts, synthetic.make_targets_from_sources; "ball" uses the SURVEY §8(d) generator), their part
    clouds scored against every source by calc_dcd once on the GPU (PairGenerator.cross: the
    per-part pickle rows of generate_pair.py), and each batch's labels chosen by the reference's
    rule on the device (PseudoLabelTable: top-10 by cd_m, < filter_threshold, semantic preference,
    mask_label over dist_src's cd_m with cl_k) when the batch is drawn, as get_labels runs per
    iteration. The labels come back to the host (the reference's get_labels returns host arrays,
    and the distinct-source tables and the graph key are built from them); the next batch's labels
    are computed on a side stream while the current step runs. Epochs visit the targets in a
    seeded shuffle ("train" mode; loader_batching), drop_last as the reference's DataLoader."""

    def __init__(self, cfg, db, device, dist_src, seed=0):
        from engine.generate_pair import PairGenerator, normalize_pts
        from train_utils.pseudo_labels import PseudoLabelTable
        self.cfg, self.db, self.device, self.seed = cfg, db, device, seed
        P = cfg["MAX_NUM_PARTS"]
        T = int(cfg.get("num_targets", 128))
        self.bs, self.shuffle = loader_batching(cfg)
        if T < self.bs:
            raise ValueError(f"num_targets ({T}) < batch size ({self.bs}): every epoch would be empty "
                             "(the reference's DataLoader drops the last partial batch)")
        kind = cfg.get("synthetic_targets", "sources")
        if kind == "sources":
            t = synthetic.make_targets_from_sources(db.points.cpu().numpy(), db.sem.cpu().numpy(), T,
                                                    cfg.get("num_points", 2048), parts=cfg.get("parts", 4),
                                                    seed=seed * 7777 + 17)
        elif kind == "ball":
            t = synthetic.make_batch(T, cfg.get("num_points", 2048), db.num_sources, max_parts=P,
                                     parts=cfg.get("parts", 4), seed=seed * 7777 + 17)
        else:
            raise ValueError(f"synthetic_targets: 'sources' or 'ball', got {kind!r}")
        self.targets = t
        rows = np.full((T, P), -1, np.int64)
        clouds, part_sem = [], []
        for j in range(T):
            k = int(t["parts"][j])
            clouds.append(resample_parts(t["x"][j], t["labels"][j], k, db.points.shape[1], seed=seed * 131 + j))
            for i in range(k):
                rows[j, i] = len(part_sem)
                part_sem.append(int(t["tgt_sem"][j][t["labels"][j] == i][0]))
        src = np.stack([normalize_pts(p) for p in db.points.cpu().numpy()])
        gen = PairGenerator(torch.from_numpy(src).to(device))
        table = gen.cross(torch.from_numpy(np.concatenate(clouds)))          # [3, parts, NS]
        self.table = PseudoLabelTable(table[2], part_sem, db.sem, np.asarray(dist_src),
                                      alpha=cfg.get("filter_threshold", 2e-2), cl_k=cfg.get("cl_k", 40),
                                      device=device)
        self.part_rows = rows
        self._rows_dev = torch.from_numpy(rows).to(device)
        self._side = torch.cuda.Stream(device=device) if torch.device(device).type == "cuda" else None
        self.n = T // self.bs
        self.epoch = 0
        self.last_sel = None

    def __len__(self):
        return self.n

    def _labels_async(self, sel):
        """get_labels of the targets `sel` on the side stream -> (pinned host tensor, event)."""
        # the table and the row map were produced on the default stream: order the side stream
        # behind it (a no-op wait once they are done)
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            idx = upload(np.asarray(sel, np.int64), self.device)
            lab = self.table.labels(self._rows_dev.index_select(0, idx))
            host = torch.empty(lab.shape, dtype=lab.dtype, pin_memory=True)
            host.copy_(lab, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return host, ev

    def __iter__(self):
        rng = np.random.Generator(np.random.PCG64([self.seed, self.epoch]))
        self.epoch += 1
        T = self.targets["x"].shape[0]
        order = rng.permutation(T) if self.shuffle else np.arange(T)
        sels = [order[i * self.bs:(i + 1) * self.bs] for i in range(self.n)]
        pending = self._labels_async(sels[0]) if sels else None
        for i, sel in enumerate(sels):
            host, ev = pending
            if i + 1 < len(sels):
                pending = self._labels_async(sels[i + 1])       # overlaps this batch's step
            ev.synchronize()
            b = {"x": self.targets["x"][sel], "labels": self.targets["labels"][sel],
                 "tgt_sem": self.targets["tgt_sem"][sel], "src_labels": host.numpy().copy()}
            self.last_sel = sel
            yield batch_to_device(b, self.device, self.db.num_sources,
                                  bucket=8 if self.cfg.get("cuda_graph") else None)


class SyntheticLoader:
    """Stands in for DataLoader(partnet_dataset) + get_labels (engine/train.py:167-197)."""

    def __init__(self, cfg, num_sources, device, seed=0):
        self.cfg, self.ns, self.device, self.seed = cfg, num_sources, device, seed
        self.n = int(cfg.get("iters_per_epoch", 10))

    def __len__(self):
        return self.n

    def __iter__(self):
        for i in range(self.n):
            b = synthetic.make_batch(loader_batching(self.cfg)[0], self.cfg.get("num_points", 2048), self.ns,
                                     max_parts=self.cfg["MAX_NUM_PARTS"], parts=self.cfg.get("parts", 4),
                                     seed=self.seed * 100003 + i)
            yield batch_to_device(b, self.device, self.ns, bucket=8 if self.cfg.get("cuda_graph") else None)


class _ScalarLog:
    def __init__(self, logdir):
        try:
            from tensorboardX import SummaryWriter
            self.w = SummaryWriter(logdir=logdir)
            self.f = None
        except ImportError:
            self.w = None
            os.makedirs(logdir, exist_ok=True)
            self.f = open(os.path.join(logdir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, global_step):
        if self.w is not None:
            self.w.add_scalar(tag, value, global_step=global_step)
        else:
            self.f.write(json.dumps({"tag": tag, "value": value, "step": global_step}) + "\n")


def save_model(model, start, epoch, cfg):
    now = datetime.datetime.now()
    log = "> {} | Epoch [{:04d}/{:04d}] | duration: {:.1f}s |".format(now.strftime("%c"), epoch, cfg["epochs"],
                                                                       (now - start).total_seconds())
    fname = os.path.join(cfg["log_path"], "checkpoint_{:04d}.pth".format(epoch))
    print("> Saving model to {}...".format(fname))
    torch.save(model, fname)
    with open(os.path.join(cfg["log_path"], "train.log"), "a") as fp:
        fp.write(log + "\n")
    print(log)


def init_distributed(cfg):
    """torchrun environment -> (rank, world, device). One process per GPU; RCCL ("nccl") on
    ROCm devices, gloo on CPU; cfg["dist_backend"] overrides the backend (gloo on GPUs: the
    multi-rank tests run every rank on the one GPU of a test box, local rank modulo the device
    count). Single process: (0, 1, cfg["device"])."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, cfg["device"]
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if str(cfg["device"]).startswith("cuda"):
        backend = cfg.get("dist_backend", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", device_id=device)
        else:
            device = torch.device("cuda", local % torch.cuda.device_count())
            torch.cuda.set_device(device)
            dist.init_process_group(backend)
    else:
        device = torch.device(cfg["device"])
        dist.init_process_group(cfg.get("dist_backend", "gloo"))
    return dist.get_rank(), dist.get_world_size(), device


def main(cfg):
    check_config(cfg, "train")
    rank, world, device = init_distributed(cfg)
    db, dist_src = load_sources(cfg, device)
    if world > 1:
        from engine.dp import DataParallelStep
        trainer = DataParallelStep(cfg, db, device)
    else:
        trainer = TrainStep(cfg, db, device)
    if cfg.get("cuda_graph", False) and torch.device(device).type == "cuda":
        # the step replayed as HIP graphs (engine/graph.py); the loaders pad the distinct-source
        # count to a multiple of 8 so that few graphs serve all batches
        from engine.graph import GraphedStep
        trainer = GraphedStep(trainer)
    # each rank draws its own shard of samples (weak scaling: batch_size per GPU)
    loader = make_loader(cfg, db, device, seed=int(cfg.get("seed", 0)) + 7919 * rank, dist_src=dist_src)
    writer = _ScalarLog(cfg["log_path"]) if rank == 0 else None
    log_every = int(cfg.get("log_every", 1))
    for epoch in range(cfg["epochs"]):
        start = datetime.datetime.now()
        if rank == 0:
            print(str(start), "training epoch", str(epoch))
        for i, batch in enumerate(loader):
            T = trainer.step(batch, epoch)
            if writer is not None and log_every and i % log_every == 0:
                for tag, v in T.items():
                    if not tag.startswith("_") and tag != "ref_cd_loss_part":
                        writer.add_scalar(tag, float(v.item()), epoch * len(loader) + i)
        trainer.scheduler.step()
        if rank == 0 and (epoch + 1) % cfg["save_epoch"] == 0:
            save_model(trainer.state_dict(), start, epoch, cfg)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return trainer


if __name__ == "__main__":
    config_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(_HERE), "config",
                                                                       "config_train_test.json")
    config = json.load(open(config_path))
    os.makedirs(config["log_path"], exist_ok=True)
    main(config)
