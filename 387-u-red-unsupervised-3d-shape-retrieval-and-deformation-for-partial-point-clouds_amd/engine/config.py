"""The reference's JSON config surface (config/config_train_test.json, config_vis_test.json) and
how each key is honoured here. The reference reads a flat dict with no validation
(engine/train.py:363-364); a key it reads that this build does not implement must fail loudly
instead of silently training something else, so check_config() raises on those.

  REFERENCE_READS      keys engine/train.py (+ get_models, optimizer_dm, load_sources, get_labels)
                       or engine/vis.py read; each implemented here with the reference meaning,
                       except the on-disk data keys, which only matter with "synthetic": false
                       (out of scope: no h5py in this image) and are accepted as inert paths
  REFERENCE_UNREAD     keys present in the shipped configs that no engine script reads: inert in
                       the reference too
  EXTRA                this build's own keys, each defaulting to the reference behaviour
Unknown keys are ignored, as the reference ignores them.
"""

REFERENCE_READS = {
    # models / dims (engine/train.py:39-101)
    "source_latent_dim", "target_latent_dim", "sem_latent_dim", "MAX_NUM_PARTS",
    "init_dm", "dm_model_path", "init_re", "re_model_path", "device",
    # optimiser (train_utils/optimizer_dm.py:68-104)
    "optimizer", "learning_rate", "momentum", "weight_decay", "lr_stepsize", "lr_decay",
    # loop, losses (engine/train.py:156-358)
    "batch_size", "epochs", "save_epoch", "log_path", "alpha", "complementme",
    "use_param_loss", "use_chamfer_loss", "use_chamfer_part_loss", "use_contrast_loss",
    "use_symmetry_loss", "use_residuals_reg", "init_p_m_loss", "use_recon",
    # pseudo-labels (dataset/dataset_utils.py:1101-1143)
    "filter_threshold", "cl_k",
    # loader: "mode" != "train" -> batch size 2, dataset order (engine/train.py:160-165,174;
    # engine/train.py loader_batching)
    "mode",
    # data location (partnet_dataset, load_sources): inert with "synthetic": true
    "base_dir", "middle_name", "category", "num_source", "num_workers", "src_connectivity",
    # inference (engine/vis.py)
    "top_k",
}
REFERENCE_UNREAD = {
    "data_dir", "use_connectivity", "action", "input_channels", "random_rot", "pooling", "n_knn",
    "lr_autodecoder", "part_latent_dim", "use_deformed_pc_consistency", "share_src_latent", "clip_vec",
}
EXTRA = {
    "synthetic", "seed", "num_points", "parts", "num_targets", "iters_per_epoch", "pseudo_labels",
    "unique_sources", "flat_adam", "fused_adam", "cuda_graph",
    "log_every", "compute_connectivity", "src_connectivity_plane", "synthetic_targets", "differentiable_gather", "sync_bn", "loss_head", "dist_backend",
    # data parallel (engine/dp.py, engine/graph.py)
    "dp_bucket_mb", "dp_last_bucket_mb", "dp_force_collectives", "graph_inline_collectives",
}

TRAIN_REQUIRED = ("source_latent_dim", "target_latent_dim", "sem_latent_dim", "MAX_NUM_PARTS", "device",
                  "optimizer", "learning_rate", "weight_decay", "lr_stepsize", "lr_decay", "batch_size",
                  "epochs", "save_epoch", "log_path", "alpha", "use_chamfer_loss", "use_chamfer_part_loss",
                  "use_contrast_loss", "use_symmetry_loss", "use_residuals_reg", "init_p_m_loss", "use_recon")


def check_config(cfg, kind="train"):
    """Raise on a reference setting this build cannot honour; returns cfg."""
    if kind == "train":
        missing = [k for k in TRAIN_REQUIRED if k not in cfg]
        if missing:      # the reference would raise KeyError mid-epoch; raise before any work
            raise KeyError(f"config is missing keys the training step reads: {missing}")
        if cfg["optimizer"] not in ("adam", "sgd"):
            # define_optimizer_dm_re_recon returns None for anything else (optimizer_dm.py:101-102)
            raise ValueError(f"optimizer {cfg['optimizer']!r}: the reference supports 'adam' and 'sgd'")
        if cfg["optimizer"] == "sgd" and "momentum" not in cfg:
            raise KeyError("optimizer 'sgd' reads cfg['momentum'] (train_utils/optimizer_dm.py:86-92)")
    if not cfg.get("synthetic", True):
        raise NotImplementedError("\"synthetic\": false (the reference's on-disk PartNet h5 / pickle readers) is "
                                  "out of scope: h5py is not in this image")
    return cfg
