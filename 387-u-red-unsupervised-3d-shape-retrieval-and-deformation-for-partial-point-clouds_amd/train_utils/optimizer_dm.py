"""Drop-in for define_optimizer_dm_re_recon (reference train_utils/optimizer_dm.py:68-104):
Adam (or SGD) over the six trained modules — the embedding layer is excluded, as in
the reference — plus StepLR(lr_stepsize, lr_decay)."""
import torch


def define_optimizer_dm_re_recon(target_encoder_full, param_decoder_full, recon_full, re_net_full,
                                 src_encoder, recon_src, embedding_layer, cfg):
    params = []
    for m in (target_encoder_full, param_decoder_full, re_net_full, recon_full, src_encoder, recon_src):
        params += list(m.parameters())
    if cfg["optimizer"] == "sgd":
        opt = torch.optim.SGD(params, lr=cfg["learning_rate"], momentum=cfg["momentum"],
                              weight_decay=cfg["weight_decay"])
    elif cfg["optimizer"] == "adam" and params and params[0].is_cuda and cfg.get("flat_adam", True):
        # the same Adam (and the six clip_grad_norm_ calls, TrainStep.clip_and_step) over flat
        # HBM buffers: ured_hip/optim.py
        from ured_hip.optim import FlatAdam
        mods = (target_encoder_full, param_decoder_full, re_net_full, recon_full, src_encoder, recon_src)
        opt = FlatAdam(params, [list(m.parameters()) for m in mods], lr=cfg["learning_rate"],
                       betas=(0.9, 0.999), eps=1e-8, weight_decay=cfg["weight_decay"])
    elif cfg["optimizer"] == "adam":
        kw = {}
        if params and params[0].is_cuda and cfg.get("fused_adam", True):
            kw["fused"] = True
        if params and params[0].is_cuda and cfg.get("cuda_graph", False):
            kw["capturable"] = True   # step counters on device: the step can be replayed as a HIP graph
        opt = torch.optim.Adam(params, lr=cfg["learning_rate"], betas=(0.9, 0.999), eps=1e-8,
                               weight_decay=cfg["weight_decay"], **kw)
    else:
        return None
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=cfg["lr_stepsize"], gamma=cfg["lr_decay"])
    return opt, sched
