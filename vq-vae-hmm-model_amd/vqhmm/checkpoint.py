"""Checkpoints in the reference's formats, written with
torch.save and read with torch.load(weights_only=True).

  save_checkpoint / load_checkpoint   src/utils/data.py:47-60:
        {'epoch', 'model_state_dict', 'optimizer_state_dict', 'loss'}
  model.state_dict() only             train.py:91, training_pipeline/train.py:137
        (VAE_HMM's 18 keys are the reference's, so these load unchanged)

`optimizer` may be a torch optimizer (as in the reference) or a TrainState.  A
TrainState's flat Adam moments and device step counter are exported as, and
restored from, torch.optim.Adam(model.parameters()).state_dict() — built by
torch's own Adam — so a checkpoint resumes under either the reference's
torch.optim.Adam or vqhmm.train_model's fused Adam.
"""
import torch


def _torch_adam(state):
    params = list(state.model.parameters())
    opt = torch.optim.Adam(params, lr=state.lr, betas=state.betas, eps=state.eps)
    index = {id(p): i for i, p in enumerate(state.model.ordered_parameters())}
    return opt, params, index


def adam_state_dict(state):
    """TrainState -> torch.optim.Adam state_dict (param ids in model.parameters() order)."""
    opt, params, index = _torch_adam(state)
    step = int(state.step_dev.item())
    if step > 0:
        for p in params:
            a, b = state.off[index[id(p)]], state.off[index[id(p)] + 1]
            opt.state[p] = {"step": torch.tensor(float(step)),
                            "exp_avg": state.exp_avg[a:b].detach().view_as(p).clone(),
                            "exp_avg_sq": state.exp_avg_sq[a:b].detach().view_as(p).clone()}
    return opt.state_dict()


def load_adam_state_dict(state, sd):
    """torch.optim.Adam state_dict -> TrainState (moments, step, lr/betas/eps)."""
    opt, params, index = _torch_adam(state)
    opt.load_state_dict(sd)
    steps = set()
    with torch.no_grad():
        state.exp_avg.zero_()
        state.exp_avg_sq.zero_()
        for p in params:
            st = opt.state.get(p)
            if not st:
                continue
            a, b = state.off[index[id(p)]], state.off[index[id(p)] + 1]
            state.exp_avg[a:b].copy_(st["exp_avg"].reshape(-1))
            state.exp_avg_sq[a:b].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(int(st["step"]))
    if len(steps) > 1:
        raise ValueError(f"Adam state has different step counts per parameter {sorted(steps)}; "
                         "TrainState keeps one counter")
    state.step_dev.fill_(steps.pop() if steps else 0)
    g = opt.param_groups[0]
    state.lr, state.betas, state.eps = float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"])


def encoder_config(model):
    """The 'config' dict of the encoder-only checkpoint (VQ_VAE+HMM.ipynb:774-781)."""
    enc = model.encoder if hasattr(model, "encoder") else model
    H, D, _ = enc.conv1.weight.shape
    return {"input_dim": int(D), "hidden_dim": int(H), "hidden_dim2": int(enc.conv2.weight.shape[0]),
            "K": int(enc.to_logits.weight.shape[0])}


def save_encoder(model, path, config=None):
    """Encoder-only checkpoint as the notebook writes it (VQ_VAE+HMM.ipynb:774):
    {'model_state_dict': trained.encoder.state_dict(), 'config': {input_dim, hidden_dim,
    hidden_dim2, K}}.  `model` is a VAE_HMM or an Encoder; config defaults to its dims."""
    enc = model.encoder if hasattr(model, "encoder") else model
    cfg = encoder_config(enc) if config is None else dict(config)
    torch.save({"model_state_dict": enc.state_dict(), "config": cfg}, path)


def load_encoder(path, map_location="cpu", defaults=None):
    """Rebuild the Encoder from an encoder-only checkpoint (VQ_VAE+HMM.ipynb:818-827,
    visualize.ipynb:62): dims from ckpt['config'] (missing keys from `defaults`, and
    hidden_dim2 falling back to hidden_dim as the notebook does), weights from
    ckpt['model_state_dict'].  Read with weights_only=True."""
    from .model import Encoder
    ck = torch.load(path, map_location=map_location, weights_only=True)
    cfg = dict(defaults or {})
    cfg.update(ck.get("config", {}))
    hidden = cfg["hidden_dim"]
    enc = Encoder(cfg["input_dim"], hidden, cfg.get("hidden_dim2", hidden), cfg["K"])
    enc.load_state_dict(ck["model_state_dict"])
    return enc


def save_checkpoint(model, optimizer, epoch, loss, path):
    """src/utils/data.py:47-53."""
    from .train import TrainState
    osd = adam_state_dict(optimizer) if isinstance(optimizer, TrainState) else optimizer.state_dict()
    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(), "optimizer_state_dict": osd,
                "loss": loss}, path)


def load_checkpoint(model, optimizer, path):
    """src/utils/data.py:56-60 -> (epoch, loss).  Loads with weights_only=True."""
    from .train import TrainState
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model_state_dict"])
    if isinstance(optimizer, TrainState):
        load_adam_state_dict(optimizer, ck["optimizer_state_dict"])
    elif optimizer is not None:
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    return ck["epoch"], ck["loss"]
