"""Checkpoints — the save/load points of the reference
driver, T/run.py:251-262 (save every save_interval updates) and :64-71 (load
with --load), kept with the same `[actor_critic, ob_rms]` meaning.

The reference pickles the whole module: `torch.save([actor_critic, ob_rms])`
and `torch.load(path)`.  That still works here (Policy drops its engine when
pickled), but torch >= 2.6 refuses such a file unless it is loaded with
weights_only=False, which executes code from the file.  save_checkpoint writes
plain tensors and builtins instead — loadable with torch.load(weights_only=True)
— and adds what the reference drops: the optimizer state (Adam moments, step
count, lr) so a resumed run continues bit-identically.

    save_checkpoint(path, actor_critic, ob_rms, agent=agent)
    actor_critic, ob_rms = load_checkpoint(path, device, agent=agent)
"""
import os

import torch

FORMAT = "ppo-dash-amd/checkpoint-1"


def _space(action_space):
    kind = action_space.__class__.__name__
    if kind == "Discrete":
        return {"kind": kind, "n": int(action_space.n)}
    return {"kind": kind, "shape": [int(s) for s in action_space.shape]}


class _Space(object):
    """duck-typed gym space rebuilt from _space() (model.py:29-40 tests __class__.__name__)"""

    def __init__(self, d):
        self.__class__ = type(d["kind"], (_Space,), {})
        if "n" in d:
            self.n = d["n"]
            self.shape = ()
        else:
            self.shape = tuple(d["shape"])


def _ob_rms_state(ob_rms):
    if ob_rms is None:
        return None
    st = {}
    for k in ("mean", "var", "count"):
        v = getattr(ob_rms, k)
        st[k] = torch.as_tensor(v).detach().cpu().clone()
    return st


class RunningMeanStd(object):
    """the fields of baselines' RunningMeanStd that ob_rms carries (envs.py VecNormalize)"""

    def __init__(self, mean, var, count):
        self.mean, self.var, self.count = mean, var, count


def policy_config(actor_critic):
    """Constructor arguments of a Policy (model.py:16), recorded so load can rebuild it."""
    base = actor_critic.base
    cfg = getattr(actor_critic, "_ctor", None)
    if cfg is None:
        raise ValueError("policy_config: Policy was not built through a2c_ppo_acktr.model.Policy")
    return {"obs_shape": list(cfg["obs_shape"]), "action_space": _space(cfg["action_space"]),
            "base": type(base).__name__, "base_kwargs": dict(cfg["base_kwargs"]),
            "vector_obs_len": int(cfg["vector_obs_len"])}


def save_checkpoint(path, actor_critic, ob_rms=None, agent=None, extra=None):
    """Write {policy state_dict, constructor config, ob_rms, optimizer state}.
    Every tensor is copied to the host; the file holds no pickled objects."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    ck = {"format": FORMAT, "config": policy_config(actor_critic),
          "policy": {k: v.detach().cpu().clone() for k, v in actor_critic.state_dict().items()},
          "ob_rms": _ob_rms_state(ob_rms), "optimizer": None, "extra": extra}
    if agent is not None:
        sd = agent.optimizer.state_dict()
        ck["optimizer"] = {"step": int(sd["step"]),
                           "exp_avg": None if sd["exp_avg"] is None else sd["exp_avg"].detach().cpu().clone(),
                           "exp_avg_sq": None if sd["exp_avg_sq"] is None else sd["exp_avg_sq"].detach().cpu().clone(),
                           "param_groups": [{k: (list(v) if isinstance(v, tuple) else v)
                                             for k, v in sd["param_groups"][0].items()}]}
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)   # a crash mid-save never leaves a truncated checkpoint behind


def load_checkpoint(path, device=None, actor_critic=None, agent=None):
    """-> (actor_critic, ob_rms), as `torch.load(...)` returns them at T/run.py:64-66.
    Loads with weights_only=True.  Rebuilds the Policy from the recorded config
    unless one is passed in, or `agent` is (then agent.actor_critic is used; its
    parameters are overwritten in place); restores the optimizer state into
    `agent` when given."""
    from . import model as M

    ck = torch.load(path, map_location="cpu", weights_only=True)
    if ck.get("format") != FORMAT:
        raise ValueError("%s: not a %s file" % (path, FORMAT))
    cfg = ck["config"]
    if actor_critic is None and agent is not None:
        # the agent trains agent.actor_critic: load into that policy, or the
        # rollouts would act with new weights while the update trains stale ones
        actor_critic = agent.actor_critic
    if actor_critic is None:
        base = {"CNNBase": M.CNNBase, "MLPBase": M.MLPBase}[cfg["base"]]
        actor_critic = M.Policy(tuple(cfg["obs_shape"]), _Space(cfg["action_space"]), base=base,
                                base_kwargs=cfg["base_kwargs"], vector_obs_len=cfg["vector_obs_len"])
    if device is not None:
        actor_critic.to(device)
    with torch.no_grad():
        sd = actor_critic.state_dict()
        missing = set(sd) ^ set(ck["policy"])
        if missing:
            raise KeyError("checkpoint/policy parameter mismatch: %s" % sorted(missing))
        for k, v in ck["policy"].items():
            if sd[k].shape != v.shape:
                raise ValueError("%s: shape %s in the checkpoint, %s in the policy" % (k, tuple(v.shape),
                                                                                     tuple(sd[k].shape)))
            sd[k].copy_(v)   # in place: engine views of the flat parameter buffer stay bound
    ob = ck["ob_rms"]
    ob_rms = None if ob is None else RunningMeanStd(ob["mean"].numpy(), ob["var"].numpy(), ob["count"].item())
    if agent is not None and ck["optimizer"] is not None:
        o = ck["optimizer"]
        dev = next(actor_critic.parameters()).device
        pg = dict(o["param_groups"][0])
        pg["betas"] = tuple(pg["betas"])
        agent.optimizer.load_state_dict({
            "step": o["step"],
            "exp_avg": None if o["exp_avg"] is None else o["exp_avg"].to(dev),
            "exp_avg_sq": None if o["exp_avg_sq"] is None else o["exp_avg_sq"].to(dev),
            "param_groups": [pg]})
    return actor_critic, ob_rms
