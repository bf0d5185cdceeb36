"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker (or the timed CPU baseline) — never as the
thing measured or shipped.  The product path (ppo-dash_amd/) never imports it.

A restatement of the reference's own CPU path in the reference's own framework
(PyTorch ops, autograd, torch.optim.Adam, clip_grad_norm_), so that it runs the
same ATen kernels the reference runs on a CPU:

  CNNBase forward            model.py:169-199 (B/ppo/model.py:192-199, V = 0)
                             -> cnn_forward()
  Policy.act + Categorical   model.py:54-66, distributions.py:17-27,54-68
                             -> act()
  compute_returns (GAE)      storage.py:82-121 (use_proper_time_limits=False)
                             -> compute_returns()
  feed_forward_generator     storage.py:123-160 (BatchSampler(SubsetRandomSampler))
  PPO.update                 algo/ppo.py:34-96 -> ppo_update()
  one T/run.py:168-248 iteration on the synthetic env -> run_iteration()

Paths are relative to ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/.
Pinned against tests/golden/cnn_update.npz (recorded by importing the
reference, tools/gen_golden.py) in tests/test_oracle_golden.py.

Two uses:
  * bench.py's cpu_baseline times run_iteration() at the reference's thread
    setting (torch.set_num_threads(1), T/run.py:55) and at the host's core count;
  * tests/test_full_size.py uses minibatch_grads() in float64 (chunked autograd on
    whatever device holds the tensors) as the reference gradient of a full
    65,536-row minibatch.
"""
import torch
import torch.nn.functional as F

# named_parameters() order of Policy(obs, Discrete(A), CNNBase(recurrent=False))
PARAM_NAMES = ("base.main.0.weight", "base.main.0.bias", "base.main.2.weight", "base.main.2.bias",
               "base.main.4.weight", "base.main.4.bias", "base.main.7.weight", "base.main.7.bias",
               "base.critic_linear.weight", "base.critic_linear.bias", "dist.linear.weight", "dist.linear.bias")


def param_shapes(hidden=512, num_inputs=4, num_actions=8):
    return [(32, num_inputs, 8, 8), (32,), (64, 32, 4, 4), (64,), (32, 64, 3, 3), (32,),
            (hidden, 32 * 7 * 7), (hidden,), (1, hidden), (1,), (num_actions, hidden), (num_actions,)]


def unflatten(flat, hidden=512, num_inputs=4, num_actions=8, dtype=torch.float32, device="cpu",
              requires_grad=False):
    """flat parameter vector (named_parameters order) -> list of leaf tensors"""
    flat = torch.as_tensor(flat)
    out, off = [], 0
    for shp in param_shapes(hidden, num_inputs, num_actions):
        n = 1
        for d in shp:
            n *= d
        t = flat[off:off + n].reshape(shp).to(device=device, dtype=dtype).clone()
        t.requires_grad_(requires_grad)
        out.append(t)
        off += n
    return out


def conv_unfold(x, w, b, stride):
    """F.conv2d as an explicit im2col GEMM (F.unfold + matmul): the same sum in
    any dtype on any device — used for the float64 reference on the GPU, where
    the vendor convolution library has no float64 path."""
    B, _, Hx, Wx = x.shape
    O, _, k, _ = w.shape
    cols = F.unfold(x, k, stride=stride)                       # [B, C*k*k, L]
    out = torch.matmul(w.reshape(O, -1), cols) + b.reshape(1, O, 1)
    Ho = (Hx - k) // stride + 1
    return out.reshape(B, O, Ho, (Wx - k) // stride + 1)


def trunk(p, x, conv=F.conv2d, masks=None):
    """CNNBase.main (model.py:176-180): x [B,C,84,84] -> features [B,H] (post-ReLU).
    masks (optional, 4 tensors shaped like the four ReLU outputs): the ReLU
    decisions to apply instead of (pre-activation > 0) — lets a reference take
    another implementation's decisions so a gradient comparison measures
    arithmetic, not which rows sit within a rounding of a ReLU boundary."""
    w1, b1, w2, b2, w3, b3, w4, b4 = p[:8]
    relu = (lambda z, k: F.relu(z)) if masks is None else (lambda z, k: z * masks[k].to(z.dtype))  # noqa: E731
    h = relu(conv(x, w1, b1, 4), 0)
    h = relu(conv(h, w2, b2, 2), 1)
    h = relu(conv(h, w3, b3, 1), 2)
    return relu(F.linear(h.reshape(h.shape[0], -1), w4, b4), 3)


def cnn_forward(p, x, conv=F.conv2d, masks=None):
    """CNNBase trunk + critic_linear (model.py:185-188) + Categorical's linear
    (distributions.py:54-68): x [B,C,84,84] float -> (value [B,1], logits [B,A])"""
    h = trunk(p, x, conv, masks)
    wc, bc, wa, ba = p[8:]
    return F.linear(h, wc, bc), F.linear(h, wa, ba)


def act(p, obs, noise=None, deterministic=False):
    """Policy.act (model.py:54-66): value, action [N,1], log_prob [N,1].  Sampling is
    torch.multinomial on the default generator (FixedCategorical.sample), or, for
    replays of recorded runs, argmax(probs / noise) — the same draw
    (SURVEY.md §8a row a9)."""
    value, logits = cnn_forward(p, obs)
    dist = torch.distributions.Categorical(logits=logits)
    if deterministic:
        action = dist.probs.argmax(dim=-1, keepdim=True)
    elif noise is not None:
        action = (dist.probs / noise).argmax(dim=-1, keepdim=True)
    else:
        action = dist.sample().unsqueeze(-1)
    logp = dist.log_prob(action.squeeze(-1)).view(action.size(0), -1).sum(-1).unsqueeze(-1)
    return value, action, logp


def compute_returns(rewards, value_preds, masks, next_value, gamma, gae_lambda):
    """storage.py:82-121, GAE branch without time limits (the ppo-dash default):
    mutates value_preds[-1], returns `returns` [T+1, N, 1]."""
    returns = torch.zeros_like(value_preds)
    value_preds[-1] = next_value
    gae = 0
    for step in reversed(range(rewards.size(0))):
        delta = rewards[step] + gamma * value_preds[step + 1] * masks[step + 1] - value_preds[step]
        gae = delta + gamma * gae_lambda * masks[step + 1] * gae
        returns[step] = gae + value_preds[step]
    return returns


def ppo_loss(p, obs, actions, old_logp, adv, vpred, ret, clip, value_coef, entropy_coef,
             use_clipped_value_loss=True, conv=F.conv2d, masks=None):
    """algo/ppo.py:57-81 for one minibatch -> (loss, value_loss, action_loss, entropy)"""
    values, logits = cnn_forward(p, obs, conv, masks)
    dist = torch.distributions.Categorical(logits=logits)
    logp = dist.log_prob(actions.squeeze(-1)).view(actions.size(0), -1).sum(-1).unsqueeze(-1)
    ent = dist.entropy().mean()
    ratio = torch.exp(logp - old_logp)
    surr1 = ratio * adv
    surr2 = torch.clamp(ratio, 1.0 - clip, 1.0 + clip) * adv
    action_loss = -torch.min(surr1, surr2).mean()
    if use_clipped_value_loss:
        vclip = vpred + (values - vpred).clamp(-clip, clip)
        value_loss = 0.5 * torch.max((values - ret).pow(2), (vclip - ret).pow(2)).mean()
    else:
        value_loss = 0.5 * (ret - values).pow(2).mean()
    loss = value_loss * value_coef + action_loss - ent * entropy_coef
    return loss, value_loss, action_loss, ent


def ppo_update(p, optimizer, obs, actions, old_logp, vpred, returns, *, ppo_epoch, num_mini_batch, clip,
               value_coef, entropy_coef, max_grad_norm, perms=None, decode=None):
    """PPO.update (algo/ppo.py:34-96) over the storage tensors (obs [T+1,N,...],
    actions/old_logp [T,N,1], vpred/returns [T+1,N,1]); minibatches as
    feed_forward_generator cuts them (storage.py:123-160): torch.randperm on the
    default generator (SubsetRandomSampler) unless `perms` [E, N*T] is given.
    decode maps stored observations to the network input (identity for fp32)."""
    T, N = actions.shape[:2]
    adv = returns[:-1] - vpred[:-1]
    adv = (adv - adv.mean()) / (adv.std() + 1e-5)
    B = T * N
    mb = B // num_mini_batch
    flat = lambda x: x.reshape(B, *x.shape[2:])  # noqa: E731  (_flatten_helper, storage.py:5-6)
    obs_r, act_r, olp_r, vp_r, ret_r, adv_r = (flat(obs[:-1]), flat(actions), flat(old_logp), flat(vpred[:-1]),
                                                flat(returns[:-1]), flat(adv))
    sums = [0.0, 0.0, 0.0]
    for e in range(ppo_epoch):
        perm = perms[e] if perms is not None else torch.randperm(B)
        for start in range(0, B - mb + 1, mb):
            idx = torch.as_tensor(perm[start:start + mb])
            x = obs_r[idx]
            x = decode(x) if decode is not None else x
            loss, vl, al, ent = ppo_loss(p, x, act_r[idx], olp_r[idx], adv_r[idx], vp_r[idx], ret_r[idx], clip,
                                         value_coef, entropy_coef)
            optimizer.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(p, max_grad_norm)
            optimizer.step()
            sums[0] += vl.item()
            sums[1] += al.item()
            sums[2] += ent.item()
    n = ppo_epoch * num_mini_batch
    return [s / n for s in sums]


def env_frames(N, C=4, count=4, gen=None):
    """A pool of synthetic observation batches (u8 / 255 as fp32) the stand-in env
    cycles through, generated outside the timed region: like the GPU's synthetic
    env, the stand-in must cost next to nothing (the reference's env is a Unity
    farm in other processes, outside the path)."""
    return [torch.randint(0, 256, (N, C, 84, 84), generator=gen).float() / 255.0 for _ in range(count)]


def run_iteration(p, optimizer, N, T, *, ppo_epoch=3, num_mini_batch=8, clip=0.1, value_coef=0.5,
                  entropy_coef=0.001, max_grad_norm=0.5, gamma=0.99, gae_lambda=0.95, p_done=0.01, gen=None,
                  frames=None):
    """One T/run.py:168-248 iteration on the reference CPU path: T x (act ->
    synthetic env step -> storage insert) with fp32 observations (the reference's
    storage dtype, storage.py:12), get_value, compute_returns, PPO.update,
    after_update.  The env is a stand-in (frames from env_frames(), U[0,1)
    rewards, Bernoulli(p_done) dones) as in bench.py's GPU workload."""
    C = p[0].shape[1]
    if frames is None:
        frames = env_frames(N, C, gen=gen)
    obs = torch.zeros(T + 1, N, C, 84, 84)
    rewards = torch.zeros(T, N, 1)
    vpred = torch.zeros(T + 1, N, 1)
    logps = torch.zeros(T, N, 1)
    actions = torch.zeros(T, N, 1, dtype=torch.int64)
    masks = torch.ones(T + 1, N, 1)
    obs[0].copy_(frames[0])
    for step in range(T):
        with torch.no_grad():
            v, a, lp = act(p, obs[step])
        frame = frames[(step + 1) % len(frames)]
        done = torch.rand(N, generator=gen) < p_done
        obs[step + 1].copy_(frame)                                           # storage.py:62-73 insert
        actions[step].copy_(a)
        logps[step].copy_(lp)
        vpred[step].copy_(v)
        rewards[step].copy_(torch.rand(N, 1, generator=gen))
        masks[step + 1].copy_((~done).float().unsqueeze(-1))
    with torch.no_grad():
        next_value, _ = cnn_forward(p, obs[-1])
    returns = compute_returns(rewards, vpred, masks, next_value, gamma, gae_lambda)
    losses = ppo_update(p, optimizer, obs, actions, logps, vpred, returns, ppo_epoch=ppo_epoch,
                        num_mini_batch=num_mini_batch, clip=clip, value_coef=value_coef, entropy_coef=entropy_coef,
                        max_grad_norm=max_grad_norm)
    obs[0].copy_(obs[-1])                                                    # after_update, storage.py:75-80
    masks[0].copy_(masks[-1])
    return losses


def _decode(obs, dev, dt):
    x = obs.to(dev).to(dt)
    return x / 255.0 if obs.dtype == torch.uint8 else x


def minibatch_grads(p, obs_u8, actions, old_logp, adv, vpred, ret, *, clip, value_coef, entropy_coef,
                    idx=None, chunk=2048, use_clipped_value_loss=True, conv=conv_unfold, masks=None):
    """Gradient of the PPO minibatch loss (algo/ppo.py:57-81, mean over all B rows)
    with respect to p, by autograd, accumulated over row chunks: every loss term is
    a mean of per-row terms, so Σ_chunks of the chunk losses scaled by |chunk|/B has
    the same gradient.  Row b is storage row idx[b] of the flat planes (obs_u8
    [R,C,84,84], the others [R]) — all rows in order when idx is None.
    u8 observations are decoded as u8/255 (SURVEY §8c input convention), float
    ones (fp16 / fp32 planes) used as stored, on p's device and dtype.  Returns (grads list, [value loss, action loss, entropy])."""
    dt, dev = p[0].dtype, p[0].device
    B = obs_u8.shape[0] if idx is None else idx.numel()
    grads = [torch.zeros_like(t) for t in p]
    tot = [0.0, 0.0, 0.0]
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        rows = slice(s, e) if idx is None else idx[s:e].to(obs_u8.device)
        x = _decode(obs_u8[rows], dev, dt)
        f = lambda t: t[rows].to(dev, dt).reshape(-1, 1)  # noqa: E731
        mk = None if masks is None else [m[s:e].to(dev) for m in masks]
        loss, vl, al, ent = ppo_loss(p, x, actions[rows].to(dev).reshape(-1, 1), f(old_logp), f(adv), f(vpred),
                                     f(ret), clip, value_coef, entropy_coef, use_clipped_value_loss, conv, mk)
        w = (e - s) / B
        g = torch.autograd.grad(loss * w, p)
        for acc, gi in zip(grads, g):
            acc += gi
        tot[0] += vl.item() * w
        tot[1] += al.item() * w
        tot[2] += ent.item() * w
    return grads, tot


def trunk_grads(p_trunk, obs_u8, dfeat, *, idx=None, chunk=2048, conv=conv_unfold):
    """Σ over rows of d(features)/d(trunk parameters) · dfeat — the trunk part of
    the backward given dL/d(features) [B,H] (rows idx[b] of obs_u8, or all)."""
    dt, dev = p_trunk[0].dtype, p_trunk[0].device
    B = dfeat.shape[0]
    grads = [torch.zeros_like(t) for t in p_trunk]
    for s in range(0, B, chunk):
        e = min(B, s + chunk)
        rows = slice(s, e) if idx is None else idx[s:e].to(obs_u8.device)
        x = _decode(obs_u8[rows], dev, dt)
        h = trunk(p_trunk, x, conv)
        g = torch.autograd.grad(h, p_trunk, grad_outputs=dfeat[s:e].to(dev, dt))
        for acc, gi in zip(grads, g):
            acc += gi
    return grads
