"""ORACLE — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker (or the timed CPU baseline) — never as the
thing measured or shipped.  The product path (ppo-dash_amd/) never imports it.

A CPU restatement (numpy) of the reference's PPO hot path:

  * RolloutStorage.compute_returns   storage.py:82-121   -> compute_returns()
        (fp32, reference op order; the C twin in gae_oracle.c is bit-exact)
  * advantage normalisation          algo/ppo.py:35-37   -> normalize_advantages()
  * feed_forward_generator indices   storage.py:123-160  -> ff_minibatches()
  * recurrent_generator env order    storage.py:162-223  -> rec_minibatches()
  * CNNBase forward                  model.py:169-199    -> cnn_forward()
  * NNBase._forward_gru              model.py:111-166    -> gru_sequence()
  * FixedCategorical sample/log_probs/entropy/mode
                                     distributions.py:17-27,54-68 -> categorical()
  * PPO clipped loss + value loss + entropy, and their gradients
                                     algo/ppo.py:51-81   -> ppo_loss_grads()
  * clip_grad_norm_ + Adam.step      algo/ppo.py:82-84   -> clip_adam()
  * one whole iteration in T/run.py:168-248 order -> run_iteration()
  * PPO.update over recurrent_generator (GRU BPTT)  -> run_update_recurrent()

All paths above are relative to ppo-dash-study/001_baseline/ppo/ (identical to
ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/ up to the V=0 edits,
SURVEY.md §2.1 row 17).  Network arithmetic is done in float64 (a stricter
checker than the reference's fp32); GAE and the advantage differences are fp32
in the reference's order.  Pinned against tests/golden/*.npz, produced by the
reference itself (tools/gen_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "libppo_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(path)
        f = ctypes.POINTER(ctypes.c_float)
        lib.oracle_compute_returns.argtypes = [f, f, f, f, f, f, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                               ctypes.c_int]
        lib.oracle_adv_stats.argtypes = [f, f, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_double)]
        _LIB = lib
    return _LIB


def _fp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


# ---------------------------------------------------------------------------
# GAE / returns (storage.py:82-121)
# ---------------------------------------------------------------------------
def compute_returns(rewards, value_preds, masks, bad_masks, next_value, use_gae, gamma,
                    gae_lambda, use_proper_time_limits=True, returns=None):
    """C oracle. rewards [T,N]; value_preds/masks/bad_masks [T+1,N]; next_value [N].
    Returns (returns [T+1,N], value_preds_out [T+1,N]); inputs are not modified."""
    r = np.ascontiguousarray(rewards, np.float32).reshape(rewards.shape[0], -1)
    T, N = r.shape
    v = np.ascontiguousarray(value_preds, np.float32).reshape(T + 1, N).copy()
    m = np.ascontiguousarray(masks, np.float32).reshape(T + 1, N)
    bm = np.ascontiguousarray(bad_masks, np.float32).reshape(T + 1, N)
    nv = np.ascontiguousarray(next_value, np.float32).reshape(N)
    ret = (np.zeros((T + 1, N), np.float32) if returns is None
           else np.ascontiguousarray(returns, np.float32).reshape(T + 1, N).copy())
    _lib().oracle_compute_returns(_fp(r), _fp(v), _fp(m), _fp(bm), _fp(nv), _fp(ret), T, N,
                                  float(gamma), float(gae_lambda), int(bool(use_gae)),
                                  int(bool(use_proper_time_limits)))
    return ret, v


def compute_returns_np(rewards, value_preds, masks, bad_masks, next_value, use_gae, gamma,
                       gae_lambda, use_proper_time_limits=True, returns=None):
    """Vectorised-over-lanes numpy twin of compute_returns (same fp32 op order)."""
    r = np.asarray(rewards, np.float32).reshape(rewards.shape[0], -1)
    T, N = r.shape
    v = np.asarray(value_preds, np.float32).reshape(T + 1, N).copy()
    m = np.asarray(masks, np.float32).reshape(T + 1, N)
    bm = np.asarray(bad_masks, np.float32).reshape(T + 1, N)
    ret = (np.zeros((T + 1, N), np.float32) if returns is None
           else np.asarray(returns, np.float32).reshape(T + 1, N).copy())
    g = np.float32(gamma)
    gl = np.float32(gamma * gae_lambda)
    if use_gae:
        v[T] = np.asarray(next_value, np.float32).reshape(N)
        gae = np.zeros(N, np.float32)
        for t in range(T - 1, -1, -1):
            delta = (r[t] + (g * v[t + 1]) * m[t + 1]) - v[t]
            gae = delta + (gl * m[t + 1]) * gae
            if use_proper_time_limits:
                gae = gae * bm[t + 1]
            ret[t] = gae + v[t]
    else:
        ret[T] = np.asarray(next_value, np.float32).reshape(N)
        for t in range(T - 1, -1, -1):
            x = (ret[t + 1] * g) * m[t + 1] + r[t]
            if use_proper_time_limits:
                x = x * bm[t + 1] + (np.float32(1.0) - bm[t + 1]) * v[t]
            ret[t] = x
    return ret, v


def adv_stats(returns, value_preds):
    """(mean, unbiased std) of returns[:-1]-value_preds[:-1] (ppo.py:35-37)."""
    ret = np.ascontiguousarray(returns, np.float32)
    T = ret.shape[0] - 1
    ret = ret.reshape(T + 1, -1)
    N = ret.shape[1]
    v = np.ascontiguousarray(value_preds, np.float32).reshape(T + 1, N)
    out = np.zeros(2, np.float64)
    _lib().oracle_adv_stats(_fp(ret), _fp(v), T, N,
                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return float(out[0]), float(out[1])


def normalize_advantages(returns, value_preds):
    """ppo.py:35-37 — fp32 difference, fp32 (a - mean) / (std + 1e-5)."""
    ret = np.asarray(returns, np.float32)
    T = ret.shape[0] - 1
    adv = ret[:-1] - np.asarray(value_preds, np.float32)[:-1]
    mean, std = adv_stats(returns, value_preds)
    return (adv - np.float32(mean)) / (np.float32(std) + np.float32(1e-5))


# ---------------------------------------------------------------------------
# minibatch samplers (storage.py:123-223).  The permutation itself is
# torch.randperm on the caller's generator (torch's SubsetRandomSampler);
# these restate how the reference cuts it.
# ---------------------------------------------------------------------------
def ff_minibatches(perm, num_mini_batch=None, mini_batch_size=None):
    """BatchSampler(SubsetRandomSampler(range(NT)), NT//M, drop_last=True)."""
    perm = np.asarray(perm, np.int64)
    if mini_batch_size is None:
        assert len(perm) >= num_mini_batch
        mini_batch_size = len(perm) // num_mini_batch
    nb = len(perm) // mini_batch_size
    return [perm[i * mini_batch_size:(i + 1) * mini_batch_size] for i in range(nb)]


def rec_minibatches(perm, num_mini_batch):
    """storage.py:168-170: chunks of N//M envs in perm order (row = t*n_env + j)."""
    perm = np.asarray(perm, np.int64)
    N = len(perm)
    assert N >= num_mini_batch
    per = N // num_mini_batch
    out = []
    for s in range(0, N, per):
        if s + per > N:
            raise IndexError(f"index {N} is out of bounds for dimension 0 with size {N}")
        out.append(perm[s:s + per])
    return out


# ---------------------------------------------------------------------------
# network (model.py:169-199, distributions.py:54-68)
# ---------------------------------------------------------------------------
def cnn_param_shapes(hidden=512, num_inputs=4, num_actions=8, recurrent=False, vector_obs_len=0):
    """named_parameters() order of Policy(obs, Discrete(A), CNNBase, ...)."""
    shapes = []
    if recurrent:  # NNBase.__init__ builds the GRU before CNNBase builds main (model.py:89-95)
        I = hidden + vector_obs_len
        shapes += [("base.gru.weight_ih_l0", (3 * hidden, I)), ("base.gru.weight_hh_l0", (3 * hidden, hidden)),
                   ("base.gru.bias_ih_l0", (3 * hidden,)), ("base.gru.bias_hh_l0", (3 * hidden,))]
    shapes += [("base.main.0.weight", (32, num_inputs, 8, 8)), ("base.main.0.bias", (32,)),
               ("base.main.2.weight", (64, 32, 4, 4)), ("base.main.2.bias", (64,)),
               ("base.main.4.weight", (32, 64, 3, 3)), ("base.main.4.bias", (32,)),
               ("base.main.7.weight", (hidden, 32 * 7 * 7)), ("base.main.7.bias", (hidden,))]
    crit_in = hidden if recurrent else hidden + vector_obs_len
    shapes += [("base.critic_linear.weight", (1, crit_in)), ("base.critic_linear.bias", (1,)),
               ("dist.linear.weight", (num_actions, hidden)), ("dist.linear.bias", (num_actions,))]
    return shapes


def unflatten(flat, shapes, dtype=np.float64):
    out, off = {}, 0
    for name, shp in shapes:
        n = int(np.prod(shp))
        out[name] = np.asarray(flat[off:off + n], dtype).reshape(shp)
        off += n
    assert off == len(flat), (off, len(flat))
    return out


def flatten(d, shapes):
    return np.concatenate([np.asarray(d[n]).reshape(-1) for n, _ in shapes])


def decode_obs(u8):
    """Input convention: u8.float() / 255.0 in fp32."""
    return np.asarray(u8, np.uint8).astype(np.float32) / np.float32(255.0)


def _conv_fwd(x, w, b, stride):
    B, C, H, W = x.shape
    O, _, k, _ = w.shape
    win = sliding_window_view(x, (k, k), axis=(2, 3))[:, :, ::stride, ::stride]
    Ho, Wo = win.shape[2], win.shape[3]
    cols = win.transpose(0, 2, 3, 1, 4, 5).reshape(B * Ho * Wo, C * k * k)
    z = cols @ w.reshape(O, -1).T + b
    return z.reshape(B, Ho, Wo, O).transpose(0, 3, 1, 2), cols


def _conv_bwd(dz, cols, w, x_shape, stride, need_dx=True):
    B, C, H, W = x_shape
    O, _, k, _ = w.shape
    Ho, Wo = dz.shape[2], dz.shape[3]
    dzm = dz.transpose(0, 2, 3, 1).reshape(-1, O)
    dw = (dzm.T @ cols).reshape(w.shape)
    db = dzm.sum(0)
    dx = None
    if need_dx:
        dcols = (dzm @ w.reshape(O, -1)).reshape(B, Ho, Wo, C, k, k)
        dx = np.zeros(x_shape, dz.dtype)
        for ky in range(k):
            for kx in range(k):
                dx[:, :, ky:ky + stride * (Ho - 1) + 1:stride, kx:kx + stride * (Wo - 1) + 1:stride] += \
                    dcols[:, :, :, :, ky, kx].transpose(0, 3, 1, 2)
    return dw, db, dx


def cnn_trunk(p, x):
    """CNNBase.main (model.py:176-180): returns features [B,H] and the cache."""
    x = np.asarray(x, p["base.main.0.weight"].dtype)
    z1, c1 = _conv_fwd(x, p["base.main.0.weight"], p["base.main.0.bias"], 4)
    a1 = np.maximum(z1, 0)
    z2, c2 = _conv_fwd(a1, p["base.main.2.weight"], p["base.main.2.bias"], 2)
    a2 = np.maximum(z2, 0)
    z3, c3 = _conv_fwd(a2, p["base.main.4.weight"], p["base.main.4.bias"], 1)
    a3 = np.maximum(z3, 0)
    f = a3.reshape(a3.shape[0], -1)
    z4 = f @ p["base.main.7.weight"].T + p["base.main.7.bias"]
    h = np.maximum(z4, 0)
    cache = dict(x_shape=x.shape, c1=c1, a1=a1, c2=c2, a2=a2, c3=c3, a3=a3, f=f, h=h)
    return h, cache


def heads(p, h):
    value = h @ p["base.critic_linear.weight"].T + p["base.critic_linear.bias"]
    logits = h @ p["dist.linear.weight"].T + p["dist.linear.bias"]
    return value[:, 0], logits


def cnn_forward(p, x):
    h, cache = cnn_trunk(p, x)
    value, logits = heads(p, h)
    return value, logits, cache


def categorical(logits, exp_noise=None, deterministic=False):
    """FixedCategorical(logits) (distributions.py:17-27; torch Categorical):
    norm = logits - logsumexp; probs = softmax; sample = argmax(probs / E),
    E ~ Exp(1) (torch>=2 multinomial fast path for one sample); mode = argmax(probs).
    Returns dict(norm_logits, probs, action, log_prob, entropy)."""
    z = np.asarray(logits, np.float64)
    zmax = z.max(-1, keepdims=True)
    lse = zmax + np.log(np.exp(z - zmax).sum(-1, keepdims=True))
    nl = z - lse
    probs = np.exp(nl)
    probs = probs / probs.sum(-1, keepdims=True)
    if deterministic or exp_noise is None:
        action = probs.argmax(-1)
    else:
        action = (probs / np.asarray(exp_noise, np.float64)).argmax(-1)
    logp = np.take_along_axis(nl, action[:, None], -1)[:, 0]
    ent = -(nl * probs).sum(-1)
    return dict(norm_logits=nl, probs=probs, action=action.astype(np.int64), log_prob=logp, entropy=ent)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def gru_cell(p, x, h):
    """torch.nn.GRU single layer, gate order (r, z, n)."""
    Wih, Whh = p["base.gru.weight_ih_l0"], p["base.gru.weight_hh_l0"]
    bih, bhh = p["base.gru.bias_ih_l0"], p["base.gru.bias_hh_l0"]
    H = h.shape[1]
    gi = x @ Wih.T + bih
    gh = h @ Whh.T + bhh
    r = sigmoid(gi[:, :H] + gh[:, :H])
    zg = sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = np.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return (1 - zg) * n + zg * h


def gru_sequence(p, x, h0, masks):
    """NNBase._forward_gru multi-step branch (model.py:116-165) restated per step:
    h_t_in = h_{t-1} * m_t (identical to the reference's segment split)."""
    T, N = masks.shape[:2]
    xs = x.reshape(T, N, -1)
    h = np.asarray(h0, np.float64)
    outs = []
    for t in range(T):
        h = gru_cell(p, xs[t], h * masks[t].reshape(N, 1))
        outs.append(h)
    return np.concatenate(outs, 0), h


def gru_sequence_cache(p, x, h0, masks):
    """gru_sequence with everything the backward needs; x [T*n, I], masks [T, n]."""
    T, n = masks.shape[:2]
    xs = x.reshape(T, n, -1)
    H = h0.shape[1]
    Wih, Whh = p["base.gru.weight_ih_l0"], p["base.gru.weight_hh_l0"]
    bih, bhh = p["base.gru.bias_ih_l0"], p["base.gru.bias_hh_l0"]
    h = np.asarray(h0, np.float64)
    cache = []
    outs = []
    for t in range(T):
        hin = h * masks[t].reshape(n, 1)
        gi = xs[t] @ Wih.T + bih
        gh = hin @ Whh.T + bhh
        r = sigmoid(gi[:, :H] + gh[:, :H])
        z = sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
        nn_ = np.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
        h = (1 - z) * nn_ + z * hin
        cache.append((hin, r, z, nn_, gh[:, 2 * H:]))
        outs.append(h)
    return np.concatenate(outs, 0), cache


def gru_backward(p, x, masks, cache, dout):
    """BPTT of gru_sequence_cache: dout [T*n, H] = dL/d(outputs) -> (grads, dx [T*n, I])."""
    T, n = masks.shape[:2]
    H = cache[0][0].shape[1]
    Wih, Whh = p["base.gru.weight_ih_l0"], p["base.gru.weight_hh_l0"]
    xs = x.reshape(T, n, -1)
    do = dout.reshape(T, n, H)
    g = {k: np.zeros_like(p[k]) for k in ("base.gru.weight_ih_l0", "base.gru.weight_hh_l0",
                                          "base.gru.bias_ih_l0", "base.gru.bias_hh_l0")}
    dx = np.zeros_like(xs)
    carry = np.zeros((n, H))
    for t in range(T - 1, -1, -1):
        hin, r, z, nn_, ghn = cache[t]
        dh = do[t] + carry
        dn = dh * (1 - z)
        dz = dh * (hin - nn_)
        dan = dn * (1 - nn_ ** 2)
        dar = dan * ghn * r * (1 - r)
        daz = dz * z * (1 - z)
        dgi = np.concatenate([dar, daz, dan], 1)
        dgh = np.concatenate([dar, daz, dan * r], 1)
        g["base.gru.weight_ih_l0"] += dgi.T @ xs[t]
        g["base.gru.bias_ih_l0"] += dgi.sum(0)
        g["base.gru.weight_hh_l0"] += dgh.T @ hin
        g["base.gru.bias_hh_l0"] += dgh.sum(0)
        dx[t] = dgi @ Wih
        carry = (dh * z + dgh @ Whh) * masks[t].reshape(n, 1)
    return g, dx.reshape(T * n, -1)


def recurrent_forward(p, obs_f32, vec, h0, masks):
    """CNNBase(recurrent) forward over a [T*n] sequence batch (rows t*n + j)."""
    feat, cache = cnn_trunk(p, obs_f32)
    x = np.concatenate([feat, np.asarray(vec, np.float64).reshape(feat.shape[0], -1)], 1)
    out, gcache = gru_sequence_cache(p, x, h0, masks)
    value, logits = heads(p, out)
    cache.update(x=x, gcache=gcache, out=out, masks=masks)
    return value, logits, cache


def recurrent_backward(p, cache, g_value, g_logits):
    H = p["base.main.7.weight"].shape[0]
    out = cache["out"]
    g = {}
    g["base.critic_linear.weight"] = g_value[None, :] @ out
    g["base.critic_linear.bias"] = np.array([g_value.sum()])
    g["dist.linear.weight"] = g_logits.T @ out
    g["dist.linear.bias"] = g_logits.sum(0)
    dout = g_value[:, None] * p["base.critic_linear.weight"] + g_logits @ p["dist.linear.weight"]
    gg, dx = gru_backward(p, cache["x"], cache["masks"], cache["gcache"], dout)
    g.update(gg)
    dz4 = dx[:, :H] * (cache["h"] > 0)
    g["base.main.7.weight"] = dz4.T @ cache["f"]
    g["base.main.7.bias"] = dz4.sum(0)
    da3 = (dz4 @ p["base.main.7.weight"]).reshape(cache["a3"].shape)
    dz3 = da3 * (cache["a3"] > 0)
    dw, db, da2 = _conv_bwd(dz3, cache["c3"], p["base.main.4.weight"], cache["a2"].shape, 1)
    g["base.main.4.weight"], g["base.main.4.bias"] = dw, db
    dz2 = da2 * (cache["a2"] > 0)
    dw, db, da1 = _conv_bwd(dz2, cache["c2"], p["base.main.2.weight"], cache["a1"].shape, 2)
    g["base.main.2.weight"], g["base.main.2.bias"] = dw, db
    dz1 = da1 * (cache["a1"] > 0)
    dw, db, _ = _conv_bwd(dz1, cache["c1"], p["base.main.0.weight"], cache["x_shape"], 4, need_dx=False)
    g["base.main.0.weight"], g["base.main.0.bias"] = dw, db
    return g


# ---------------------------------------------------------------------------
# MLPBase (model.py:202-234): actor / critic towers Linear-Tanh-Linear-Tanh
# ---------------------------------------------------------------------------
def mlp_param_shapes(num_inputs=4, hidden=64, num_actions=2):
    """named_parameters() order of Policy((num_inputs,), Discrete(A), MLPBase)."""
    I, H = num_inputs, hidden
    return [("base.actor.0.weight", (H, I)), ("base.actor.0.bias", (H,)),
            ("base.actor.2.weight", (H, H)), ("base.actor.2.bias", (H,)),
            ("base.critic.0.weight", (H, I)), ("base.critic.0.bias", (H,)),
            ("base.critic.2.weight", (H, H)), ("base.critic.2.bias", (H,)),
            ("base.critic_linear.weight", (1, H)), ("base.critic_linear.bias", (1,)),
            ("dist.linear.weight", (num_actions, H)), ("dist.linear.bias", (num_actions,))]


def mlp_forward(p, x):
    """value = critic_linear(critic(x)), logits = dist.linear(actor(x)) (model.py:222-234)."""
    x = np.asarray(x, p["base.actor.0.weight"].dtype)
    cache = dict(x=x)
    for tower in ("actor", "critic"):
        h1 = np.tanh(x @ p[f"base.{tower}.0.weight"].T + p[f"base.{tower}.0.bias"])
        h2 = np.tanh(h1 @ p[f"base.{tower}.2.weight"].T + p[f"base.{tower}.2.bias"])
        cache[tower] = (h1, h2)
    value = cache["critic"][1] @ p["base.critic_linear.weight"].T + p["base.critic_linear.bias"]
    logits = cache["actor"][1] @ p["dist.linear.weight"].T + p["dist.linear.bias"]
    return value[:, 0], logits, cache


def mlp_backward(p, cache, g_value, g_logits):
    x = cache["x"]
    g_value = np.asarray(g_value, x.dtype)
    g_logits = np.asarray(g_logits, x.dtype)
    a2, c2 = cache["actor"][1], cache["critic"][1]
    g = {"base.critic_linear.weight": g_value[None, :] @ c2, "base.critic_linear.bias": np.array([g_value.sum()]),
         "dist.linear.weight": g_logits.T @ a2, "dist.linear.bias": g_logits.sum(0)}
    douts = {"critic": g_value[:, None] * p["base.critic_linear.weight"], "actor": g_logits @ p["dist.linear.weight"]}
    for tower in ("actor", "critic"):
        h1, h2 = cache[tower]
        dz2 = douts[tower] * (1 - h2 * h2)
        g[f"base.{tower}.2.weight"] = dz2.T @ h1
        g[f"base.{tower}.2.bias"] = dz2.sum(0)
        dz1 = (dz2 @ p[f"base.{tower}.2.weight"]) * (1 - h1 * h1)
        g[f"base.{tower}.0.weight"] = dz1.T @ x
        g[f"base.{tower}.0.bias"] = dz1.sum(0)
    return g


# ---------------------------------------------------------------------------
# CartPole-v1 (gym.envs.classic_control.cartpole, the c1 environment; the
# reference reaches it through T/envs.py:40-96).  fp32 restatement of the
# synthetic GPU env's dynamics and its counter-RNG resets.
# ---------------------------------------------------------------------------
_M64 = (1 << 64) - 1


def mix64(z):
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def u01_open0(h):
    return ((h >> np.uint64(40)).astype(np.uint32).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def cartpole_reset_state(seed, counter, lanes):
    lanes = np.asarray(lanes, np.uint64)
    with np.errstate(over="ignore"):
        key = np.uint64(seed) ^ mix64(np.uint64(counter) * np.uint64(0x100000001B3) + lanes * np.uint64(0x9E3779B1)
                                      + np.uint64(0xCA27))
        st = [(u01_open0(mix64(key + np.uint64(i))) - np.float32(0.5)) * np.float32(0.1) for i in range(4)]
    return np.stack(st, 1).astype(np.float32)


def cartpole_step(state, steps, action, seed, counter, max_steps=500):
    """One auto-resetting step for every lane.  Returns (state', steps', obs,
    reward, mask, bad_mask, ep_len); action None = reset all lanes."""
    state = np.array(state, np.float32)
    steps = np.array(steps, np.int32)
    N = state.shape[0]
    f = np.float32
    reward = np.zeros(N, f)
    mask = np.ones(N, f)
    bad = np.ones(N, f)
    ep_len = np.zeros(N, f)
    if action is None:
        reset = np.ones(N, bool)
    else:
        gravity, masscart, masspole = f(9.8), f(1.0), f(0.1)
        total_mass = masspole + masscart
        length = f(0.5)
        pml = masspole * length
        tau = f(0.02)
        theta_thr, x_thr = f(12.0 * 2.0 * 3.14159265358979 / 360.0), f(2.4)
        x, x_dot, theta, theta_dot = (state[:, i].copy() for i in range(4))
        force = np.where(np.asarray(action).reshape(-1) == 1, f(10.0), f(-10.0)).astype(f)
        ct, sn = np.cos(theta), np.sin(theta)
        temp = (force + pml * theta_dot * theta_dot * sn) / total_mass
        thetaacc = (gravity * sn - ct * temp) / (length * (f(4.0 / 3.0) - masspole * ct * ct / total_mass))
        xacc = temp - pml * thetaacc * ct / total_mass
        x = x + tau * x_dot
        x_dot = x_dot + tau * xacc
        theta = theta + tau * theta_dot
        theta_dot = theta_dot + tau * thetaacc
        state = np.stack([x, x_dot, theta, theta_dot], 1).astype(f)
        steps = steps + 1
        done = (x < -x_thr) | (x > x_thr) | (theta < -theta_thr) | (theta > theta_thr)
        trunc = ~done & (steps >= max_steps)
        reward[:] = 1.0
        mask[done | trunc] = 0.0
        bad[trunc] = 0.0
        reset = done | trunc
        ep_len[reset] = steps[reset]
    if reset.any():
        lanes = np.nonzero(reset)[0]
        state[lanes] = cartpole_reset_state(seed, counter, lanes)
        steps[lanes] = 0
    return state, steps, state.copy(), reward, mask, bad, ep_len


# ---------------------------------------------------------------------------
# PPO loss and its gradients (algo/ppo.py:61-81) with torch's autograd
# conventions: min/max split the gradient 1/2-1/2 at ties; clamp passes it
# inside the closed interval; relu passes it where the output is > 0.
# ---------------------------------------------------------------------------
def loss_head_grads(value, logits, actions, old_logp, adv, vpred_old, returns, clip,
                    value_coef, entropy_coef, use_clipped_value_loss=True):
    B = value.shape[0]
    cat = categorical(logits)
    nl, probs, ent_row = cat["norm_logits"], cat["probs"], cat["entropy"]
    a = np.asarray(actions).reshape(B).astype(np.int64)
    logp = np.take_along_axis(nl, a[:, None], -1)[:, 0]
    A = np.asarray(adv, np.float64).reshape(B)
    ratio = np.exp(logp - np.asarray(old_logp, np.float64).reshape(B))
    surr1 = ratio * A
    rc = np.clip(ratio, 1.0 - clip, 1.0 + clip)
    surr2 = rc * A
    action_loss = -np.minimum(surr1, surr2).mean()
    w1 = np.where(surr1 < surr2, 1.0, np.where(surr1 == surr2, 0.5, 0.0))
    w2 = 1.0 - w1
    inr = ((ratio >= 1.0 - clip) & (ratio <= 1.0 + clip)).astype(np.float64)
    g_logp = -(1.0 / B) * (w1 * A + w2 * A * inr) * ratio
    v = np.asarray(value, np.float64).reshape(B)
    vo = np.asarray(vpred_old, np.float64).reshape(B)
    R = np.asarray(returns, np.float64).reshape(B)
    if use_clipped_value_loss:
        dv = v - vo
        vpc = vo + np.clip(dv, -clip, clip)
        l1 = (v - R) ** 2
        l2 = (vpc - R) ** 2
        value_loss = 0.5 * np.maximum(l1, l2).mean()
        u1 = np.where(l1 > l2, 1.0, np.where(l1 == l2, 0.5, 0.0))
        u2 = 1.0 - u1
        vin = ((dv >= -clip) & (dv <= clip)).astype(np.float64)
        g_v = value_coef * (0.5 / B) * (u1 * 2 * (v - R) + u2 * 2 * (vpc - R) * vin)
    else:
        value_loss = 0.5 * ((R - v) ** 2).mean()
        g_v = value_coef * (1.0 / B) * (v - R)
    entropy = ent_row.mean()
    onehot = np.zeros_like(probs)
    onehot[np.arange(B), a] = 1.0
    g_logits = g_logp[:, None] * (onehot - probs) + (entropy_coef / B) * probs * (nl + ent_row[:, None])
    return dict(value_loss=value_loss, action_loss=action_loss, entropy=entropy,
                g_value=g_v, g_logits=g_logits, logp=logp)


def cnn_backward(p, cache, g_value, g_logits):
    """Backward of cnn_forward for dL/dvalue [B], dL/dlogits [B,A] → grads dict."""
    h = cache["h"]
    g_value = np.asarray(g_value, h.dtype)
    g_logits = np.asarray(g_logits, h.dtype)
    g = {}
    g["base.critic_linear.weight"] = g_value[None, :] @ h
    g["base.critic_linear.bias"] = np.array([g_value.sum()])
    g["dist.linear.weight"] = g_logits.T @ h
    g["dist.linear.bias"] = g_logits.sum(0)
    dh = g_value[:, None] * p["base.critic_linear.weight"] + g_logits @ p["dist.linear.weight"]
    dz4 = dh * (h > 0)
    g["base.main.7.weight"] = dz4.T @ cache["f"]
    g["base.main.7.bias"] = dz4.sum(0)
    da3 = (dz4 @ p["base.main.7.weight"]).reshape(cache["a3"].shape)
    dz3 = da3 * (cache["a3"] > 0)
    dw, db, da2 = _conv_bwd(dz3, cache["c3"], p["base.main.4.weight"], cache["a2"].shape, 1)
    g["base.main.4.weight"], g["base.main.4.bias"] = dw, db
    dz2 = da2 * (cache["a2"] > 0)
    dw, db, da1 = _conv_bwd(dz2, cache["c2"], p["base.main.2.weight"], cache["a1"].shape, 2)
    g["base.main.2.weight"], g["base.main.2.bias"] = dw, db
    dz1 = da1 * (cache["a1"] > 0)
    dw, db, _ = _conv_bwd(dz1, cache["c1"], p["base.main.0.weight"], cache["x_shape"], 4, need_dx=False)
    g["base.main.0.weight"], g["base.main.0.bias"] = dw, db
    return g


def clip_adam(params, grads, m, v, step, lr, eps, max_norm, beta1=0.9, beta2=0.999):
    """clip_grad_norm_(max_norm) then torch.optim.Adam single-tensor step `step`
    (1-based) on flat float64 vectors; returns (params, m, v, clipped, total_norm)."""
    total = float(np.sqrt((grads.astype(np.float64) ** 2).sum()))
    coef = max_norm / (total + 1e-6)
    g = grads * min(coef, 1.0)
    m = m + (1 - beta1) * (g - m)
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = np.sqrt(v) / (bc2 ** 0.5) + eps
    params = params - (lr / bc1) * (m / denom)
    return params, m, v, g, total


def run_iteration(flat_params, shapes, obs_u8, exp_noise, rewards, masks, perms, *, num_mini_batch,
                  clip=0.1, value_coef=0.5, entropy_coef=0.001, lr=1e-4, eps=1e-5, max_grad_norm=0.5,
                  gamma=0.99, gae_lambda=0.95, dtype=np.float64):
    """One T/run.py:168-248 iteration (feed-forward CNN) replayed on recorded env
    data: obs_u8 [T+1,N,C,84,84], exp_noise [T,N,A], rewards/masks [T,N],
    perms [E, N*T] (the randperms the update draws).  Returns a dict."""
    T1, N = obs_u8.shape[:2]
    T = T1 - 1
    p = unflatten(flat_params, shapes, dtype)
    vals, acts, logps = np.zeros((T, N)), np.zeros((T, N), np.int64), np.zeros((T, N))
    for t in range(T):
        value, logits, _ = cnn_forward(p, decode_obs(obs_u8[t]))
        c = categorical(logits, exp_noise[t])
        vals[t], acts[t], logps[t] = value, c["action"], c["log_prob"]
    nv, _, _ = cnn_forward(p, decode_obs(obs_u8[T]))
    vp = np.zeros((T + 1, N), np.float32)
    vp[:T] = vals.astype(np.float32)
    mk = np.ones((T + 1, N), np.float32)
    mk[1:] = np.asarray(masks, np.float32).reshape(T, N)
    ret, vp = compute_returns(np.asarray(rewards, np.float32).reshape(T, N), vp, mk, np.ones_like(mk),
                              nv.astype(np.float32), True, gamma, gae_lambda, False)
    adv = normalize_advantages(ret, vp)
    flat = np.asarray(flat_params, dtype).copy()
    m = np.zeros_like(flat)
    v = np.zeros_like(flat)
    step = 0
    losses = np.zeros(3)
    first = None
    obs_rows = obs_u8[:T].reshape(T * N, *obs_u8.shape[2:])
    for perm in perms:
        for idx in ff_minibatches(perm, num_mini_batch):
            p = unflatten(flat, shapes, dtype)
            value, logits, cache = cnn_forward(p, decode_obs(obs_rows[idx]))
            lg = loss_head_grads(value, logits, acts.reshape(-1)[idx], logps.reshape(-1)[idx],
                                 adv.reshape(-1)[idx], vp[:T].reshape(-1)[idx], ret[:T].reshape(-1)[idx],
                                 clip, value_coef, entropy_coef)
            g = flatten(cnn_backward(p, cache, lg["g_value"], lg["g_logits"]), shapes).astype(dtype)
            step += 1
            flat, m, v, gc, _ = clip_adam(flat, g, m, v, step, lr, eps, max_grad_norm)
            if first is None:
                first = dict(values=value, logp=lg["logp"], clipped_grad=gc)
            losses += [lg["value_loss"], lg["action_loss"], lg["entropy"]]
    losses /= len(perms) * num_mini_batch   # ppo.py:90 divides by epochs x num_mini_batch
    return dict(values=vals, actions=acts, log_probs=logps, next_value=nv, returns=ret,
                value_preds=vp, advantages=adv, final_params=flat, losses=losses, first=first,
                last_clipped_grad=gc)


def run_update_recurrent(flat_params, shapes, obs_u8, vec, h0, masks, actions, old_logp, value_preds, returns,
                         perms, *, num_mini_batch, clip=0.1, value_coef=0.5, entropy_coef=0.01, lr=1e-3,
                         eps=1e-5, max_grad_norm=0.5, dtype=np.float64):
    """PPO.update of a recurrent policy (algo/ppo.py:34-96 with
    recurrent_generator, storage.py:162-223; the GRU over each env column from
    the rollout's first hidden state, model.py:116-165) replayed on a recorded
    rollout: obs_u8 [T+1,N,C,84,84], vec [T+1,N,V], h0 [N,H] (hidden state of
    step 0), masks [T+1,N], actions / old_logp [T,N], value_preds / returns
    [T+1,N] (fp32, as compute_returns left them), perms [E,N] (the randperms
    the update draws).  Returns final params, per-minibatch losses, each
    minibatch's pre-clip gradient and total norm, and the epoch-mean losses."""
    T1, N = obs_u8.shape[:2]
    T = T1 - 1
    adv = normalize_advantages(np.asarray(returns, np.float32).reshape(T + 1, N),
                               np.asarray(value_preds, np.float32).reshape(T + 1, N))
    flat = np.asarray(flat_params, dtype).copy()
    m = np.zeros_like(flat)
    v = np.zeros_like(flat)
    step = 0
    mb_losses, preclip, norms = [], [], []
    vp = np.asarray(value_preds, np.float64).reshape(T + 1, N)
    ret = np.asarray(returns, np.float64).reshape(T + 1, N)
    acts = np.asarray(actions).reshape(T, N)
    olp = np.asarray(old_logp, np.float64).reshape(T, N)
    mk = np.asarray(masks, np.float64).reshape(T + 1, N)
    for perm in perms:
        for envs in rec_minibatches(perm, num_mini_batch):
            p = unflatten(flat, shapes, dtype)
            obs = obs_u8[:T][:, envs].reshape(T * len(envs), *obs_u8.shape[2:])
            x_vec = np.asarray(vec, np.float64)[:T][:, envs].reshape(T * len(envs), -1)
            value, logits, cache = recurrent_forward(p, decode_obs(obs), x_vec, np.asarray(h0, dtype)[envs],
                                                     mk[:T][:, envs])
            f = lambda a: a[:, envs].reshape(-1)  # noqa: E731  rows t * n + j (_flatten_helper order)
            lg = loss_head_grads(value, logits, f(acts), f(olp), f(adv), f(vp[:T]), f(ret[:T]), clip,
                                 value_coef, entropy_coef)
            g = flatten(recurrent_backward(p, cache, lg["g_value"], lg["g_logits"]), shapes).astype(dtype)
            step += 1
            flat, m, v, _, total = clip_adam(flat, g, m, v, step, lr, eps, max_grad_norm)
            mb_losses.append([lg["value_loss"], lg["action_loss"], lg["entropy"]])
            preclip.append(g)
            norms.append(total)
    mb_losses = np.array(mb_losses)
    return dict(final_params=flat, mb_losses=mb_losses, preclip_grads=preclip, total_norms=np.array(norms),
                losses=mb_losses.mean(0), advantages=adv)
