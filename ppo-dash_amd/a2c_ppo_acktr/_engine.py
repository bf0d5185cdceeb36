"""HIP execution engines behind Policy / PPO.

CNNEngine        CNNBase, feed-forward (model.py:169-199)
RecurrentEngine  CNNBase + [vector obs] + GRU (model.py:89-166, 192-199)

Each owns the flat parameter / gradient buffers (every nn.Parameter of the
Policy is re-pointed to a view of one contiguous fp32 buffer, so clip + Adam is
one pass), the per-step packed weight copies, and grow-only workspaces.

Per PPO minibatch (every box is a libppo_hip.so kernel):
  conv1(obs rows gathered by index, u8) -> conv2 -> conv3 -> fc       (MFMA fwd)
  [recurrent: concat vector obs -> gi = x·W_ihᵀ -> T x fused GRU step]
  heads_train (value/logits/Categorical/PPO loss + dL/dlogits, dL/dfeature)
  [recurrent: T x (gate grads, dh·W_hh), dW_hh, dW_ih, dx]
  fc dgrad | fc wgrad | conv3 dgrad | conv3 wgrad | conv2 dgrad | conv2 wgrad | conv1 wgrad
  wgrad slab reduces -> flat grad  [RCCL all-reduce when world_size > 1]
  grad Σg² -> clip + Adam -> pack weights
"""
import contextlib

import os

import torch

from . import _dist
from ._hip import call, ptr, stream

# ppo_trunk_fwd (conv1 -> conv2 -> conv3 in one launch) for u8 rows; PPO_FUSED_TRUNK=0
# runs the three launches (same-box A/B, tools/ab_bench.sh)
FUSED_TRUNK = os.environ.get("PPO_FUSED_TRUNK", "1") != "0"
FEAT = 32 * 7 * 7  # conv3 output, flattened


def _with_precision(fn):
    """Run an engine entry point at the policy's arithmetic precision: the split
    GEMMs' part-product count is 6 (fp32-accurate) normally and 1 — bf16-rounded
    operands, fp32 accumulation — after Policy.half() (T/run.py:84-85)."""
    def wrapper(self, *args, **kwargs):
        if not getattr(self.policy, "_half_mode", False):
            return fn(self, *args, **kwargs)
        prev = call("ppo_tune_get", b"products")
        if prev != 1:
            call("ppo_tune_set", b"products", 1)
        try:
            return fn(self, *args, **kwargs)
        finally:
            if prev != 1:
                call("ppo_tune_set", b"products", prev)
    wrapper.__name__, wrapper.__doc__ = fn.__name__, fn.__doc__
    return wrapper


class _Workspace:
    def __init__(self):
        self.bufs = {}
        self.version = 0   # bumped by every (re)allocation: a captured graph's buffers moved

    def get(self, name, numel, dtype=torch.float32, device=None):
        t = self.bufs.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype or t.device != device:
            t = torch.empty(max(int(numel), 1), dtype=dtype, device=device)
            self.bufs[name] = t
            self.version += 1
        return t


class CNNEngine:
    """Binds to a Policy whose base is a non-recurrent CNNBase."""

    # parameter indices in policy.parameters() order (named_parameters order)
    W1, B1, W2, B2, W3, B3, W4, B4, WC, BC, WA, BA = range(12)
    recurrent = False

    def __init__(self, policy, device):
        self.policy = policy
        self.device = device
        base = policy.base
        self.C = base.main[0].weight.shape[1]
        self.H = base.main[7].weight.shape[0]
        self.A = policy.dist.linear.weight.shape[0]
        if self.H > 512 or self.H % 4 != 0:
            raise NotImplementedError(f"hidden_size {self.H}: the HIP engine supports multiples of 4 up to 512")
        if not self.recurrent and base.critic_linear.weight.shape[1] != self.H:
            raise NotImplementedError("vector observations with a non-recurrent CNNBase are not supported "
                                      "(the reference crashes there too: Categorical expects hidden_size inputs)")
        self.params = list(policy.parameters())
        self.ws = {"act": _Workspace(), "train": _Workspace()}
        self.act_ws = "act"   # workspace of the forward (act / get_value / evaluate) paths
        self.obs_decode = None   # (mean fp32 [84][84][3] device tensor | None, std) for raw u8 RGB frames
        self.packed = None
        self._pack_key = None
        self.epoch = 0  # bumped by every in-place parameter write done by HIP kernels
        self._flatten()
        self.rng_seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        self.rng_counter = 0
        self._n_cu = None   # CU count of the device, read at the first weight gradient
        self._init_status()

    def _init_status(self):
        # device status words: [0] persistent-GRU timeout of the running update
        # (sticky; gates clip + Adam), [1] optimizer steps skipped by a guard,
        # [2] persistent-GRU timeout of evaluate_sequence
        self.status = torch.zeros(4, dtype=torch.int32, device=self.device)

    def status_ptr(self, i):
        return self.status.data_ptr() + 4 * i

    # ------------------------------------------------------------ parameters
    def _flatten(self):
        n = sum(p.numel() for p in self.params)
        flat = torch.empty(n, device=self.device)
        grad = torch.zeros(n, device=self.device)
        off = 0
        self.offsets = []
        with torch.no_grad():
            for p in self.params:
                k = p.numel()
                flat[off:off + k].copy_(p.data.reshape(-1))
                p.data = flat[off:off + k].view_as(p)
                p.grad = grad[off:off + k].view_as(p)
                self.offsets.append(off)
                off += k
        self.flat, self.grad, self.numel = flat, grad, n
        self.epoch += 1

    @contextlib.contextmanager
    def using_workspace(self, name):
        """Route the forward paths through workspace `name` (e.g. a captured HIP
        graph's own buffers, which no eager call may reallocate)."""
        self.ws.setdefault(name, _Workspace())
        prev, self.act_ws = self.act_ws, name
        try:
            yield self.ws[name]
        finally:
            self.act_ws = prev

    def is_bound(self):
        base = self.flat.data_ptr()
        for p, off in zip(self.params, self.offsets):
            if p.data.data_ptr() != base + 4 * off or not p.is_cuda:
                return False
        return True

    def ensure_bound(self):
        if not self.is_bound():
            self._flatten()

    def pv(self, i):
        """raw pointer of parameter i (in policy.parameters() order)"""
        return self.flat.data_ptr() + 4 * self.offsets[i]

    def gv(self, i):
        return self.grad.data_ptr() + 4 * self.offsets[i]

    def pack(self, force=False):
        key = (sum(p._version for p in self.params), self.epoch)
        if not force and self.packed is not None and key == self._pack_key:
            return
        if self.packed is None:
            self.packed = torch.empty(call("ppo_packed_weights_size", self.H), device=self.device)
            offs = torch.zeros(6, dtype=torch.int64)
            call("ppo_packed_offsets", self.H, offs.data_ptr())
            self.poff = [int(x) for x in offs]
        call("ppo_pack_weights", self.pv(self.W2), self.pv(self.W3), self.pv(self.W4), self.H,
             self.packed.data_ptr(), stream())
        self._pack_extra()
        self._pack_key = key

    def _pack_extra(self):
        pass

    def pk(self, seg):
        """pointer to packed segment: 0 W2p 1 W3p 2 W4p 3 W4T 4 W3d 5 W2d"""
        return self.packed.data_ptr() + 4 * self.poff[seg]

    # ---------------------------------------------------------------- forward
    @staticmethod
    def _obs_args(obs):
        if obs.dtype == torch.uint8:
            return 1
        if obs.dtype == torch.float32:
            return 0
        raise TypeError(f"observations must be uint8, float32 or float16, got {obs.dtype}")

    @staticmethod
    def _is_rgb(obs):
        """raw u8 RGB frames [..., 84, 84, 3] (decoded inside conv1 by obs_decode)"""
        return obs.dtype == torch.uint8 and tuple(obs.shape[-3:]) == (84, 84, 3)

    def set_obs_decode(self, mean, std):
        """NormalizeWrapper + FrameStackMono(2) of raw RGB frames, fused into conv1:
        mean (fp32-representable [84][84][3], or None) and std (u/255: None, 255)."""
        if self.C != 4:
            raise NotImplementedError("the fused RGB decode produces FrameStackMono(2)'s 4 channels (C = 4)")
        if mean is not None:
            m64 = torch.as_tensor(mean, dtype=torch.float64).reshape(84, 84, 3)
            m32 = m64.to(torch.float32)
            if not torch.equal(m32.to(torch.float64), m64):
                raise ValueError("the fused decode needs fp32-representable means (NormalizeWrapper's files hold "
                                 "fp32 values); use ObsPreprocess into fp32 storage otherwise")
            mean = m32.contiguous().to(self.device)
        if not float(std):
            raise ValueError("std must be non-zero")
        self.obs_decode = (mean, float(std))

    def _conv1(self, obs, idx, B, a1, m1, s):
        """conv1 (+ ReLU, + mask bits when m1 is given) of B rows of obs"""
        if self._is_rgb(obs):
            if self.obs_decode is None:
                raise TypeError("raw u8 RGB frames need the fused decode: Policy.set_obs_decode(ObsPreprocess)")
            mean, std = self.obs_decode
            call("ppo_conv1_fwd_rgb", obs.data_ptr(), ptr(idx, torch.int64, "idx"), 0, B, ptr(mean), std,
                 self.pv(self.W1), self.pv(self.B1), a1.data_ptr(), ptr(m1), s)
        elif m1 is not None:
            call("ppo_conv1_fwd_mask", obs.data_ptr(), self._obs_args(obs), ptr(idx, torch.int64, "idx"), 0, self.C,
                 B, self.pv(self.W1), self.pv(self.B1), a1.data_ptr(), m1.data_ptr(), s)
        else:
            call("ppo_conv1_fwd", obs.data_ptr(), self._obs_args(obs), ptr(idx, torch.int64, "idx"), 0, self.C, B,
                 self.pv(self.W1), self.pv(self.B1), a1.data_ptr(), s)

    def _obs_f32(self, obs, idx, B, ws):
        """fp16 observations (RolloutStorage.half(), storage.py:48-58): the rows the
        trunk reads (idx into the plane, or the batch) converted to an fp32
        workspace; u8 / fp32 observations pass through."""
        if obs.dtype != torch.float16:
            return obs, idx
        x = ws.get("obs32", B * self.C * 84 * 84, device=self.device)
        call("ppo_gather_f16_to_f32", obs.data_ptr(), ptr(idx, torch.int64, "idx"), x.data_ptr(), B,
             self.C * 84 * 84, stream())
        return x, None

    def trunk(self, obs, idx, B, ws, out=None, ldo=None):
        """conv1..fc on B samples: obs is either a [B,C,84,84] batch (idx None) or the
        storage plane whose rows idx[b] are gathered inside conv1.  Writes the fc
        output (post-ReLU) to `out` (row stride ldo) or a workspace [B,H]."""
        dev = self.device
        obs, idx = self._obs_f32(obs, idx, B, ws)
        a1 = ws.get("a1", B * 400 * 32, device=dev)
        a2 = ws.get("a2", B * 81 * 64, device=dev)
        a3 = ws.get("a3", B * FEAT, device=dev)
        if out is None:
            out, ldo = ws.get("h", B * self.H, device=dev), self.H
        s = stream()
        train = ws is self.ws["train"]
        # training forward: conv1 and conv2 also write their ReLU masks as bits,
        # read by the conv2 / conv3 dgrads instead of the fp32 activations
        # (and conv3's, read by the fc dgrad instead of a3)
        m1 = ws.get("m1bits", B * 400, dtype=torch.int32, device=dev) if train else None
        m2 = ws.get("m2bits", B * 81, dtype=torch.int64, device=dev) if train else None
        m3 = ws.get("m3bits", B * 49, dtype=torch.int32, device=dev) if train else None
        if obs.dtype == torch.uint8 and self.C == 4 and not self._is_rgb(obs) and FUSED_TRUNK and not train:
            # u8 rows: conv1 -> conv2 -> conv3 in one persistent launch (ppo_trunk_fwd)
            call("ppo_trunk_fwd", obs.data_ptr(), ptr(idx, torch.int64, "idx"), 0, B, self.pv(self.W1),
                 self.pv(self.B1), a1.data_ptr(), None, self.pk(0), self.pv(self.B2), a2.data_ptr(), None,
                 self.pk(1), self.pv(self.B3), a3.data_ptr(), s)
        else:
            self._conv1(obs, idx, B, a1, m1[:B * 400] if train else None, s)
            if train:
                call("ppo_conv2_fwd_mask", a1.data_ptr(), B, self.pk(0), self.pv(self.B2), a2.data_ptr(),
                     m2.data_ptr(), s)
                call("ppo_conv3_fwd_mask", a2.data_ptr(), B, self.pk(1), self.pv(self.B3), a3.data_ptr(),
                     m3.data_ptr(), s)
            else:
                call("ppo_conv2_fwd", a1.data_ptr(), B, self.pk(0), self.pv(self.B2), a2.data_ptr(), s)
                call("ppo_conv3_fwd", a2.data_ptr(), B, self.pk(1), self.pv(self.B3), a3.data_ptr(), s)
        if train:
            self._mask_rows = B
        nb = call("ppo_fc_fwd_ws_bytes", B, self.H)   # rollout-sized B: split-K into a workspace slab
        if nb:
            fws = ws.get("fc_ws", nb // 4, device=dev)
            call("ppo_fc_fwd_ws", a3.data_ptr(), B, self.pk(2), self.pv(self.B4), self.H, out.data_ptr(), ldo,
                 fws.data_ptr(), nb, s)
        else:
            call("ppo_fc_fwd", a3.data_ptr(), B, self.pk(2), self.pv(self.B4), self.H, out.data_ptr(), ldo, s)
        return out

    def _check_obs(self, obs):
        obs = obs if obs.is_cuda else obs.to(self.device)
        if self.obs_decode is not None and self._is_rgb(obs) and obs.dim() == 4:
            return obs.contiguous()
        if tuple(obs.shape[1:]) != (self.C, 84, 84):
            raise RuntimeError(f"CNNBase expects [N,{self.C},84,84] observations"
                               + (" or raw [N,84,84,3] u8 frames" if self.obs_decode is not None else "")
                               + f", got {tuple(obs.shape)}")
        return obs.contiguous()

    def _heads(self, h, B, deterministic=False, noise=None, given=None, want_entropy=False, value_only=False,
               hv=None):
        value = torch.empty(B, 1, device=self.device)
        if value_only:
            action = logp = ent = None
        else:
            action = given if given is not None else torch.empty(B, 1, dtype=torch.int64, device=self.device)
            logp = torch.empty(B, 1, device=self.device)
            ent = torch.empty(B, device=self.device) if want_entropy else None
        if noise is not None:
            noise = noise.to(self.device, torch.float32).contiguous()
            if noise.shape != (B, self.A):
                raise RuntimeError(f"noise must be [{B},{self.A}]")
        self.rng_counter += 1
        call("ppo_heads_act", h.data_ptr(), ptr(hv), B, self.H, self.pv(self.WC), self.pv(self.BC), self.pv(self.WA),
             self.pv(self.BA), self.A, ptr(noise), self.rng_seed, self.rng_counter, int(bool(deterministic)),
             ptr(given.reshape(-1).contiguous() if given is not None else None, torch.int64, "action"),
             value.data_ptr(), None if given is not None or value_only else action.data_ptr(),
             ptr(logp), ptr(ent), stream())
        return value, action, logp, ent

    def mean(self, x):
        """model.py:77 dist.entropy().mean() on the device (0-d tensor)"""
        out = torch.empty((), device=self.device)
        call("ppo_mean_f32", x.data_ptr(), x.numel(), out.data_ptr(), stream())
        return out

    @_with_precision
    def act(self, obs, deterministic=False, noise=None, given=None, want_entropy=False, value_only=False):
        self.ensure_bound()
        self.pack()
        obs = self._check_obs(obs)
        B = obs.shape[0]
        h = self.trunk(obs, None, B, self.ws[self.act_ws])
        return self._heads(h, B, deterministic, noise, given, want_entropy, value_only)

    # --------------------------------------------------------------- training
    def _heads_train(self, storage, adv, idx, feat, B, hp, loss_acc, dfeat, feat_act, feat_v=None, dfeat_v=None):
        ws, dev, H, A, s = self.ws["train"], self.device, self.H, self.A, stream()
        nblk = call("ppo_heads_train_blocks", B)
        part_w = ws.get("part_w", nblk * (1 + A) * H, device=dev)
        part_b = ws.get("part_b", nblk * (1 + A), device=dev)
        part_l = ws.get("part_l", nblk * 4, device=dev)
        inv_b = 1.0 / B
        call("ppo_heads_train", feat.data_ptr(), ptr(feat_v), B, H, self.pv(self.WC), self.pv(self.BC), self.pv(self.WA),
             self.pv(self.BA), A, idx.data_ptr(), 0, storage.actions.data_ptr(), storage.action_log_probs.data_ptr(),
             adv.data_ptr(), storage.value_preds.data_ptr(), storage.returns.data_ptr(), hp["clip"], hp["value_coef"],
             hp["entropy_coef"], inv_b, int(hp["use_clipped_value_loss"]), int(feat_act), dfeat.data_ptr(),
             ptr(dfeat_v), part_w.data_ptr(), part_b.data_ptr(), part_l.data_ptr(), s)
        call("ppo_heads_reduce", part_w.data_ptr(), part_b.data_ptr(), part_l.data_ptr(), nblk, H, A,
             self.gv(self.WC), self.gv(self.BC), self.gv(self.WA), self.gv(self.BA), loss_acc.data_ptr(), inv_b, 1.0,
             int(hp["use_clipped_value_loss"]), s)

    def _trunk_backward(self, B, dh, obs, idx):
        """dh: dL/d(fc pre-activation) [B,H] (ReLU mask applied) -> trunk gradients."""
        ws, dev, s = self.ws["train"], self.device, stream()
        a1 = ws.bufs["a1"]
        a2, a3 = ws.bufs["a2"], ws.bufs["a3"]
        dz3 = ws.get("dz3", B * FEAT, device=dev)
        dz2 = ws.get("dz2", B * 81 * 64, device=dev)
        dz1 = ws.get("dz1", B * 400 * 32, device=dev)
        bits = getattr(self, "_mask_rows", None) == B   # masks of this minibatch's forward
        if bits:
            call("ppo_fc_dgrad_bits", dh.data_ptr(), B, self.H, self.pk(3), ws.bufs["m3bits"].data_ptr(),
                 dz3.data_ptr(), s)
        else:
            call("ppo_linear_dgrad_mask", dh.data_ptr(), B, self.H, self.pk(3), FEAT, a3.data_ptr(), dz3.data_ptr(),
                 s)
        self._wgrad("fc", B, dh, a3, None, s)
        # the fc + heads tail of the flat gradient (the last parameters in torch order,
        # 92 % of the bytes at H = 512) is final here: its all-reduce (G > 1) overlaps
        # the conv backward on a side stream (_dist.start_bucket); PPO's step waits for it
        _dist.start_bucket(self.grad[self.offsets[self.W4]:])
        if bits:
            call("ppo_conv3_dgrad_bits", dz3.data_ptr(), B, self.pk(4), ws.bufs["m2bits"].data_ptr(), dz2.data_ptr(),
                 s)
        else:
            call("ppo_conv3_dgrad", dz3.data_ptr(), B, self.pk(4), a2.data_ptr(), dz2.data_ptr(), s)
        self._wgrad("conv3", B, dz3, a2, None, s)
        if bits:
            call("ppo_conv2_dgrad_bits", dz2.data_ptr(), B, self.pk(5), ws.bufs["m1bits"].data_ptr(), dz1.data_ptr(),
                 s)
        else:
            call("ppo_conv2_dgrad", dz2.data_ptr(), B, self.pk(5), a1.data_ptr(), dz1.data_ptr(), s)
        self._wgrad("conv2", B, dz2, a1, None, s)
        if obs.dtype == torch.float16:   # the rows trunk() converted for this minibatch
            obs, idx = ws.bufs["obs32"], None
        self._wgrad("conv1", B, dz1, obs, idx, s)

    def _finish_step(self, optimizer):
        optimizer._step_flat(self)
        self.epoch += 1
        self.pack(force=True)

    @_with_precision
    def train_minibatch(self, storage, adv, idx, hp, loss_acc, optimizer):
        """Forward + backward + (all-reduce) + clip + Adam for one minibatch of
        storage rows idx (int64 [B], device)."""
        self.ensure_bound()
        self.pack()
        _dist.begin_minibatch()
        B = idx.numel()
        ws = self.ws["train"]
        h = self.trunk(storage.obs, idx, B, ws)
        dh = ws.get("dh", B * self.H, device=self.device)
        self._heads_train(storage, adv, idx, h, B, hp, loss_acc, dh, feat_act=1)
        self._trunk_backward(B, dh, storage.obs, idx)
        self._finish_step(optimizer)

    def _wgrad(self, layer, B, dz, x, idx, s):
        dev = self.device
        ws = self.ws["train"]
        if layer == "conv1":
            M, NW, kind, ka, kb, wi, bi, R, tiles = 32, self.C * 64, 0, 0, 0, self.W1, self.B1, B * 400, 1
        elif layer == "conv2":
            M, NW, kind, ka, kb, wi, bi, R, tiles = 64, 512, 1, 4, 32, self.W2, self.B2, B * 81, 4
        elif layer == "conv3":
            M, NW, kind, ka, kb, wi, bi, R, tiles = 32, 576, 1, 3, 64, self.W3, self.B3, B * 49, 5
        else:
            M, NW, kind, ka, kb, wi, bi, R, tiles = self.H, FEAT, 2, 32, 49, self.W4, self.B4, B, \
                ((self.H + 127) // 128) * 13
        # the image-resident conv wgrad kernels walk any number of images per block:
        # one block per CU (their LDS allows no more) — measured conv3 0.80 -> 0.70 ms,
        # conv1 / conv2 -1 %, and 2-8x fewer split-K slabs to reduce
        if self._n_cu is None:
            self._n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count
        target = max(self._n_cu, -(-B // 512)) * tiles if layer in ("conv1", "conv2", "conv3") else 2048
        Z = call("ppo_wgrad_splits", R, tiles, target, 16)
        slab = ws.get("slab", Z * M * NW, device=dev)
        slab_b = ws.get("slab_b", Z * M, device=dev)
        if layer == "conv1" and self._is_rgb(x):
            mean, std = self.obs_decode
            call("ppo_conv1_wgrad_rgb", dz.data_ptr(), x.data_ptr(), ptr(idx), 0, B, ptr(mean), std, Z,
                 slab.data_ptr(), slab_b.data_ptr(), s)
        elif layer == "conv1":
            call("ppo_conv1_wgrad", dz.data_ptr(), x.data_ptr(), self._obs_args(x), ptr(idx), 0, self.C, B, Z,
                 slab.data_ptr(), slab_b.data_ptr(), s)
        elif layer == "conv2":
            call("ppo_conv2_wgrad", dz.data_ptr(), x.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        elif layer == "conv3":
            call("ppo_conv3_wgrad", dz.data_ptr(), x.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        else:
            call("ppo_linear_wgrad", dz.data_ptr(), x.data_ptr(), B, self.H, FEAT, Z, slab.data_ptr(),
                 slab_b.data_ptr(), s)
        # u8 4-channel observations are staged as integers (1/255 in the reduce); RGB frames are decoded to fp32
        scale = 1.0 / 255.0 if layer == "conv1" and x.dtype == torch.uint8 and not self._is_rgb(x) else 1.0
        call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, M, NW, kind, ka, kb, self.gv(wi), self.gv(bi),
             scale, 0, s)

    def _dense_wgrad(self, dy, x, R, N, K, kind, a, wi, bi):
        """dW[n][k] = Σ_r dy[r][n] x[r][k] (+ bias) -> grad planes wi, bi"""
        ws, dev, s = self.ws["train"], self.device, stream()
        tiles = ((N + 127) // 128) * ((K + 127) // 128)
        Z = call("ppo_wgrad_splits", R, tiles, 2048, 16)
        slab = ws.get("slab", Z * N * K, device=dev)
        slab_b = ws.get("slab_b", Z * N, device=dev)
        call("ppo_linear_wgrad", dy.data_ptr(), x.data_ptr(), R, N, K, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, N, K, kind, a, 0, self.gv(wi), self.gv(bi),
             1.0, 0, s)


class RecurrentEngine(CNNEngine):
    """CNNBase(recurrent=True) + vector obs: x = cat(fc(obs), vec) -> GRU -> heads.
    Parameter order: gru.{weight_ih, weight_hh, bias_ih, bias_hh}, main.*, critic, dist."""

    GIH, GHH, GBI, GBH = range(4)
    W1, B1, W2, B2, W3, B3, W4, B4, WC, BC, WA, BA = range(4, 16)
    recurrent = True

    def __init__(self, policy, device):
        gru = policy.base.gru
        self.V = policy.base.vector_obs_len
        H = policy.base.main[7].weight.shape[0]
        self.I = H + self.V
        self.Ip = (self.I + 3) // 4 * 4   # GEMM rows padded to 16-B multiples
        if gru.weight_ih_l0.shape != (3 * H, self.I) or H % 32 != 0:
            raise NotImplementedError("GRU engine needs hidden_size a multiple of 32 (<= 512)")
        self.gru_packed = None
        super().__init__(policy, device)

    def _pack_extra(self):
        H, Ip = self.H, self.Ip
        if self.gru_packed is None:
            self.gru_packed = torch.empty(3 * H * Ip + 6 * H * H, device=self.device)
        gp = self.gru_packed.data_ptr()
        self.wih_pad, self.wihT, self.whhT = gp, gp + 4 * 3 * H * Ip, gp + 4 * (3 * H * Ip + 3 * H * H)
        call("ppo_gru_pack", self.pv(self.GIH), self.pv(self.GHH), H, self.I, Ip, self.wih_pad, self.wihT, self.whhT,
             stream())

    def _input(self, obs, vec, idx, B, ws, rows_vec=None):
        """x_pad [B][Ip] = (fc(obs) | vector obs | 0-pad) and gi = x·W_ihᵀ + b_ih [B][3H]."""
        dev, s, H, Ip = self.device, stream(), self.H, self.Ip
        x = ws.get("xpad", B * Ip, device=dev)
        self.trunk(obs, idx, B, ws, out=x, ldo=Ip)
        if Ip > H:
            src = vec if vec is not None else x   # V == 0: only the zero pad is written
            call("ppo_concat_cols", src.data_ptr(), ptr(rows_vec), B, self.V if vec is not None else 0,
                 x.data_ptr(), Ip, H, Ip - H, s)
        gi = ws.get("gi", B * 3 * H, device=dev)
        call("ppo_linear_fwd_ex", x.data_ptr(), None, B, Ip, Ip, self.wih_pad, self.pv(self.GBI), 3 * H,
             gi.data_ptr(), 3 * H, 0, s)
        return x, gi

    def _vec(self, vec, B):
        if self.V == 0:
            return None
        return vec.to(self.device, torch.float32).reshape(B, self.V).contiguous()

    @_with_precision
    def act(self, obs, deterministic=False, noise=None, given=None, want_entropy=False, value_only=False,
            vec=None, hxs=None, masks=None):
        """Single step (model.py:112-115): returns (value, action, logp, entropy, hxs')."""
        self.ensure_bound()
        self.pack()
        obs = self._check_obs(obs)
        B = obs.shape[0]
        ws = self.ws[self.act_ws]
        _, gi = self._input(obs, self._vec(vec, B), None, B, ws)
        hxs = hxs.to(self.device, torch.float32).reshape(B, self.H).contiguous()
        m = masks.to(self.device, torch.float32).reshape(B).contiguous() if masks is not None else None
        hout = torch.empty(B, self.H, device=self.device)
        call("ppo_gru_step_fwd", hxs.data_ptr(), ptr(m), None, self.pv(self.GHH), self.pv(self.GBH), gi.data_ptr(),
             B, self.H, hout.data_ptr(), None, None, None, None, None, stream())
        value, action, logp, ent = self._heads(hout, B, deterministic, noise, given, want_entropy, value_only)
        return value, action, logp, ent, hout

    @_with_precision
    def evaluate_sequence(self, obs, vec, hxs, masks, action):
        """Multi-step branch (model.py:116-165): rows are t*N + n."""
        self.ensure_bound()
        self.pack()
        obs = self._check_obs(obs)
        R = obs.shape[0]
        N = hxs.shape[0]
        T = R // N
        ws = self.ws[self.act_ws]
        _, gi = self._input(obs, self._vec(vec, R), None, R, ws)
        hxs = hxs.to(self.device, torch.float32).reshape(N, self.H).contiguous()
        m = masks.to(self.device, torch.float32).reshape(R).contiguous()
        hout = torch.empty(R, self.H, device=self.device)
        H, s = self.H, stream()
        cnt = ws.get("gru_cnt", call("ppo_gru_seq_counters", N), torch.int32, self.device)
        call("ppo_gru_seq_fwd_ws", hxs.data_ptr(), m.data_ptr(), None, self.pv(self.GHH), self.pv(self.GBH),
             gi.data_ptr(), T, N, H, hout.data_ptr(), None, None, None, None, None, cnt.data_ptr(), self.status_ptr(2),
             s)
        if int(self.status[2].item()):   # stream-ordered read of the launch's error word
            self.status[2].zero_()
            raise RuntimeError("evaluate_actions: the persistent GRU kernel timed out (its outputs are invalid; "
                               "ppo_gru_persist_set(0) selects the per-step launches)")
        value, _, logp, ent = self._heads(hout, R, given=action.to(self.device, torch.int64), want_entropy=True)
        return value, logp, ent, hout[(T - 1) * N:]

    @_with_precision
    def train_minibatch_rec(self, storage, adv, envs, hp, loss_acc, optimizer):
        """recurrent_generator minibatch (storage.py:162-223): whole T-sequences of
        the n envs `envs` (int64 device), BPTT over the full T, then one Adam step."""
        self.ensure_bound()
        self.pack()
        _dist.begin_minibatch()
        dev, H, s = self.device, self.H, stream()
        T, N, n = storage.num_steps, storage.rewards.shape[1], envs.numel()
        R = T * n
        ws = self.ws["train"]
        idx = ws.get("ridx", R, torch.int64, dev)[:R]
        call("ppo_rec_indices", envs.data_ptr(), n, T, N, idx.data_ptr(), s)
        h0 = ws.get("h0", n * H, device=dev)
        call("ppo_gather_rows", storage.recurrent_hidden_states.data_ptr(), envs.data_ptr(), h0.data_ptr(), n,
             4 * H, s)
        vec = storage.vector_obs if self.V else None
        x, gi = self._input(storage.obs, vec, idx, R, ws, rows_vec=idx if self.V else None)
        hout = ws.get("hout", R * H, device=dev)
        sv = {k: ws.get("s_" + k, R * H, device=dev) for k in ("r", "z", "n", "ghn", "hin")}
        masks = storage.masks
        cnt = ws.get("gru_cnt", call("ppo_gru_seq_counters", n), torch.int32, dev)
        # error word status[0]: sticky for the update, gates every clip + Adam after a timeout;
        # no gradient bucket may still be reducing on a side stream beside the persistent launch
        _dist.assert_no_pending("train_minibatch_rec")
        call("ppo_gru_seq_fwd_ws", h0.data_ptr(), masks.data_ptr(), idx.data_ptr(), self.pv(self.GHH),
             self.pv(self.GBH), gi.data_ptr(), T, n, H, hout.data_ptr(), sv["r"].data_ptr(), sv["z"].data_ptr(),
             sv["n"].data_ptr(), sv["ghn"].data_ptr(), sv["hin"].data_ptr(), cnt.data_ptr(), self.status_ptr(0), s)
        dout = ws.get("dout", R * H, device=dev)
        self._heads_train(storage, adv, idx, hout, R, hp, loss_acc, dout, feat_act=0)
        # backward through time
        dgi = ws.get("dgi", R * 3 * H, device=dev)
        dgh = ws.get("dgh", R * 3 * H, device=dev)
        dhz = ws.get("dhz", n * H, device=dev)
        carry = ws.get("carry", n * H, device=dev)
        # persistent BPTT on the same counters (the forward has finished on this stream) and error word
        _dist.assert_no_pending("train_minibatch_rec bptt")
        call("ppo_gru_seq_bwd_ws", dout.data_ptr(), sv["r"].data_ptr(), sv["z"].data_ptr(), sv["n"].data_ptr(),
             sv["ghn"].data_ptr(), sv["hin"].data_ptr(), masks.data_ptr(), idx.data_ptr(), self.whhT, T, n, H,
             dgi.data_ptr(), dgh.data_ptr(), dhz.data_ptr(), carry.data_ptr(), cnt.data_ptr(), self.status_ptr(0), s)
        self._dense_wgrad(dgh, sv["hin"], R, 3 * H, H, 0, 0, self.GHH, self.GBH)
        self._dense_wgrad(dgi, x, R, 3 * H, self.Ip, 3, self.I, self.GIH, self.GBI)
        dh = ws.get("dh", R * H, device=dev)
        call("ppo_linear_dgrad_ex", dgi.data_ptr(), R, 3 * H, self.wihT, H, x.data_ptr(), self.Ip, 1, dh.data_ptr(),
             s)
        self._trunk_backward(R, dh, storage.obs, idx)
        self._finish_step(optimizer)


class MLPEngine(CNNEngine):
    """MLPBase (model.py:202-234): actor / critic towers Linear-tanh-Linear-tanh on
    x = cat(obs, vector_obs); value from the critic tower, logits from the actor's.
    Parameter order: actor.0, actor.2, critic.0, critic.2, critic_linear, dist."""

    AW1, AB1, AW2, AB2, CW1, CB1, CW2, CB2, WC, BC, WA, BA = range(12)

    def __init__(self, policy, device):   # noqa: D401 — own init, shares the CNNEngine machinery
        base = policy.base
        if base.is_recurrent:
            raise NotImplementedError("recurrent MLPBase is not on the HIP path")
        self.policy, self.device = policy, device
        self.H = base._hidden_size
        self.I = base.actor[0].weight.shape[1]
        self.V = base.vector_obs_len
        self.obs_dim = self.I - self.V
        self.Ip = (self.I + 3) // 4 * 4
        self.A = policy.dist.linear.weight.shape[0]
        if self.H % 4 != 0 or self.H > 512:
            raise NotImplementedError(f"MLPBase hidden_size {self.H}: multiples of 4 up to 512")
        self.params = list(policy.parameters())
        self.ws = {"act": _Workspace(), "train": _Workspace()}
        self.act_ws = "act"
        self.packed = None
        self._pack_key = None
        self.epoch = 0
        self._flatten()
        self.rng_seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        self.rng_counter = 0
        self._init_status()

    def pack(self, force=False):
        key = (sum(p._version for p in self.params), self.epoch)
        if not force and self.packed is not None and key == self._pack_key:
            return
        H, Ip, s = self.H, self.Ip, stream()
        if self.packed is None:
            self.packed = torch.empty(2 * H * Ip + 2 * H * H, device=self.device)
        b = self.packed.data_ptr()
        self.aw1, self.cw1 = b, b + 4 * H * Ip
        self.aw2T, self.cw2T = b + 8 * H * Ip, b + 8 * H * Ip + 4 * H * H
        for w, dst in ((self.AW1, self.aw1), (self.CW1, self.cw1)):   # first layers padded to Ip inputs
            call("ppo_concat_cols", self.pv(w), None, H, self.I, dst, Ip, 0, Ip, s)
        call("ppo_transpose", self.pv(self.AW2), H, H, self.aw2T, s)
        call("ppo_transpose", self.pv(self.CW2), H, H, self.cw2T, s)
        self._pack_key = key

    def _x(self, obs, vec, idx, B, ws):
        """x_pad [B][Ip] = (obs | vector obs | 0)"""
        dev, s = self.device, stream()
        x = ws.get("x", B * self.Ip, device=dev)
        call("ppo_concat_cols", obs.data_ptr(), ptr(idx), B, self.obs_dim, x.data_ptr(), self.Ip, 0,
             self.obs_dim if self.V else self.Ip, s)
        if self.V:
            call("ppo_concat_cols", vec.data_ptr(), ptr(idx), B, self.V, x.data_ptr(), self.Ip, self.obs_dim,
                 self.Ip - self.obs_dim, s)
        return x

    def towers(self, x, B, ws):
        dev, H, Ip, s = self.device, self.H, self.Ip, stream()
        out = {}
        for name, w1, b1, w2, b2 in (("a", self.aw1, self.AB1, self.AW2, self.AB2),
                                     ("c", self.cw1, self.CB1, self.CW2, self.CB2)):
            h1 = ws.get(name + "1", B * H, device=dev)
            h2 = ws.get(name + "2", B * H, device=dev)
            call("ppo_linear_fwd_ex", x.data_ptr(), None, B, Ip, Ip, w1, self.pv(b1), H, h1.data_ptr(), H, 2, s)
            call("ppo_linear_fwd_ex", h1.data_ptr(), None, B, H, H, self.pv(w2), self.pv(b2), H, h2.data_ptr(), H, 2, s)
            out[name] = (h1, h2)
        return out

    @_with_precision
    def act(self, obs, deterministic=False, noise=None, given=None, want_entropy=False, value_only=False, vec=None):
        self.ensure_bound()
        self.pack()
        obs = (obs if obs.is_cuda else obs.to(self.device)).to(torch.float32).reshape(obs.shape[0], -1).contiguous()
        B = obs.shape[0]
        if obs.shape[1] != self.obs_dim:
            raise RuntimeError(f"MLPBase expects [N,{self.obs_dim}] observations, got {tuple(obs.shape)}")
        ws = self.ws[self.act_ws]
        v = vec.to(self.device, torch.float32).reshape(B, self.V).contiguous() if self.V else None
        x = self._x(obs, v, None, B, ws)
        t = self.towers(x, B, ws)
        return self._heads(t["a"][1], B, deterministic, noise, given, want_entropy, value_only, hv=t["c"][1])

    @_with_precision
    def train_minibatch(self, storage, adv, idx, hp, loss_acc, optimizer):
        self.ensure_bound()
        self.pack()
        _dist.begin_minibatch()
        dev, H, B = self.device, self.H, idx.numel()
        ws = self.ws["train"]
        x = self._x(storage.obs, storage.vector_obs if self.V else None, idx, B, ws)
        t = self.towers(x, B, ws)
        da2 = ws.get("da2", B * H, device=dev)
        dc2 = ws.get("dc2", B * H, device=dev)
        self._heads_train(storage, adv, idx, t["a"][1], B, hp, loss_acc, da2, feat_act=2, feat_v=t["c"][1],
                          dfeat_v=dc2)
        for name, d2, w1, b1, w2, b2, w2T in (("a", da2, self.AW1, self.AB1, self.AW2, self.AB2, self.aw2T),
                                               ("c", dc2, self.CW1, self.CB1, self.CW2, self.CB2, self.cw2T)):
            h1 = t[name][0]
            self._dense_wgrad(d2, h1, B, H, H, 0, 0, w2, b2)
            d1 = ws.get("d1" + name, B * H, device=dev)
            call("ppo_linear_dgrad_ex", d2.data_ptr(), B, H, w2T, H, h1.data_ptr(), H, 2, d1.data_ptr(), stream())
            self._dense_wgrad(d1, x, B, H, self.Ip, 3, self.I, w1, b1)
        self._finish_step(optimizer)
