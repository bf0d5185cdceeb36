"""HIP execution engine behind Policy / PPO (CNNBase, feed-forward).

Owns the flat parameter / gradient buffers (every nn.Parameter of the Policy is
re-pointed to a view of one contiguous fp32 buffer, so clip + Adam is one pass),
the per-step packed weight copies, and grow-only activation workspaces.

Call sequence per PPO minibatch (every box is a libppo_hip.so kernel):
  conv1(obs rows gathered by index, u8 decode) -> conv2 -> conv3 -> fc        (MFMA fwd)
  heads_train (value/logits/Categorical/PPO loss + dL/dlogits, dL/dfeat)    (fused)
  fc dgrad | fc wgrad | conv3 dgrad | conv3 wgrad | conv2 dgrad | conv2 wgrad | conv1 wgrad  (MFMA bwd)
  wgrad slab reduces -> flat grad  [RCCL all-reduce when world_size > 1]
  grad Σg² -> clip + Adam -> pack weights
"""
import torch

from ._hip import call, ptr, stream

FEAT = 32 * 7 * 7  # conv3 output, flattened


class _Workspace:
    def __init__(self):
        self.bufs = {}

    def get(self, name, numel, dtype=torch.float32, device=None):
        t = self.bufs.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype or t.device != device:
            t = torch.empty(max(int(numel), 1), dtype=dtype, device=device)
            self.bufs[name] = t
        return t


class CNNEngine:
    """Binds to a Policy whose base is CNNBase (non-recurrent)."""

    def __init__(self, policy, device):
        self.policy = policy
        self.device = device
        base = policy.base
        self.C = base.main[0].weight.shape[1]
        self.H = base.main[7].weight.shape[0]
        self.A = policy.dist.linear.weight.shape[0]
        if self.H % 64 != 0:
            raise NotImplementedError(f"hidden_size {self.H}: the HIP heads need a multiple of 64 (64..512)")
        if base.critic_linear.weight.shape[1] != self.H:
            raise NotImplementedError("vector observations with a non-recurrent CNNBase are not supported "
                                      "(the reference crashes there too: Categorical expects hidden_size inputs)")
        self.params = list(policy.parameters())
        self.ws = {"act": _Workspace(), "train": _Workspace()}
        self.packed = None
        self._pack_key = None
        self.epoch = 0  # bumped by every in-place parameter write done by HIP kernels
        self._flatten()
        self.rng_seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        self.rng_counter = 0

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

    def is_bound(self):
        if self.flat is None:
            return False
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

    # parameter indices (CNNBase non-recurrent, named_parameters order)
    W1, B1, W2, B2, W3, B3, W4, B4, WC, BC, WA, BA = range(12)

    def pack(self, force=False):
        key = (sum(p._version for p in self.params), self.epoch)
        if not force and self.packed is not None and key == self._pack_key:
            return
        if self.packed is None:
            self.packed = torch.empty(call("ppo_packed_weights_size", self.H), device=self.device)
            offs = (torch.zeros(6, dtype=torch.int64))
            call("ppo_packed_offsets", self.H, offs.data_ptr())
            self.poff = [int(x) for x in offs]
        call("ppo_pack_weights", self.pv(self.W2), self.pv(self.W3), self.pv(self.W4), self.H,
             self.packed.data_ptr(), stream())
        self._pack_key = key

    def pk(self, seg):
        """pointer to packed segment: 0 W2p 1 W3p 2 W4p 3 W4T 4 W3d 5 W2d"""
        return self.packed.data_ptr() + 4 * self.poff[seg]

    # ---------------------------------------------------------------- forward
    def _obs_args(self, obs):
        if obs.dtype == torch.uint8:
            return 1
        if obs.dtype == torch.float32:
            return 0
        raise TypeError(f"observations must be uint8 or float32, got {obs.dtype}")

    def trunk(self, obs, idx, B, ws):
        """conv1..fc on B samples: obs is either a [B,C,84,84] batch (idx None) or the
        storage plane whose rows idx[b] are gathered inside conv1.  Returns feat [B,H]."""
        dev = self.device
        is_u8 = self._obs_args(obs)
        a1 = ws.get("a1", B * 400 * 32, device=dev)
        a2 = ws.get("a2", B * 81 * 64, device=dev)
        a3 = ws.get("a3", B * FEAT, device=dev)
        h = ws.get("h", B * self.H, device=dev)
        s = stream()
        call("ppo_conv1_fwd", obs.data_ptr(), is_u8, ptr(idx, torch.int64, "idx"), 0, self.C, B, self.pv(self.W1),
             self.pv(self.B1), a1.data_ptr(), s)
        call("ppo_conv2_fwd", a1.data_ptr(), B, self.pk(0), self.pv(self.B2), a2.data_ptr(), s)
        call("ppo_conv3_fwd", a2.data_ptr(), B, self.pk(1), self.pv(self.B3), a3.data_ptr(), s)
        call("ppo_linear_relu_fwd", a3.data_ptr(), B, FEAT, self.pk(2), self.pv(self.B4), self.H, h.data_ptr(), s)
        return h

    def _check_obs(self, obs):
        obs = obs if obs.is_cuda else obs.to(self.device)
        if tuple(obs.shape[1:]) != (self.C, 84, 84):
            raise RuntimeError(f"CNNBase expects [N,{self.C},84,84] observations, got {tuple(obs.shape)}")
        return obs.contiguous()

    def act(self, obs, deterministic=False, noise=None, given=None, want_entropy=False, value_only=False):
        self.ensure_bound()
        self.pack()
        obs = self._check_obs(obs)
        B = obs.shape[0]
        ws = self.ws["act"]
        h = self.trunk(obs, None, B, ws)
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
        call("ppo_heads_act", h.data_ptr(), B, self.H, self.pv(self.WC), self.pv(self.BC), self.pv(self.WA),
             self.pv(self.BA), self.A, ptr(noise), self.rng_seed, self.rng_counter, int(bool(deterministic)),
             ptr(given.reshape(-1).contiguous() if given is not None else None, torch.int64, "action"),
             value.data_ptr(), None if given is not None or value_only else action.data_ptr(),
             ptr(logp), ptr(ent), stream())
        return value, action, logp, ent

    # --------------------------------------------------------------- training
    def train_minibatch(self, storage, adv, idx, hp, loss_acc, optimizer):
        """Forward + backward + (all-reduce) + clip + Adam for one minibatch of
        storage rows idx (int64 [B], device)."""
        self.ensure_bound()
        self.pack()
        dev, H, A = self.device, self.H, self.A
        B = idx.numel()
        ws = self.ws["train"]
        s = stream()
        obs = storage.obs
        h = self.trunk(obs, idx, B, ws)
        a1, a2, a3 = ws.bufs["a1"], ws.bufs["a2"], ws.bufs["a3"]
        nblk = call("ppo_heads_train_blocks", B)
        dh = ws.get("dh", B * H, device=dev)
        part_w = ws.get("part_w", nblk * (1 + A) * H, device=dev)
        part_b = ws.get("part_b", nblk * (1 + A), device=dev)
        part_l = ws.get("part_l", nblk * 3, device=dev)
        inv_b = 1.0 / B
        call("ppo_heads_train", h.data_ptr(), B, H, self.pv(self.WC), self.pv(self.BC), self.pv(self.WA),
             self.pv(self.BA), A, idx.data_ptr(), 0, storage.actions.data_ptr(), storage.action_log_probs.data_ptr(),
             adv.data_ptr(), storage.value_preds.data_ptr(), storage.returns.data_ptr(), hp["clip"], hp["value_coef"],
             hp["entropy_coef"], inv_b, int(hp["use_clipped_value_loss"]), dh.data_ptr(), part_w.data_ptr(),
             part_b.data_ptr(), part_l.data_ptr(), s)
        call("ppo_heads_reduce", part_w.data_ptr(), part_b.data_ptr(), part_l.data_ptr(), nblk, H, A,
             self.gv(self.WC), self.gv(self.BC), self.gv(self.WA), self.gv(self.BA), loss_acc.data_ptr(), inv_b, 1.0,
             int(hp["use_clipped_value_loss"]), s)
        dz3 = ws.get("dz3", B * FEAT, device=dev)
        dz2 = ws.get("dz2", B * 81 * 64, device=dev)
        dz1 = ws.get("dz1", B * 400 * 32, device=dev)
        # fc
        call("ppo_linear_dgrad_mask", dh.data_ptr(), B, H, self.pk(3), FEAT, a3.data_ptr(), dz3.data_ptr(), s)
        self._wgrad("fc", B, dh, a3, None, s)
        # conv3
        call("ppo_conv3_dgrad", dz3.data_ptr(), B, self.pk(4), a2.data_ptr(), dz2.data_ptr(), s)
        self._wgrad("conv3", B, dz3, a2, None, s)
        # conv2
        call("ppo_conv2_dgrad", dz2.data_ptr(), B, self.pk(5), a1.data_ptr(), dz1.data_ptr(), s)
        self._wgrad("conv2", B, dz2, a1, None, s)
        # conv1 (weights only)
        self._wgrad("conv1", B, dz1, obs, idx, s)
        optimizer._step_flat(self)
        self.epoch += 1
        self.pack(force=True)

    # wgrad layer table: (M rows, NW cols, reduce kind, a, b, w index, b index, tiles)
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
        Z = call("ppo_wgrad_splits", R, tiles, 2048, 16)
        slab = ws.get("slab", Z * M * NW, device=dev)
        slab_b = ws.get("slab_b", Z * M, device=dev)
        if layer == "conv1":
            call("ppo_conv1_wgrad", dz.data_ptr(), x.data_ptr(), self._obs_args(x), ptr(idx), 0, self.C, B, Z,
                 slab.data_ptr(), slab_b.data_ptr(), s)
        elif layer == "conv2":
            call("ppo_conv2_wgrad", dz.data_ptr(), x.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        elif layer == "conv3":
            call("ppo_conv3_wgrad", dz.data_ptr(), x.data_ptr(), B, Z, slab.data_ptr(), slab_b.data_ptr(), s)
        else:
            call("ppo_linear_wgrad", dz.data_ptr(), x.data_ptr(), B, self.H, FEAT, Z, slab.data_ptr(),
                 slab_b.data_ptr(), s)
        scale = 1.0 / 255.0 if layer == "conv1" and x.dtype == torch.uint8 else 1.0   # u8 staged as integers
        call("ppo_wgrad_reduce", slab.data_ptr(), slab_b.data_ptr(), Z, M, NW, kind, ka, kb, self.gv(wi), self.gv(bi),
             scale, 0, s)
