"""PPO — drop-in for a2c_ppo_acktr/algo/ppo.py (reference
ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/algo/ppo.py:7-96).

update(rollouts) keeps the reference's semantics — advantages normalised over
all T*N samples (:35-37), ppo_epoch passes of num_mini_batch minibatches cut
from torch.randperm on the default CPU generator (:43-51, bit-identical index
sets), clipped surrogate + clipped value loss + entropy (:61-81),
clip_grad_norm_ + Adam (:82-84), mean losses returned as floats (:86-96) —
but each minibatch is one fused HIP pipeline with no autograd: the obs rows
are gathered inside conv1, the loss gradient is analytic, and the losses are
accumulated on the device (one device->host copy per update instead of three
per minibatch).

Multi-GPU (new; the reference's PPO path has no collectives):
with torch.distributed initialised each rank owns its own env lanes and
storage; per update one 3-double all-reduce makes the advantage statistics
global, per minibatch one all-reduce (RCCL over xGMI) sums the flat gradient,
and clip + Adam run on the averaged gradient so all ranks stay identical.
"""
import torch

from .. import _dist
from .._hip import call, stream


class FlatAdam(object):
    """torch.optim.Adam-compatible façade over one flat parameter buffer.
    param_groups[0]['lr'] is read at every step (utils.update_linear_schedule)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, max_grad_norm=None):
        self.param_groups = [{"params": list(params), "lr": lr, "betas": betas, "eps": eps, "weight_decay": 0,
                              "amsgrad": False}]
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self.exp_avg = None
        self.exp_avg_sq = None
        self._partials = None
        self.last_grad_norm = None
        self._norm = None
        # (int32 [1] error word, float64 [1] bad-action count, int* skipped-step count)
        # set by PPO.update: a guarded step is skipped on the device (on every rank
        # when any rank's guard is set, _dist.global_guard)
        self.guard = None
        self._gflag = None

    def zero_grad(self, set_to_none=False):
        for p in self.param_groups[0]["params"]:
            if p.grad is not None:
                p.grad.zero_()

    def _step_flat(self, eng):
        """all-reduce (G>1) -> Σg² partials -> fused clip + Adam on eng.flat."""
        n = eng.numel
        if self.exp_avg is None:
            self.exp_avg = torch.zeros(n, device=eng.device)
            self.exp_avg_sq = torch.zeros(n, device=eng.device)
        elif self.exp_avg.numel() != n or self.exp_avg_sq is None or self.exp_avg_sq.numel() != n:
            raise RuntimeError(f"Adam state holds {self.exp_avg.numel()} moments for {n} parameters "
                               "(optimizer state of a different policy?)")
        elif self.exp_avg.device != eng.device or self.exp_avg_sq.device != eng.device:
            # restored on another device (e.g. a checkpoint loaded before .to(device)):
            # keep the moments — step_count's bias correction assumes them
            self.exp_avg = self.exp_avg.to(eng.device, torch.float32).contiguous()
            self.exp_avg_sq = self.exp_avg_sq.to(eng.device, torch.float32).contiguous()
        if self._partials is None or self._partials.device != eng.device:   # also after load_state_dict
            self._partials = torch.empty(call("ppo_grad_partials_count", n), dtype=torch.float64, device=eng.device)
            self._norm = torch.zeros(1, dtype=torch.float64, device=eng.device)
        scale = _dist.allreduce_grads(eng.grad)   # (waits for the fc + heads bucket the backward started)
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        self.step_count += 1
        s = stream()
        call("ppo_grad_sumsq", eng.grad.data_ptr(), n, scale, self._partials.data_ptr(), s)
        mn = self.max_grad_norm if self.max_grad_norm is not None else -1.0
        gi = gd = sk = None
        if self.guard is not None:
            err, bad, sk = self.guard
            if _dist.active():
                # the gradient is already summed over ranks: any rank's failure skips the
                # step on every rank (one 8-byte all-reduce), so all ranks stay identical
                if self._gflag is None or self._gflag.device != eng.device:
                    self._gflag = torch.zeros(1, dtype=torch.float64, device=eng.device)
                gd = _dist.global_guard(err, bad, self._gflag).data_ptr()
            else:
                gi, gd = err.data_ptr(), bad.data_ptr()
        call("ppo_clip_adam_guarded", eng.flat.data_ptr(), eng.grad.data_ptr(), self.exp_avg.data_ptr(),
             self.exp_avg_sq.data_ptr(), n, self._partials.data_ptr(), scale, float(mn), float(g["lr"]),
             float(b1), float(b2), float(g["eps"]), self.step_count, self._norm.data_ptr(), gi, gd, sk, s)

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "param_groups": [{k: v for k, v in self.param_groups[0].items() if k != "params"}]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg = sd["exp_avg"]
        self.exp_avg_sq = sd["exp_avg_sq"]
        self.param_groups[0].update(sd["param_groups"][0])


class PPO():
    def __init__(self,
                 actor_critic,
                 clip_param,
                 ppo_epoch,
                 num_mini_batch,
                 value_loss_coef,
                 entropy_coef,
                 lr=None,
                 eps=None,
                 max_grad_norm=None,
                 use_clipped_value_loss=True):
        self.actor_critic = actor_critic
        self.clip_param = clip_param
        self.ppo_epoch = ppo_epoch
        self.num_mini_batch = num_mini_batch
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.optimizer = FlatAdam(actor_critic.parameters(), lr=lr, eps=eps, max_grad_norm=max_grad_norm)
        self._loss_acc = None
        if _dist.active():
            # one-time parameter broadcast so every rank starts from rank 0's weights
            eng = actor_critic.hip_engine()
            _dist.broadcast_params(eng.flat)
            eng.epoch += 1

    def update(self, rollouts):
        eng = self.actor_critic.hip_engine()
        advantages = rollouts.normalized_advantages()            # ppo.py:35-37
        if self._loss_acc is None or self._loss_acc.device != eng.device:
            # {value loss, action loss, entropy} sums, the count of stored actions outside
            # [0, A), and (filled at the end) the persistent-GRU timeout flag
            self._loss_acc = torch.zeros(5, dtype=torch.float64, device=eng.device)
        else:
            self._loss_acc.zero_()
        # device guards of every clip + Adam of this update: a persistent-GRU timeout
        # (status[0]) or an out-of-range stored action (loss_acc[3]) turns the step
        # into a no-op on the device, counted in status[1]; _losses() raises
        eng.status[:2].zero_()
        self.optimizer.guard = (eng.status[0:1], self._loss_acc[3:4], eng.status_ptr(1))
        hp = {"clip": float(self.clip_param), "value_coef": float(self.value_loss_coef),
              "entropy_coef": float(self.entropy_coef), "use_clipped_value_loss": bool(self.use_clipped_value_loss)}
        num_steps, num_processes = rollouts.rewards.size()[0:2]
        if self.actor_critic.is_recurrent:
            self._update_recurrent(eng, rollouts, advantages, hp, num_processes)
            return self._losses()
        batch_size = num_processes * num_steps
        assert batch_size >= self.num_mini_batch, (
            "PPO requires the number of processes ({}) "
            "* number of steps ({}) = {} "
            "to be greater than or equal to the number of PPO mini batches ({})."
            "".format(num_processes, num_steps, batch_size, self.num_mini_batch))
        mini_batch_size = batch_size // self.num_mini_batch
        for e in range(self.ppo_epoch):
            # SubsetRandomSampler's draw (storage.py:138-141), same generator
            perm = torch.randperm(batch_size).to(eng.device, non_blocking=True)
            for start in range(0, batch_size - mini_batch_size + 1, mini_batch_size):
                idx = perm[start:start + mini_batch_size]
                eng.train_minibatch(rollouts, advantages, idx, hp, self._loss_acc, self.optimizer)
        return self._losses()

    def _update_recurrent(self, eng, rollouts, advantages, hp, num_processes):
        """recurrent_generator semantics (storage.py:162-223): env order from
        torch.randperm(N) on the default CPU generator, N//M whole sequences per
        minibatch, BPTT over the full rollout."""
        assert num_processes >= self.num_mini_batch, (
            "PPO requires the number of processes ({}) "
            "to be greater than or equal to the number of "
            "PPO mini batches ({}).".format(num_processes, self.num_mini_batch))
        per = num_processes // self.num_mini_batch
        for e in range(self.ppo_epoch):
            perm = torch.randperm(num_processes)
            for start in range(0, num_processes, per):
                if start + per > num_processes:
                    raise IndexError("index {} is out of bounds for dimension 0 with size {}".format(
                        num_processes, num_processes))
                envs = perm[start:start + per].to(eng.device, non_blocking=True)
                eng.train_minibatch_rec(rollouts, advantages, envs, hp, self._loss_acc, self.optimizer)

    def _losses(self):
        eng = self.actor_critic.hip_engine()
        self._loss_acc[4].copy_(eng.status[0])    # the timeout flag travels with the losses (one all-reduce):
        _dist.allreduce_losses(self._loss_acc)     # every rank sees any rank's failure and raises with it
        num_updates = self.ppo_epoch * self.num_mini_batch        # ppo.py:90 (not the drop_last count)
        acc = self._loss_acc.tolist()                              # one D2H per update
        self.optimizer.guard = None
        if acc[3] > 0 or acc[4] > 0:
            # the guarded steps were no-ops on the device: undo their step count so the
            # parameters, moments and step counter are those of the last good step
            self.optimizer.step_count -= int(eng.status[1].item())
            eng.status[:2].zero_()
        if acc[4] > 0:
            # a persistent GRU sequence kernel gave up a bounded wait: no step used its outputs
            raise RuntimeError("PPO.update: persistent GRU kernel timed out; the optimizer steps from that "
                               "minibatch on were skipped (ppo_gru_persist_set(0) selects the step launches)")
        if acc[3] > 0:
            # the reference's log_probs gather (distributions.py:22) raises on such an index, before
            # its optimizer step; each epoch visits every stored row once, hence / ppo_epoch
            raise IndexError("PPO.update: {:.0f} stored action(s) outside [0, {}) in the rollout".format(
                acc[3] * _dist.world_size() / self.ppo_epoch, eng.A))
        value_loss_epoch, action_loss_epoch, dist_entropy_epoch = (x / num_updates for x in acc[:3])
        return value_loss_epoch, action_loss_epoch, dist_entropy_epoch
