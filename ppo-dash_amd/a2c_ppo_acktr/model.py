"""Actor-critic networks — drop-in for a2c_ppo_acktr/model.py (reference
ppo-dash-training/pytorch-a2c-ppo-acktr-gail/a2c_ppo_acktr/model.py:10-234).

The modules are built exactly as the reference builds them (same layer
constructors, same init calls, same order), so under the same
torch.manual_seed the initial parameters are identical.  The layers are only
parameter containers: act / get_value / evaluate_actions run on the MI355X
through libppo_hip.so (see _engine.py); there is no CPU compute path.

Differences from the reference, all documented in DESIGN.md:
  * CNNBase accepts uint8 observations and decodes u8/255 inside conv1.
  * MLPBase's constructor takes (num_inputs, vector_obs_len, ...) so that
    Policy can build it (the reference mis-calls it, model.py:28 vs :203).
  * evaluate_actions returns values without an autograd graph; PPO.update runs
    its own fused HIP backward.
  * MLPBase's forward uses cat(obs, vector_obs) as its input (the reference
    builds a tuple there, model.py:225-226).
"""
import numpy as np
import torch
import torch.nn as nn

from ._hip import require_device
from .distributions import Bernoulli, Categorical, DiagGaussian
from .utils import init


class Flatten(nn.Module):
    def forward(self, x):
        return x.view(x.size(0), -1)


_SAMPLING = {"mode": "device"}


def set_sampling_mode(mode):
    """'device' (default): Exp(1) sampling noise from a counter-based RNG on the GPU.
    'host': draw it with torch.empty(N, A).exponential_(1) on the default CPU
    generator — the draw torch.multinomial makes on the reference CPU path — so a
    seeded run consumes the host generator exactly like the reference does."""
    if mode not in ("device", "host"):
        raise ValueError(mode)
    _SAMPLING["mode"] = mode


class Policy(nn.Module):
    def __init__(self, obs_shape, action_space, base=None, base_kwargs=None, vector_obs_len=0):
        super(Policy, self).__init__()
        if base_kwargs is None:
            base_kwargs = {}
        if base is None:
            if len(obs_shape) == 3:
                base = CNNBase
            elif len(obs_shape) == 1:
                base = MLPBase
            else:
                raise NotImplementedError
        # constructor arguments, for checkpoint.save_checkpoint (state_dict-based files)
        self._ctor = {"obs_shape": tuple(obs_shape), "action_space": action_space, "base_kwargs": dict(base_kwargs),
                      "vector_obs_len": vector_obs_len}
        self.base = base(obs_shape[0], vector_obs_len, **base_kwargs)
        if action_space.__class__.__name__ == "Discrete":
            num_outputs = action_space.n
            self.dist = Categorical(self.base.output_size, num_outputs)
        elif action_space.__class__.__name__ == "Box":
            num_outputs = action_space.shape[0]
            self.dist = DiagGaussian(self.base.output_size, num_outputs)
        elif action_space.__class__.__name__ == "MultiBinary":
            num_outputs = action_space.shape[0]
            self.dist = Bernoulli(self.base.output_size, num_outputs)
        else:
            raise NotImplementedError
        self._engine = None

    @property
    def is_recurrent(self):
        return self.base.is_recurrent

    @property
    def recurrent_hidden_state_size(self):
        """Size of rnn_hx."""
        return self.base.recurrent_hidden_state_size

    def forward(self, visual_inputs, vector_inputs, rnn_hxs, masks):
        raise NotImplementedError

    # ------------------------------------------------------------- precision
    def half(self):
        """--half-precision (T/run.py:84-85 calls actor_critic.half()): every
        trunk / GRU / head GEMM then multiplies bf16-rounded operands — one
        bf16 MFMA product with fp32 accumulation instead of the six-product fp32
        emulation — which is the matrix cores' native rate.  Unlike the
        reference (fp16 parameters and fp16 Adam state), the parameters,
        gradients and Adam moments stay fp32 masters; Policy.float() returns to
        fp32 arithmetic.  Returns self, as nn.Module.half() does."""
        self._half_mode = True
        return self

    def float(self):
        self._half_mode = False
        return super(Policy, self).float()

    @property
    def half_precision(self):
        return getattr(self, "_half_mode", False)

    def set_obs_decode(self, preprocess):
        """Feed raw u8 RGB frames [N][84][84][3] (VecPyTorch(..., fused=True),
        RolloutStorage(..., (84, 84, 3), obs_dtype=torch.uint8)) instead of the fp32
        4-channel policy input: the env-side NormalizeWrapper + FrameStackMono(2) +
        TransposeImage + .float() chain (T/make_env.py:411-413) that `preprocess`
        (a vec_env.ObsPreprocess, mono=True) describes then runs inside conv1's
        operand loader, bit-identical to it (csrc/conv1f.hip).  None switches back."""
        eng = self.hip_engine()
        if preprocess is None:
            eng.obs_decode = None
            return self
        if not preprocess.mono or preprocess.size != 84:
            raise NotImplementedError("the fused decode is FrameStackMono(2) on 84x84 frames (mono=True)")
        if preprocess.mode == "norm":
            eng.set_obs_decode(preprocess.mean, preprocess.std)
        else:
            eng.set_obs_decode(None, 255.0 if preprocess.mode == "div255" else 1.0)
        return self

    # ------------------------------------------------------------- engine
    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None   # torch.save([actor_critic, ob_rms]) pickles the module, not the engine
        return st

    def hip_engine(self, device=None):
        require_device()
        if not isinstance(self.dist, Categorical):
            raise NotImplementedError("only Discrete action spaces run on the MI355X engine")
        if device is None:
            p = next(self.parameters())
            device = p.device if p.is_cuda else torch.device("cuda", torch.cuda.current_device())
        if self._engine is None or self._engine.device != device:
            from ._engine import CNNEngine, MLPEngine, RecurrentEngine
            if not next(self.parameters()).is_cuda:
                self.to(device)
            if isinstance(self.base, MLPBase):
                self._engine = MLPEngine(self, device)
            else:
                self._engine = (RecurrentEngine if self.base.is_recurrent else CNNEngine)(self, device)
        self._engine.ensure_bound()
        return self._engine

    def _noise(self, n):
        if _SAMPLING["mode"] == "host":
            return torch.empty(n, self.dist.linear.weight.shape[0]).exponential_(1)
        return None

    # ----------------------------------------------------------------- API
    def act(self, visual_inputs, vector_inputs, rnn_hxs, masks, deterministic=False):
        """model.py:54-66 -> (value [N,1], action [N,1] int64, action_log_probs [N,1], rnn_hxs)."""
        eng = self.hip_engine()
        n = visual_inputs.shape[0]
        noise = None if deterministic else self._noise(n)
        if self.is_recurrent:
            value, action, logp, _, rnn_hxs = eng.act(visual_inputs, deterministic=deterministic, noise=noise,
                                                      vec=vector_inputs, hxs=rnn_hxs, masks=masks)
            return value, action, logp, rnn_hxs
        if isinstance(self.base, MLPBase):
            value, action, logp, _ = eng.act(visual_inputs, deterministic=deterministic, noise=noise,
                                             vec=vector_inputs)
            return value, action, logp, rnn_hxs
        value, action, logp, _ = eng.act(visual_inputs, deterministic=deterministic, noise=noise)
        return value, action, logp, rnn_hxs

    def get_value(self, visual_inputs, vector_inputs, rnn_hxs, masks):
        """model.py:68-70."""
        eng = self.hip_engine()
        if self.is_recurrent:
            return eng.act(visual_inputs, value_only=True, vec=vector_inputs, hxs=rnn_hxs, masks=masks)[0]
        if isinstance(self.base, MLPBase):
            return eng.act(visual_inputs, value_only=True, vec=vector_inputs)[0]
        value, _, _, _ = eng.act(visual_inputs, value_only=True)
        return value

    def evaluate_actions(self, visual_inputs, vector_inputs, rnn_hxs, masks, action):
        """model.py:72-79 -> (value [B,1], action_log_probs [B,1], dist_entropy (0-d), rnn_hxs)."""
        eng = self.hip_engine()
        action = action.to(eng.device, torch.int64)
        if self.is_recurrent:
            if visual_inputs.shape[0] == rnn_hxs.shape[0]:   # model.py:112 single-step branch
                value, _, logp, ent, rnn_hxs = eng.act(visual_inputs, given=action, want_entropy=True,
                                                       vec=vector_inputs, hxs=rnn_hxs, masks=masks)
            else:                                             # model.py:116-165 sequence branch
                value, logp, ent, rnn_hxs = eng.evaluate_sequence(visual_inputs, vector_inputs, rnn_hxs, masks,
                                                                  action)
            return value, logp, eng.mean(ent), rnn_hxs
        if isinstance(self.base, MLPBase):
            value, _, logp, ent = eng.act(visual_inputs, given=action, want_entropy=True, vec=vector_inputs)
        else:
            value, _, logp, ent = eng.act(visual_inputs, given=action, want_entropy=True)
        return value, logp, eng.mean(ent), rnn_hxs


class NNBase(nn.Module):
    def __init__(self, recurrent, recurrent_input_size, hidden_size):
        super(NNBase, self).__init__()
        self._hidden_size = hidden_size
        self._recurrent = recurrent
        if recurrent:
            self.gru = nn.GRU(recurrent_input_size, hidden_size)
            for name, param in self.gru.named_parameters():
                if 'bias' in name:
                    nn.init.constant_(param, 0)
                elif 'weight' in name:
                    nn.init.orthogonal_(param)

    @property
    def is_recurrent(self):
        return self._recurrent

    @property
    def recurrent_hidden_state_size(self):
        if self._recurrent:
            return self._hidden_size
        return 1

    @property
    def output_size(self):
        return self._hidden_size


class CNNBase(NNBase):
    """model.py:169-199: conv 8/4 -> conv 4/2 -> conv 3/1 -> fc(1568, H), ReLU after each."""

    def __init__(self, num_inputs, vector_obs_len=0, recurrent=False, hidden_size=512):
        super(CNNBase, self).__init__(recurrent, hidden_size + vector_obs_len, hidden_size)
        init_ = lambda m: init(m, nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0),
                               nn.init.calculate_gain('relu'))
        self.main = nn.Sequential(
            init_(nn.Conv2d(num_inputs, 32, 8, stride=4)), nn.ReLU(),
            init_(nn.Conv2d(32, 64, 4, stride=2)), nn.ReLU(),
            init_(nn.Conv2d(64, 32, 3, stride=1)), nn.ReLU(), Flatten(),
            init_(nn.Linear(32 * 7 * 7, hidden_size)), nn.ReLU())
        init_ = lambda m: init(m, nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0))
        if recurrent:
            self.critic_linear = init_(nn.Linear(hidden_size, 1))
        else:
            self.critic_linear = init_(nn.Linear(hidden_size + vector_obs_len, 1))
        self.vector_obs_len = vector_obs_len
        self.train()

    def forward(self, visual_inputs, vector_inputs, rnn_hxs, masks):
        raise NotImplementedError("CNNBase runs through Policy.act/get_value/evaluate_actions on the HIP engine")


class MLPBase(NNBase):
    """model.py:202-234 (constructor signature fixed so Policy can build it)."""

    def __init__(self, num_inputs, vector_obs_len=0, recurrent=False, hidden_size=64):
        super(MLPBase, self).__init__(recurrent, num_inputs + vector_obs_len, hidden_size)
        num_inputs = num_inputs + vector_obs_len
        if recurrent:
            num_inputs = hidden_size
        self.vector_obs_len = vector_obs_len
        init_ = lambda m: init(m, nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0), np.sqrt(2))
        self.actor = nn.Sequential(
            init_(nn.Linear(num_inputs, hidden_size)), nn.Tanh(),
            init_(nn.Linear(hidden_size, hidden_size)), nn.Tanh())
        self.critic = nn.Sequential(
            init_(nn.Linear(num_inputs, hidden_size)), nn.Tanh(),
            init_(nn.Linear(hidden_size, hidden_size)), nn.Tanh())
        self.critic_linear = init_(nn.Linear(hidden_size, 1))
        self.train()

    def forward(self, visual_inputs, vector_inputs, rnn_hxs, masks):
        raise NotImplementedError("MLPBase runs through Policy.act/get_value/evaluate_actions on the HIP engine")
