"""Evaluation path: T/run_evaluation.py:25-122 steps one
env with Policy.act(obs, vector_obs, hxs, masks, deterministic) — batch 1, GRU
state carried across steps, masks zeroed on done.  At batch 1 every act is a
chain of ~10 tiny kernels, so launch overhead, not arithmetic, sets the step
latency.  GraphedActor records that chain once into a HIP graph (torch.cuda.graph
drives hipStreamBeginCapture on the current stream, which is where every
libppo_hip.so launch goes) and replays it per step: inputs are copied into
static buffers, one graph launch runs the whole forward.

The graph holds raw pointers, so everything it touches is kept stable: the
forward runs in the engine's own "graph" workspace (no eager act, get_value or
rollout at another batch size reallocates it), the packed weight planes are
refreshed in place before a replay when the parameters changed, and the graph is
re-captured when the flat parameter buffer or the packed planes were
reallocated (Policy re-bound, moved, or a new engine).  Only deterministic
acting is graphed (the stochastic sampler's RNG counter is a launch argument
and would freeze inside a graph).

Two ways to drive it:
  act(obs, vec, hxs, masks)  Policy.act's signature; checks every call that the
                             graph is still valid (engine, buffers, precision,
                             parameter versions) and copies the inputs in.
  replay()                   the evaluation loop's fast path: the caller writes
                             the next observation / masks straight into the
                             pointer-stable inputs (ga.obs, ga.vec, ga.masks) and
                             the graph itself feeds its new hidden state back into
                             ga.hxs (carry_hidden=True); no host checks — call
                             refresh() after changing the parameters.
"""
import torch


class GraphedActor(object):
    def __init__(self, policy, num_envs=1, obs_dtype=torch.float32, device=None, warmup=2, carry_hidden=False):
        eng = policy.hip_engine(device)
        self.policy, self.device, self.warmup = policy, eng.device, warmup
        self.carry_hidden = bool(carry_hidden) and policy.is_recurrent
        base = policy.base
        C = base.main[0].weight.shape[1]
        V = getattr(base, "vector_obs_len", 0)
        Hh = policy.recurrent_hidden_state_size
        dev = self.device
        self.obs = torch.zeros(num_envs, C, 84, 84, dtype=obs_dtype, device=dev)
        self.vec = torch.zeros(num_envs, V, device=dev)
        self.hxs = torch.zeros(num_envs, Hh, device=dev)
        self.masks = torch.ones(num_envs, 1, device=dev)
        self.captures = 0
        self._capture()

    def _capture(self):
        dev = self.device
        self.eng = self.policy.hip_engine(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with self.eng.using_workspace("graph"):
            with torch.cuda.stream(side):   # warm-up: workspaces, packed weights, device attributes
                for _ in range(self.warmup):
                    self._act()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self._act()
                if self.carry_hidden:   # h' -> the next replay's h, inside the graph
                    self.hxs.copy_(self.out[3])
        self._key = self._pack_key()
        self._ptrs = self._pointers()
        self.captures += 1

    def _act(self):
        with torch.no_grad():
            return self.policy.act(self.obs, self.vec, self.hxs, self.masks, deterministic=True)

    def _pack_key(self):
        return (sum(p._version for p in self.eng.params), self.eng.epoch)

    def _pointers(self):
        """every buffer address baked into the graph that could be reallocated, and
        the arithmetic mode the kernels were captured with (Policy.half() / float()
        switch the GEMMs' part-product count, a launch argument frozen in the graph)"""
        e = self.eng
        gp = getattr(e, "gru_packed", None)
        ws = e.ws["graph"]
        return (id(e), e.flat.data_ptr(), e.packed.data_ptr(), None if gp is None else gp.data_ptr(),
                id(ws), ws.version,   # any workspace reallocation bumps its version
                bool(getattr(self.policy, "_half_mode", False)))

    def refresh(self):
        """re-validate after the caller changed the policy (parameters updated in
        place, moved, re-bound, half()/float()): re-capture or re-pack as needed"""
        eng = self.policy.hip_engine(self.device)
        if eng is not self.eng or self._pointers() != self._ptrs:
            self._capture()
        elif self._pack_key() != self._key:
            self.eng.pack(force=True)
            self._key = self._pack_key()

    def replay(self):
        """one deterministic act of the inputs in ga.obs / ga.vec / ga.hxs / ga.masks
        -> (value, action, log_prob, rnn_hxs) output buffers (overwritten by the next
        replay); with carry_hidden the new hidden state is already in ga.hxs"""
        self.graph.replay()
        return self.out

    def act(self, visual_inputs, vector_inputs, rnn_hxs, masks, deterministic=True):
        """Policy.act (model.py:54-66) for the captured batch -> (value, action, log_prob, rnn_hxs)"""
        if not deterministic:
            raise NotImplementedError("GraphedActor replays deterministic acting only; use Policy.act to sample")
        self.refresh()   # buffers moved: re-capture; parameters updated in place: re-pack
        for dst, src in ((self.obs, visual_inputs), (self.vec, vector_inputs), (self.hxs, rnn_hxs),
                         (self.masks, masks)):
            if dst.numel() and src is not dst:
                dst.copy_(src.reshape(dst.shape), non_blocking=True)
        self.graph.replay()
        # the graph's output buffers, overwritten by the next act (as torch.cuda.graphs
        # outputs are); the hidden state fed back in is copied before that happens
        return self.out
