"""--half-precision (T/run.py:84-85, 137-138, 212-214; storage.py:48-58): Policy.half()
switches the trunk / GRU / head GEMMs to one bf16 MFMA product per fp32 product
(bf16-rounded operands, fp32 accumulation); RolloutStorage.half() stores float
image observations as fp16.  Parity is held to float64 at a stated bf16
tolerance (bf16 keeps 8 significand bits: a product of two rounded operands is
within 2^-8 relative): per-tensor relative Frobenius error of the minibatch
gradient <= 2e-2, forward values / log-probs within 2e-2 of max|value|."""
import numpy as np
import pytest
import torch

from oracle import ppo_oracle as O
from oracle import torch_ref as TR

pytestmark = pytest.mark.gpu

HP = {"clip": 0.1, "value_coef": 0.5, "entropy_coef": 0.001, "use_clipped_value_loss": True}
BF16_TOL = 2e-2


class _GradCapture(object):
    def _step_flat(self, eng):
        self.grad = eng.grad.clone()


def _storage(gpu, T, N, A, seed, obs_dtype=torch.uint8):
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(A), 1, obs_dtype=obs_dtype, device=gpu)
    g = torch.Generator().manual_seed(seed)
    st.obs.copy_(torch.randint(0, 256, st.obs.shape, dtype=torch.uint8, generator=g).to(gpu).to(obs_dtype))
    st.actions.copy_(torch.randint(0, A, st.actions.shape, generator=g).to(gpu))
    st.action_log_probs.copy_((torch.log(torch.rand(st.action_log_probs.shape, generator=g)) * 0.3 - 2.0).to(gpu))
    st.value_preds.copy_(torch.randn(st.value_preds.shape, generator=g).to(gpu) * 0.1)
    st.returns.copy_(torch.randn(st.returns.shape, generator=g).to(gpu))
    return st


@pytest.mark.parametrize("obs_dtype", [torch.uint8, torch.float16])
def test_half_minibatch_gradient_vs_float64(gpu, obs_dtype):
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    H, T, N, A = 512, 16, 256, 8
    torch.manual_seed(4)
    pol = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    with torch.no_grad():
        pol.dist.linear.weight.mul_(30.0)
    flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    pol.to(gpu)
    assert pol.half() is pol and pol.half_precision
    assert next(pol.parameters()).dtype == torch.float32          # fp32 masters
    st = _storage(gpu, T, N, A, 5, torch.uint8)
    if obs_dtype == torch.float16:   # normalised frames stored as fp16 (make_env.py:81-104)
        st.obs = (st.obs.float() / 255.0).half()
    adv = torch.randn(T, N, generator=torch.Generator().manual_seed(6)).to(gpu)
    idx = torch.randperm(T * N, generator=torch.Generator().manual_seed(7))[:4096].to(gpu)
    eng = pol.hip_engine()
    loss = torch.zeros(4, dtype=torch.float64, device=gpu)
    cap = _GradCapture()
    eng.train_minibatch(st, adv, idx, HP, loss, cap)
    torch.cuda.synchronize()
    p = TR.unflatten(flat0, H, dtype=torch.float64, device=gpu, requires_grad=True)
    obs_u8 = st.obs[:T].reshape(T * N, 4, 84, 84)   # fp16 planes: the stored fp16 values, exactly
    fl = lambda t: t[:T].reshape(T * N, *t.shape[2:])  # noqa: E731
    grads, losses = TR.minibatch_grads(p, obs_u8, fl(st.actions), fl(st.action_log_probs), adv.reshape(-1),
                                       fl(st.value_preds), fl(st.returns), idx=idx, clip=HP["clip"],
                                       value_coef=HP["value_coef"], entropy_coef=HP["entropy_coef"])
    got = O.unflatten(cap.grad.cpu().numpy(), O.cnn_param_shapes(H))
    for (name, _), ref in zip(O.cnn_param_shapes(H), grads):
        ref = ref.cpu().numpy()
        fro = np.linalg.norm(got[name] - ref) / max(np.linalg.norm(ref), 1e-12)
        print(f"{name:28s} half-mode relative Frobenius error {fro:.2e}", flush=True)
        assert fro <= BF16_TOL, (name, fro)
    np.testing.assert_allclose(loss[:3].cpu().numpy(), losses, rtol=BF16_TOL, atol=1e-4)
    pol.float()
    if obs_dtype != torch.float16:
        # back to fp32 on the u8 plane: the engine repacks the fp32 weights, so its
        # gradient equals, bit for bit, that of a fresh fp32 policy that never ran in
        # half mode (whose accuracy test_full_size.py holds against float64)
        torch.manual_seed(4)
        fresh = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
        with torch.no_grad():
            fresh.dist.linear.weight.mul_(30.0)
        fresh.to(gpu)
        assert torch.equal(torch.cat([q.detach().reshape(-1) for q in fresh.parameters()]),
                           torch.cat([q.detach().reshape(-1) for q in pol.parameters()]))
        cap_back, cap_fresh = _GradCapture(), _GradCapture()
        eng.train_minibatch(st, adv, idx, HP, loss, cap_back)
        fresh.hip_engine().train_minibatch(st, adv, idx, HP, loss, cap_fresh)
        torch.cuda.synchronize()
        assert torch.equal(cap_back.grad, cap_fresh.grad)
        return
    # back to fp32 arithmetic on the fp16 plane: its rows are widened exactly (fp16 ->
    # fp32) and then take conv1's fp32-row kernels, whose accuracy test_full_size.py
    # holds against independent float64 references at the u8 bar.  Here: the fp16
    # plane gives bit for bit the gradient of an fp32 plane holding the same values.
    cap16, cap32 = _GradCapture(), _GradCapture()
    eng.train_minibatch(st, adv, idx, HP, loss, cap16)
    st.obs = st.obs.float()
    eng.train_minibatch(st, adv, idx, HP, loss, cap32)
    torch.cuda.synchronize()
    assert torch.equal(cap16.grad, cap32.grad)


def test_half_precision_run_py_flow(gpu):
    """The T/run.py --half-precision sequence through the drop-in API:
    actor_critic.half(); rollouts.half() on the reference's fp32 observation
    storage (-> fp16 plane); fp16 observations and masks from the caller
    (make_env.py:81-104, run.py:212-214); act / insert / compute_returns /
    update.  Values and log-probs stored by the rollout match the float64
    forward at the bf16 tolerance, and the update trains."""
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    N, T, H = 32, 8, 512
    torch.manual_seed(1)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    flat0 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).clone()
    pol.half()
    pol.to(gpu)
    agent = PPO(pol, 0.1, 2, 4, 0.5, 0.001, lr=1e-4, eps=1e-5, max_grad_norm=0.5)
    rollouts = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), pol.recurrent_hidden_state_size)
    rollouts.half()
    assert rollouts.obs.dtype == torch.float16
    g = torch.Generator().manual_seed(2)
    frames = [(torch.randint(0, 256, (N, 4, 84, 84), generator=g).float() / 255.0).half() for _ in range(T + 1)]
    rollouts.obs[0].copy_(frames[0])
    rollouts.to(gpu)
    for step in range(T):
        with torch.no_grad():
            value, action, logp, hxs = pol.act(rollouts.obs[step], rollouts.vector_obs[step],
                                               rollouts.recurrent_hidden_states[step], rollouts.masks[step])
        masks = torch.FloatTensor([[0.0] if i == step else [1.0] for i in range(N)]).half()
        bad_masks = torch.ones(N, 1).half()
        rollouts.insert(frames[step + 1].to(gpu), rollouts.vector_obs[step + 1], hxs, action, logp, value,
                        torch.rand(N, 1, generator=g), masks, bad_masks)
    with torch.no_grad():
        nv = pol.get_value(rollouts.obs[-1], rollouts.vector_obs[-1], rollouts.recurrent_hidden_states[-1],
                           rollouts.masks[-1])
    rollouts.compute_returns(nv, True, 0.99, 0.95, False)
    # stored values / log-probs vs the float64 forward of the fp16 frames
    p64 = O.unflatten(flat0.numpy(), O.cnn_param_shapes(H))
    x = torch.stack(frames[:T]).reshape(T * N, 4, 84, 84).double().numpy()
    value, logits, _ = O.cnn_forward(p64, x)
    nl = O.categorical(logits)["norm_logits"]
    acts = rollouts.actions.reshape(-1).cpu().numpy()
    lp = np.take_along_axis(nl, acts[:, None], 1)[:, 0]
    scale = max(np.abs(value).max(), 1.0)
    np.testing.assert_allclose(rollouts.value_preds[:T].reshape(-1).cpu().numpy(), value, atol=BF16_TOL * scale)
    np.testing.assert_allclose(rollouts.action_log_probs.reshape(-1).cpu().numpy(), lp, atol=BF16_TOL * 3)
    before = torch.cat([q.detach().reshape(-1) for q in pol.parameters()]).clone()
    losses = agent.update(rollouts)
    rollouts.after_update()
    after = torch.cat([q.detach().reshape(-1) for q in pol.parameters()])
    assert all(np.isfinite(losses)) and (after - before).abs().max().item() > 0


@pytest.mark.parametrize("conv1_wgrad", [5, 8, 9])
def test_minibatch_gradient_deterministic(gpu, conv1_wgrad):
    """The fused minibatch backward is run-to-run deterministic (fixed-order
    reductions everywhere): two identical minibatches give bit-identical
    gradients, for both conv1 weight-gradient kernels."""
    from a2c_ppo_acktr import _hip as Hh
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.synthetic import Discrete
    H, T, N, A = 512, 16, 256, 8
    torch.manual_seed(4)
    pol = M.Policy((4, 84, 84), Discrete(A), base=M.CNNBase, base_kwargs={"recurrent": False, "hidden_size": H})
    pol.to(gpu)
    st = _storage(gpu, T, N, A, 5, torch.uint8)
    adv = torch.randn(T, N, generator=torch.Generator().manual_seed(6)).to(gpu)
    idx = torch.randperm(T * N, generator=torch.Generator().manual_seed(7))[:4096].to(gpu)
    eng = pol.hip_engine()
    old = Hh.call("ppo_tune_get", b"conv1_wgrad")
    Hh.call("ppo_tune_set", b"conv1_wgrad", conv1_wgrad)
    try:
        grads = []
        for _ in range(3):
            loss = torch.zeros(4, dtype=torch.float64, device=gpu)
            cap = _GradCapture()
            eng.train_minibatch(st, adv, idx, HP, loss, cap)
            torch.cuda.synchronize()
            grads.append(cap.grad)
    finally:
        Hh.call("ppo_tune_set", b"conv1_wgrad", old)
    assert torch.equal(grads[0], grads[1]) and torch.equal(grads[0], grads[2])
