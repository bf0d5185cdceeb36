"""Reference replays at the production hidden sizes.

The fixtures are recorded from the reference's own modules by
tools/gen_golden.py (container side): a whole T/run.py iteration of the
CNNBase at c3's H = 512 (`cnn_update_h512.npz`: 4 envs x 4 steps; and
`cnn_update_wide.npz`: 128 envs x 128 steps in one 16,384-sample minibatch,
wide enough that ppo_fc_fwd takes the production 128 x 128 fc tiles), and the
recurrent PPO.update at c5's H = 256 + 14 vector obs (`gru_update_h256.npz`),
which runs the persistent split-bf16 GRU forward and BPTT.  Production-size
tensors are stored as digests (every 8th element, per-tensor max |x| and L2).

Replayed through the drop-in API in host-sampling mode (the reference's
multinomial draw on the default CPU generator), starting from the recorded
initial parameters: actions bit-exact, log-probs / values / returns within
1e-5, losses within 1e-4 relative, the first minibatch's pre-clip gradient
within 1e-5 of each tensor's max |g| (sampled) and its per-tensor L2 within
1e-5 relative, final parameters within 2e-5 (sampled).
References: T/a2c_ppo_acktr/storage.py:82-223, model.py:54-199,
algo/ppo.py:34-96, T/run.py:168-248.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ppo_oracle as O

pytestmark = pytest.mark.gpu


def _dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return t if dtype is None else t.to(dtype)


def _load_flat(pol, flat):
    with torch.no_grad():
        off = 0
        for p in pol.parameters():
            p.copy_(torch.from_numpy(np.ascontiguousarray(flat[off:off + p.numel()])).view_as(p))
            off += p.numel()


def _digest_check(got_flat, d, prefix, shapes, tol, rel=True, scale=1.0):
    """rel: sampled elements within tol x the tensor's max |x| and each tensor's L2
    within 1e-5 relative (gradients); else within tol absolute and the L2 within
    tol x sqrt(numel) (parameters: an Adam step moves every element by ~lr whatever
    its size)."""
    idx = d[f"{prefix}_idx"]
    ref = d[f"{prefix}_sampled"].astype(np.float64) * scale
    got = np.asarray(got_flat, np.float64)
    off = 0
    for k, (name, shape) in enumerate(shapes):
        n = int(np.prod(shape))
        sel = (idx >= off) & (idx < off + n)
        tmax = d[f"{prefix}_tmax"][k] * scale
        err = np.abs(got[idx[sel]] - ref[sel]).max()
        l2, l2ref = np.sqrt((got[off:off + n] ** 2).sum()), d[f"{prefix}_tl2"][k] * scale
        if rel:
            assert err <= tol * max(tmax, 1e-6), (prefix, name, err, tmax)
            np.testing.assert_allclose(l2, l2ref, rtol=1e-5, err_msg=f"{prefix} {name}")
        else:
            assert err <= tol, (prefix, name, err)
            assert abs(l2 - l2ref) <= tol * np.sqrt(n), (prefix, name, l2, l2ref)
        off += n
    assert off == got.size


def _grads_vs_float64(got_flat, d, shapes, fro_tol=3e-5, max_tol=1e-4, ratio=2.0, floor=1e-6):
    """The first minibatch's gradient against the fixture's float64 digest of the
    same gradient (oracle/torch_ref float64 autograd on the recorded rollout), with
    the reference's own fp32 gradient (its digest) as the precision yardstick — the
    rule of tests/helpers/gradcheck.py on the sampled elements: per tensor, max |err|
    <= max(max_tol, ratio x the reference's) of max |g|, relative Frobenius error <=
    max(fro_tol, ratio x the reference's) and <= ratio x the reference's + floor."""
    idx = d["mb0_grad_f64_idx"]
    f64 = d["mb0_grad_f64_sampled"].astype(np.float64)
    r32 = d["mb0_preclip_grad_sampled"].astype(np.float64)
    got = np.asarray(got_flat, np.float64)[idx]
    off, bad = 0, []
    for k, (name, shape) in enumerate(shapes):
        n = int(np.prod(shape))
        sel = (idx >= off) & (idx < off + n)
        scale, norm = max(d["mb0_grad_f64_tmax"][k], 1e-12), max(np.linalg.norm(f64[sel]), 1e-12)
        e, e32 = got[sel] - f64[sel], r32[sel] - f64[sel]
        mx, fro = np.abs(e).max() / scale, np.linalg.norm(e) / norm
        mx32, fro32 = np.abs(e32).max() / scale, np.linalg.norm(e32) / norm
        line = f"{name:28s} HIP max {mx:.2e} fro {fro:.2e} | reference fp32 max {mx32:.2e} fro {fro32:.2e}"
        print(line, flush=True)
        if not (mx <= max(max_tol, ratio * mx32) and fro <= max(fro_tol, ratio * fro32)
                and fro <= ratio * fro32 + floor):
            bad.append(line)
        off += n
    assert not bad, bad


def _capture_steps(agent):
    grads, accs = [], []
    orig = agent.optimizer._step_flat

    def step_capture(e):
        grads.append(e.grad.clone())          # clip_grad_norm_'s input (before clip + Adam)
        accs.append(agent._loss_acc[:3].clone())
        return orig(e)

    agent.optimizer._step_flat = step_capture
    return grads, accs, orig


def _cnn_replay(gpu, d, obs_u8):
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    torch.set_num_threads(1)
    torch.manual_seed(1)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase,
                   base_kwargs={"recurrent": False, "hidden_size": hidden}, vector_obs_len=0)
    # the default generator after construction = the reference's (its sampling and
    # randperm draws start here); the parameters themselves come from the fixture
    # (orthogonal_'s QR may round differently on this host's CPU)
    assert np.array_equal(torch.get_rng_state().numpy(), d["rng_after_init"])
    _load_flat(pol, d["init_params"])
    pol.to(gpu)
    agent = PPO(pol, 0.1, E, Mb, 0.5, 0.001, lr=float(d["lr"][0]), eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [0], Discrete(8), pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=gpu)
    st.obs.copy_(obs_u8)
    grads, accs, orig = _capture_steps(agent)
    M.set_sampling_mode("host")
    try:
        for step in range(T):
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                  st.masks[step])
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, _dev(d["rewards"][step]),
                      _dev(d["masks"][step]), torch.ones(N, 1, device=gpu))
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)
        losses = agent.update(st)
    finally:
        M.set_sampling_mode("device")
        agent.optimizer._step_flat = orig
    assert np.array_equal(st.actions.cpu().numpy(), d["actions"])
    np.testing.assert_allclose(st.action_log_probs.cpu().numpy(), d["action_log_probs"], atol=1e-5)
    np.testing.assert_allclose(st.value_preds[:T].cpu().numpy(), d["values"], atol=1e-5)
    np.testing.assert_allclose(st.returns.cpu().numpy(), d["returns"], atol=1e-5)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4, atol=1e-6)
    assert len(grads) == E * Mb
    shapes = O.cnn_param_shapes(hidden)
    if "mb0_grad_f64_idx" in d.files:   # a production-size minibatch: held to the reference's own precision
        _grads_vs_float64(grads[0].cpu().numpy(), d, shapes)
    else:
        _digest_check(grads[0].cpu().numpy(), d, "mb0_preclip_grad", shapes, 1e-5)
    final = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu().numpy()
    _digest_check(final, d, "final_params", shapes, 2e-5, rel=False)


def test_cnn_h512_iteration_replays_reference(gpu):
    """c3's CNNBase (H = 512) through one whole reference iteration (4 envs x 4
    steps, E = 2, M = 2): the production-size conv / fc / heads kernels at the
    replay's minibatch of 8 samples."""
    d = golden("cnn_update_h512.npz")
    _cnn_replay(gpu, d, _dev(d["obs_u8"]))


def test_cnn_wide_iteration_replays_reference(gpu):
    """c3's CNNBase (H = 512) over 128 envs x 128 steps with one 16,384-sample
    minibatch (E = 1, M = 1): ceil(16384 / 128) x (512 / 128) = 512 fc tiles >= 2 x
    the CU count, so ppo_fc_fwd runs the production 128 x 128 tile kernel
    (DenseReluFwdB<XP128>) and the persistent conv kernels walk 64 images per
    block, as at c3's 65,536-sample minibatch.  The observations are regenerated
    from the fixture's generator seed (checked by byte sum and CRC-32).  The
    gradient of this 16,384-sample minibatch is checked against its float64 value
    with the reference's own fp32 error as the bar (_grads_vs_float64): the
    reference itself is 5.5e-5 (max) / 4.0e-5 (Frobenius) from float64 on conv1's
    weight gradient here."""
    import zlib
    d = golden("cnn_update_wide.npz")
    hidden, N, T, E, Mb = (int(x) for x in d["meta"])
    assert -(-N * T // 128) * (hidden // 128) >= 2 * torch.cuda.get_device_properties(0).multi_processor_count
    o = torch.randint(0, 256, (T + 1, N, 4, 84, 84), dtype=torch.uint8,
                      generator=torch.Generator().manual_seed(int(d["obs_seed"][0])))
    on = o.numpy()
    assert [int(on.sum(dtype=np.int64)), zlib.crc32(on.tobytes())] == [int(x) for x in d["obs_check"]]
    _cnn_replay(gpu, d, o.to(gpu))


def test_recurrent_h256_iteration_replays_reference(gpu):
    """c5's recurrent policy (GRU H = 256 + 14 vector obs; 8 envs x 16 steps, masks
    with zeros, a carried initial hidden state; E = 2, M = 2): the persistent
    whole-sequence GRU forward and BPTT on the six-product split-bf16 W_hh MFMAs
    (H >= 128), asserted taken through the BPTT's path report."""
    from a2c_ppo_acktr import _hip as Hh
    from a2c_ppo_acktr import model as M
    from a2c_ppo_acktr.algo import PPO
    from a2c_ppo_acktr.storage import RolloutStorage
    from a2c_ppo_acktr.synthetic import Discrete
    d = golden("gru_update_h256.npz")
    hidden, V, N, T, E, Mb = (int(x) for x in d["meta"])
    clip, vcoef, ecoef = (float(x) for x in d["coefs"])
    assert Hh.call("ppo_gru_persist_get") & 3 == 3, "persistent forward and BPTT are the defaults"
    torch.set_num_threads(1)
    torch.manual_seed(31)
    pol = M.Policy((4, 84, 84), Discrete(8), base=M.CNNBase, base_kwargs={"recurrent": True, "hidden_size": hidden},
                   vector_obs_len=V)
    assert np.array_equal(torch.get_rng_state().numpy(), d["rng_after_init"])
    _load_flat(pol, d["init_params"])
    pol.to(gpu)
    agent = PPO(pol, clip, E, Mb, vcoef, ecoef, lr=float(d["lr"][0]), eps=1e-5, max_grad_norm=0.5)
    st = RolloutStorage(T, N, (4, 84, 84), [V], Discrete(8), pol.recurrent_hidden_state_size,
                        obs_dtype=torch.uint8, device=gpu)
    st.obs.copy_(_dev(d["obs_u8"]))
    st.vector_obs.copy_(_dev(d["vector_obs"]))
    st.recurrent_hidden_states[0].copy_(_dev(d["h0"]))
    st.masks[0].copy_(_dev(d["masks0"]))
    eng = pol.hip_engine()
    grads, accs, orig = _capture_steps(agent)
    M.set_sampling_mode("host")
    try:
        for step in range(T):
            v, a, lp, h = pol.act(st.obs[step], st.vector_obs[step], st.recurrent_hidden_states[step],
                                  st.masks[step])
            st.insert(st.obs[step + 1], st.vector_obs[step + 1], h, a, lp, v, _dev(d["rewards"][step]),
                      _dev(d["masks"][step]), torch.ones(N, 1, device=gpu))
        nv = pol.get_value(st.obs[-1], st.vector_obs[-1], st.recurrent_hidden_states[-1], st.masks[-1])
        st.compute_returns(nv, True, 0.99, 0.95, False)
        losses = agent.update(st)
    finally:
        M.set_sampling_mode("device")
        agent.optimizer._step_flat = orig
    torch.cuda.synchronize()
    # the BPTT's report (ppo_gru_seq_counters layout: [G step counters][G reports]): 1 = the
    # group ran the persistent kernel; 0 would mean the step launches ran
    n = N // Mb
    G = -(-n // 32)
    cnt = eng.ws["train"].bufs["gru_cnt"].cpu().numpy()
    assert (cnt[G:2 * G] == 1).all(), cnt[:2 * G]
    assert np.array_equal(st.actions.cpu().numpy(), d["actions"])
    np.testing.assert_allclose(st.action_log_probs.cpu().numpy(), d["action_log_probs"], atol=1e-5)
    np.testing.assert_allclose(st.value_preds[:T].cpu().numpy(), d["values"], atol=1e-5)
    np.testing.assert_allclose(st.recurrent_hidden_states[-1].cpu().numpy(), d["hidden_T"], atol=1e-5)
    np.testing.assert_allclose(st.returns.cpu().numpy(), d["returns"], atol=1e-5)
    assert len(grads) == E * Mb
    shapes = O.cnn_param_shapes(hidden, recurrent=True, vector_obs_len=V)
    _digest_check(grads[0].cpu().numpy(), d, "mb0_preclip_grad", shapes, 1e-5)
    acc = torch.stack(accs + [agent._loss_acc[:3].clone()]).cpu().numpy()
    mb = np.diff(np.concatenate([np.zeros((1, 3)), acc[:-1]], 0), axis=0)
    np.testing.assert_allclose(mb, d["mb_losses"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4, atol=1e-6)
    final = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).cpu().numpy()
    _digest_check(final, d, "final_params", shapes, 2e-5, rel=False)
