"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container, where the reference checkout is mounted read-only at
/root/reference (it never travels to the GPU box; only the .npz/.json outputs are committed).

What is executed (nothing is copied into this repo):
  * cleanrl/architectures/ppo.py is imported as a module (PPObj, PPODefault: pure torch);
  * the GAE block cleanrl/ppo_atari_oc.py:533-547 and the minibatch-update block :566-610 are read
    as text by line range, dedented, compiled and exec'd against seeded torch CPU tensors with a
    real PPObj agent (the scripts themselves cannot be imported: tyro, gymnasium, SB3, ocatari
    are not installed).

Fixtures:
  gae_{T}x{N}.npz     inputs + advantages/returns of the reference loop
  loss_{name}.npz     minibatch inputs, the actor/critic outputs (logits, value) and their
                      autograd grads, and the loss scalars, from the reference update block
  sample_{name}.npz   logits, the Exp(1) noise torch draws, and Categorical.sample()/log_prob/
                      entropy from PPObj.get_action_and_value under a fixed seed
  td_{name}.npz       dqn_atari_oc.py:378-382 (TD target, gathered Q, MSE loss) exec'd with stub
                      Q / target networks, plus d loss / d q by autograd
  ppobj_small.npz     a small PPObj's state_dict + input + reference outputs
  update_2mb[_cnn].npz two consecutive minibatch updates of the reference block :566-610 (forward,
                      loss, backward, clip_grad_norm_, Adam) on a small PPObj: the state_dict
                      before, after the first and after the second update, and both grad norms
  init_{name}.json    per-parameter checksums of seeded default-size agents + outputs on a fixed
                      input (pins layer order, state-dict keys and orthogonal init order)

    python tests/golden/gen_golden.py [update_config2 update_config3 ...]
"""
from __future__ import annotations

import json
import sys
import textwrap
import types
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
SCRIPT = REF / "cleanrl" / "ppo_atari_oc.py"
GAE_LINES = (533, 547)
UPDATE_LINES = (566, 610)
DQN_SCRIPT = REF / "cleanrl" / "dqn_atari_oc.py"
TD_LINES = (378, 382)
PPO_SCRIPT = REF / "cleanrl" / "ppo.py"
PPO_AGENT_LINES = (94, 126)   # layer_init + Agent (tanh-MLP actor / critic)
PPO_UPDATE_LINES = (250, 290)  # minibatch forward, loss, zero_grad, backward, clip, Adam
BUFFERS = REF / "cleanrl_utils" / "buffers.py"
REPLAY_METHOD_LINES = (379, 431)  # ReplayBuffer.add / sample / _get_samples (SB3 restatement)

sys.dont_write_bytecode = True
sys.path.insert(0, str(REF / "cleanrl"))
from architectures.ppo import PPODefault, PPObj  # noqa: E402  (the reference's own modules)


def block(lines, script=SCRIPT):
    src = script.read_text().splitlines()[lines[0] - 1:lines[1]]
    return compile(textwrap.dedent("\n".join(src)), f"{script}:{lines[0]}-{lines[1]}", "exec")


GAE_CODE = block(GAE_LINES)
UPDATE_CODE = block(UPDATE_LINES)
TD_CODE = block(TD_LINES, DQN_SCRIPT)
PPO_AGENT_CODE = block(PPO_AGENT_LINES, PPO_SCRIPT)
PPO_UPDATE_CODE = block(PPO_UPDATE_LINES, PPO_SCRIPT)


class Space:
    def __init__(self, shape=None, n=None):
        self.shape = shape
        self.n = n


class Envs:
    def __init__(self, obs_shape, n_actions):
        self.observation_space = Space(shape=obs_shape)
        self.action_space = Space(shape=(), n=n_actions)


# ---------------------------------------------------------------------------------------------
def gen_gae(T, N, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "jaxtest":  # the distributions of tests/test_jax_compute_gae.py:76-87
        dones = rng.integers(0, 2, (T, N)).astype(np.float32)
        values = rng.random((T, N), dtype=np.float32)
        rewards = rng.uniform(-1, 1, (T, N)).astype(np.float32)
        next_value = rng.random(N, dtype=np.float32)
        next_done = rng.integers(0, 2, N).astype(np.float32)
    else:  # synthetic Pong-like rollout
        u = rng.random((T, N))
        rewards = np.where(u < 0.005, 1.0, np.where(u < 0.01, -1.0, 0.0)).astype(np.float32)
        rewards = rewards + (rng.standard_normal((T, N)) * 0.05).astype(np.float32)
        dones = (rng.random((T, N)) < 0.02).astype(np.float32)
        values = (rng.standard_normal((T, N)) * 3).astype(np.float32)
        next_value = (rng.standard_normal(N) * 3).astype(np.float32)
        next_done = (rng.random(N) < 0.02).astype(np.float32)
    nv_t = torch.from_numpy(next_value)
    agent = types.SimpleNamespace(get_value=lambda x: nv_t.reshape(N, 1))
    args = types.SimpleNamespace(num_steps=T, gamma=0.99, gae_lambda=0.95)
    ns = dict(torch=torch, agent=agent, args=args, device="cpu", next_obs=None,
              rewards=torch.from_numpy(rewards), values=torch.from_numpy(values),
              dones=torch.from_numpy(dones), next_done=torch.from_numpy(next_done))
    exec(GAE_CODE, ns)
    np.savez_compressed(OUT / f"gae_{T}x{N}.npz", rewards=rewards, values=values, dones=dones,
                        next_value=next_value, next_done=next_done, gamma=0.99, gae_lambda=0.95,
                        advantages=ns["advantages"].numpy(), returns=ns["returns"].numpy())


# ---------------------------------------------------------------------------------------------
def gen_loss(name, *, norm_adv, clip_vloss, B=1024, M=256, F=6, A=6, seed=0, clip_coef=0.1,
             ties=False):
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    agent = PPObj(Envs((4, F), A), "cpu", (32, 64), (32,))
    b_obs = torch.from_numpy(rng.integers(0, 160, (B, 4, F)).astype(np.float32))
    with torch.no_grad():
        hid = agent.network(b_obs)
        lg = agent.actor(hid)
        val = agent.critic(hid).view(-1)
        dist = torch.distributions.Categorical(logits=lg)
        b_actions = dist.sample()
        lp = dist.log_prob(b_actions)
    spread = torch.from_numpy((rng.standard_normal(B) * 0.15).astype(np.float32))
    b_logprobs = lp + spread
    if ties:  # ratio == 1 exactly for a quarter of the batch: every max() ties there
        b_logprobs[: B // 4] = lp[: B // 4]
    b_values = val + torch.from_numpy((rng.standard_normal(B) * 0.3).astype(np.float32))
    b_returns = val + torch.from_numpy((rng.standard_normal(B) * 1.0).astype(np.float32))
    b_advantages = torch.from_numpy((rng.standard_normal(B) * 2.0).astype(np.float32))
    mb_inds = rng.permutation(B)[:M]

    captured = {}

    def grab(key):
        def hook(mod, inp, out):
            out.retain_grad()
            captured[key] = out
        return hook

    h1 = agent.actor.register_forward_hook(grab("logits"))
    h2 = agent.critic.register_forward_hook(grab("value"))
    args = types.SimpleNamespace(clip_coef=clip_coef, norm_adv=norm_adv, clip_vloss=clip_vloss,
                                 ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, track=False,
                                 minibatch_size=M)
    optimizer = optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    ns = dict(torch=torch, nn=nn, np=np, agent=agent, args=args, optimizer=optimizer,
              b_obs=b_obs, b_actions=b_actions, b_logprobs=b_logprobs,
              b_advantages=b_advantages, b_returns=b_returns, b_values=b_values,
              mb_inds=mb_inds, clipfracs=[], start=0)
    exec(UPDATE_CODE, ns)
    h1.remove()
    h2.remove()
    mba = b_advantages[mb_inds]
    stats = np.array([ns["loss"].item(), ns["pg_loss"].item(), ns["v_loss"].item(),
                      ns["entropy_loss"].item(), ns["old_approx_kl"].item(),
                      ns["approx_kl"].item(), ns["clipfracs"][-1],
                      mba.mean().item() if norm_adv else 0.0,
                      mba.std().item() if norm_adv else 0.0], np.float32)
    np.savez_compressed(
        OUT / f"loss_{name}.npz", logits=captured["logits"].detach().numpy(),
        new_value=captured["value"].detach().numpy().reshape(-1),
        dlogits=captured["logits"].grad.numpy(),
        dvalue=captured["value"].grad.numpy().reshape(-1), mb_inds=mb_inds.astype(np.int64),
        b_actions=b_actions.numpy().astype(np.int64), b_logprobs=b_logprobs.numpy(),
        b_advantages=b_advantages.numpy(), b_returns=b_returns.numpy(),
        b_values=b_values.numpy(), stats=stats, clip_coef=clip_coef, ent_coef=0.01, vf_coef=0.5,
        norm_adv=norm_adv, clip_vloss=clip_vloss, grad_norm=float(ns["gn"]))


# ---------------------------------------------------------------------------------------------
def gen_sample(name, N, A, F, seed):
    torch.manual_seed(1234)
    agent = PPObj(Envs((4, F), A), "cpu", (32, 64), (32,))
    # scale the actor up so the policy is far from uniform (more informative argmax cases)
    with torch.no_grad():
        agent.actor.weight.mul_(40.0)
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.integers(0, 160, (N, 4, F)).astype(np.float32))
    captured = {}
    h = agent.actor.register_forward_hook(lambda m, i, o: captured.__setitem__("logits", o))
    torch.manual_seed(seed)
    with torch.no_grad():
        action, logprob, entropy, value = agent.get_action_and_value(x)
    h.remove()
    torch.manual_seed(seed)
    noise = torch.empty((N, A), dtype=torch.float32).exponential_()
    np.savez_compressed(OUT / f"sample_{name}.npz", logits=captured["logits"].numpy(),
                        noise=noise.numpy(), action=action.numpy().astype(np.int64),
                        logprob=logprob.numpy(), entropy=entropy.numpy(),
                        value=value.numpy().reshape(-1))


# ---------------------------------------------------------------------------------------------
def gen_ppobj_small():
    torch.manual_seed(7)
    agent = PPObj(Envs((4, 6), 6), "cpu", (16, 32), (16,))
    rng = np.random.default_rng(7)
    x = torch.from_numpy(rng.integers(0, 160, (32, 4, 6)).astype(np.float32))
    with torch.no_grad():
        hid = agent.network(x)
        logits = agent.actor(hid)
        value = agent.get_value(x)
    sd = {f"sd::{k}": v.numpy() for k, v in agent.state_dict().items()}
    np.savez_compressed(OUT / "ppobj_small.npz", x=x.numpy(), logits=logits.numpy(),
                        value=value.numpy(), encoder_dims=np.array([16, 32]),
                        decoder_dims=np.array([16]), **sd)


def gen_init(name, ctor, obs_shape, A, seed, x_scale):
    torch.manual_seed(seed)
    agent = ctor(Envs(obs_shape, A))
    rng = np.random.default_rng(seed)
    x = torch.from_numpy((rng.random((4,) + obs_shape) * x_scale).astype(np.float32).round())
    with torch.no_grad():
        hid = agent.network(x)
        logits = agent.actor(hid)
        value = agent.critic(hid)
    info = {
        "seed": seed, "obs_shape": list(obs_shape), "n_actions": A, "x_scale": x_scale,
        "num_params": int(sum(p.numel() for p in agent.parameters())),
        "params": {k: {"shape": list(v.shape), "sum": float(v.double().sum()),
                       "abs_sum": float(v.double().abs().sum())}
                   for k, v in agent.state_dict().items()},
        "logits": logits.double().numpy().tolist(), "value": value.double().numpy().tolist(),
    }
    (OUT / f"init_{name}.json").write_text(json.dumps(info, indent=1))


def gen_td(name, B, A, seed):
    """dqn_atari_oc.py:378-382 with stub q / target networks returning seeded Q values."""
    rng = np.random.default_rng(seed)
    q = torch.from_numpy((rng.standard_normal((B, A)) * 2).astype(np.float32)).requires_grad_(True)
    q_next = torch.from_numpy((rng.standard_normal((B, A)) * 2).astype(np.float32))
    data = types.SimpleNamespace(
        observations=torch.zeros(B, 1), next_observations=torch.zeros(B, 1),
        actions=torch.from_numpy(rng.integers(0, A, (B, 1))),
        rewards=torch.from_numpy(rng.choice([-1.0, 0.0, 0.0, 0.0, 1.0], (B, 1)).astype(np.float32)),
        dones=torch.from_numpy((rng.random((B, 1)) < 0.2).astype(np.float32)))
    ns = dict(torch=torch, F=torch.nn.functional, data=data, args=types.SimpleNamespace(gamma=0.99),
              q_network=lambda x: q, target_network=lambda x: q_next)
    exec(TD_CODE, ns)
    ns["loss"].backward()
    np.savez_compressed(OUT / f"td_{name}.npz", q=q.detach().numpy(), q_next=q_next.numpy(),
                        actions=data.actions.numpy().reshape(-1), rewards=data.rewards.numpy().reshape(-1),
                        dones=data.dones.numpy().reshape(-1), gamma=0.99,
                        td_target=ns["td_target"].numpy(), loss=ns["loss"].item(),
                        q_values=ns["old_val"].mean().item(), dq=q.grad.numpy())


def gen_update(B=512, M=256, F=6, A=6, seed=21, pixels=False, name="update_2mb", enc=(32, 64),
               dec=(32,)):
    """Two minibatch updates (one epoch of 2 minibatches) through the reference's update block,
    with its Adam (lr 2.5e-4, eps 1e-5) and clip_grad_norm_(0.5): the whole learner step.
    pixels: the NatureCNN (PPODefault) on u8-valued 4x84x84 stacks instead of a small PPObj."""
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    if pixels:
        agent = PPODefault(Envs((4, 84, 84), A), "cpu")
        b_obs = torch.from_numpy(rng.integers(0, 256, (B, 4, 84, 84)).astype(np.float32))
    else:
        agent = PPObj(Envs((4, F), A), "cpu", enc, dec)
        b_obs = torch.from_numpy(rng.integers(0, 160, (B, 4, F)).astype(np.float32))
    with torch.no_grad():
        hid = agent.network(b_obs)
        dist = torch.distributions.Categorical(logits=agent.actor(hid))
        b_actions = dist.sample()
        lp = dist.log_prob(b_actions)
        val = agent.critic(hid).view(-1)
    b_logprobs = lp + torch.from_numpy((rng.standard_normal(B) * 0.15).astype(np.float32))
    b_values = val + torch.from_numpy((rng.standard_normal(B) * 0.3).astype(np.float32))
    b_returns = val + torch.from_numpy((rng.standard_normal(B) * 1.0).astype(np.float32))
    b_advantages = torch.from_numpy((rng.standard_normal(B) * 2.0).astype(np.float32))
    perm = rng.permutation(B)
    args = types.SimpleNamespace(clip_coef=0.1, norm_adv=True, clip_vloss=True, ent_coef=0.01,
                                 vf_coef=0.5, max_grad_norm=0.5, track=False, minibatch_size=M)
    optimizer = optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    sds = [{k: v.detach().clone().numpy() for k, v in agent.state_dict().items()}]
    gns = []
    for start in (0, M):
        ns = dict(torch=torch, nn=nn, np=np, agent=agent, args=args, optimizer=optimizer,
                  b_obs=b_obs, b_actions=b_actions, b_logprobs=b_logprobs,
                  b_advantages=b_advantages, b_returns=b_returns, b_values=b_values,
                  mb_inds=perm[start:start + M], clipfracs=[], start=start)
        exec(UPDATE_CODE, ns)
        gns.append(float(ns["gn"]))
        sds.append({k: v.detach().clone().numpy() for k, v in agent.state_dict().items()})
    out = dict(b_obs=b_obs.numpy(), b_actions=b_actions.numpy().astype(np.int64),
               b_logprobs=b_logprobs.numpy(), b_values=b_values.numpy(),
               b_returns=b_returns.numpy(), b_advantages=b_advantages.numpy(),
               perm=perm.astype(np.int64), M=M, grad_norms=np.array(gns, np.float64))
    big = 1 << 16  # parameters above this size: a fixed sample of elements (keeps the file small)
    pick = {}
    for i, sd in enumerate(sds):
        for k, v in sd.items():
            if pixels and i == 0:  # sd0 is the seeded init: checksums only (the test re-creates it)
                out[f"sum0::{k}"] = np.array([v.astype(np.float64).sum(),
                                              (v.astype(np.float64) ** 2).sum()])
                continue
            if v.size > big:
                if k not in pick:
                    pick[k] = np.sort(rng.choice(v.size, 4096, replace=False)).astype(np.int64)
                    out[f"pick::{k}"] = pick[k]
                out[f"sd{i}::{k}"] = v.reshape(-1)[pick[k]]
            else:
                out[f"sd{i}::{k}"] = v
    if pixels:
        out["b_obs"] = b_obs.numpy().astype(np.uint8)  # exact: integer pixel values
    np.savez_compressed(OUT / f"{name}.npz", **out)


def config2_weights(agent, seed):
    """Seeded PPObj parameters from numpy's PCG64 stream (platform-independent, so the GPU test
    re-creates them bit for bit without shipping 9 MB of weights; a CPU orthogonal_ init would
    differ in the last bits between LAPACK builds): weight [out, in] ~ N(0, 1) * gain / sqrt(in)
    with layer_init's gains (sqrt 2 network, 0.01 actor, 1 critic), bias ~ N(0, 1) * 0.05, in
    state_dict order. The update block does not care how the weights were made."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, v in agent.state_dict().items():
        if k.endswith("weight"):
            gain = 0.01 if k.startswith("actor") else 1.0 if k.startswith("critic") else 2 ** 0.5
            w = rng.standard_normal(tuple(v.shape)) * (gain / np.sqrt(v.shape[1]))
        else:
            w = rng.standard_normal(tuple(v.shape)) * 0.05
        sd[k] = torch.from_numpy(w.astype(np.float32))
    return sd


def gen_update_config2(T=128, N=128, F=12, A=6, W=4, seed=25, name="update_config2"):
    """BASELINE config 2 at the network's real size: PPObj(encoder (256, 512, 1024, 512),
    decoder (512,)) on a rollout-structured batch of T x N = 128 x 128 Pong-obj samples, and two
    minibatch updates of 4096 through the reference's update block (ppo_atari_oc.py:566-610).

    The rollout obeys the frame-stack rule the trainer's frame dedup relies on: obs [T+1, N, W, F]
    with obs[t] = obs[t-1] shifted by env n's frame of step t, or W copies of it where
    dones[t, n] (FrameStack's reset fill; obs[0] likewise where dones[0, n]). Features: x U{0..159},
    y U{0..209}, w, h U{1..16} (integers: exact in bf16 storage). Actions and log-probs
    are the reference agent's own samples, values its critic (+ noise), rewards sparse +-1, and
    advantages / returns come from the reference's GAE block (:533-547) with bootstrap
    V(obs[T]). Stored: inputs, the 2 x 4096 permutation, per-minibatch loss scalars and grad
    norms, the parameters after each update (tensors above 64K elements as 4096 fixed samples)
    and checksums of the seeded initial ones (config2_weights)."""
    rng = np.random.default_rng(seed)
    hi = np.array([160, 210, 17, 17] * (F // 4))
    lo = np.array([0, 0, 1, 1] * (F // 4))

    def frames(n):
        return rng.integers(lo, hi, (n, F)).astype(np.float32)

    dones = (rng.random((T + 1, N)) < 0.02).astype(np.float32)
    obs = np.zeros((T + 1, N, W, F), np.float32)
    obs[0] = rng.integers(lo, hi, (N, W, F))
    obs[0][dones[0] != 0] = obs[0][dones[0] != 0][:, -1:, :]
    for t in range(1, T + 1):
        f = frames(N)
        obs[t] = np.concatenate([obs[t - 1][:, 1:], f[:, None]], 1)
        d = dones[t] != 0
        obs[t][d] = f[d][:, None, :]
    agent = PPObj(Envs((W, F), A), "cpu", (256, 512, 1024, 512), (512,))
    sd0 = config2_weights(agent, seed)
    agent.load_state_dict(sd0)
    b_obs = torch.from_numpy(obs[:T].reshape(T * N, W, F))
    torch.manual_seed(seed)
    with torch.no_grad():
        hid = agent.network(b_obs)
        dist = torch.distributions.Categorical(logits=agent.actor(hid))
        b_actions = dist.sample()
        lp = dist.log_prob(b_actions)
        val = agent.critic(hid).view(-1)
        next_value = agent.critic(agent.network(torch.from_numpy(obs[T]))).view(-1)
    u = rng.random((T, N))
    rewards = np.where(u < 0.005, 1.0, np.where(u < 0.01, -1.0, 0.0)).astype(np.float32)
    values = (val + torch.from_numpy((rng.standard_normal(T * N) * 0.3).astype(np.float32)))
    values = values.view(T, N).contiguous()
    nv = next_value.reshape(N)
    ns = dict(torch=torch, agent=types.SimpleNamespace(get_value=lambda x: nv.reshape(1, N)),
              args=types.SimpleNamespace(num_steps=T, gamma=0.99, gae_lambda=0.95),
              device="cpu", next_obs=None, rewards=torch.from_numpy(rewards), values=values,
              dones=torch.from_numpy(dones[:T]), next_done=torch.from_numpy(dones[T]))
    exec(GAE_CODE, ns)
    b_advantages = ns["advantages"].reshape(-1)
    b_returns = ns["returns"].reshape(-1)
    b_values = values.reshape(-1)
    b_logprobs = lp + torch.from_numpy((rng.standard_normal(T * N) * 0.15).astype(np.float32))
    B, M = T * N, T * N // 4
    perm = rng.permutation(B)
    args = types.SimpleNamespace(clip_coef=0.1, norm_adv=True, clip_vloss=True, ent_coef=0.01,
                                 vf_coef=0.5, max_grad_norm=0.5, track=False, minibatch_size=M)
    optimizer = optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    sds = [{k: v.detach().clone().numpy() for k, v in agent.state_dict().items()}]
    gns, stats, grads, pre32 = [], [], [], []
    for start in (0, M):
        mb_inds = perm[start:start + M]
        ns = dict(torch=torch, nn=_recording_nn(agent, pre32), np=np, agent=agent, args=args,
                  optimizer=optimizer, b_obs=b_obs, b_actions=b_actions, b_logprobs=b_logprobs,
                  b_advantages=b_advantages, b_returns=b_returns, b_values=b_values,
                  mb_inds=mb_inds, clipfracs=[], start=start)
        exec(UPDATE_CODE, ns)
        gns.append(float(ns["gn"]))
        # the gradients the optimizer saw (after clip_grad_norm_): per-tensor norms + samples
        grads.append({k: p.grad.detach().clone().numpy() for k, p in agent.named_parameters()})
        mba = b_advantages[mb_inds]
        stats.append([ns["loss"].item(), ns["pg_loss"].item(), ns["v_loss"].item(),
                      ns["entropy_loss"].item(), ns["old_approx_kl"].item(),
                      ns["approx_kl"].item(), ns["clipfracs"][-1], mba.mean().item(),
                      mba.std().item()])
        sds.append({k: v.detach().clone().numpy() for k, v in agent.state_dict().items()})
    out = dict(obs=obs.astype(np.uint8), dones=dones, actions=b_actions.numpy().astype(np.int64),
               logprobs=b_logprobs.numpy(), values=b_values.numpy(), rewards=rewards,
               next_value=nv.numpy(), advantages=b_advantages.numpy(),
               returns=b_returns.numpy(), perm=perm[:2 * M].astype(np.int64), M=M, seed=seed,
               grad_norms=np.array(gns, np.float64), stats=np.array(stats, np.float32))
    assert np.array_equal(out["obs"].astype(np.float32), obs)
    pick_rng = np.random.default_rng(seed + 1)
    for k, v in sds[0].items():
        v64 = v.astype(np.float64)
        out[f"sum0::{k}"] = np.array([v64.sum(), (v64 ** 2).sum()])
    for i, sd in enumerate(sds[1:], 1):
        for k, v in sd.items():
            if v.size > (1 << 16):
                if f"pick::{k}" not in out:
                    out[f"pick::{k}"] = np.sort(pick_rng.choice(v.size, 4096, replace=False))
                out[f"sd{i}::{k}"] = v.reshape(-1)[out[f"pick::{k}"]]
            else:
                out[f"sd{i}::{k}"] = v
    for i, gd in enumerate(grads):
        for k, v in gd.items():
            out[f"gnorm{i}::{k}"] = np.array([np.linalg.norm(v.astype(np.float64)),
                                             np.abs(v).max()])
            out[f"grad{i}::{k}"] = (v.reshape(-1)[out[f"pick::{k}"]] if f"pick::{k}" in out
                                   else v)
    # f64 twin: the same update block on the same inputs in float64, at the reference's own f32
    # parameters before each minibatch (so minibatch 1 is evaluated where the f32 reference
    # evaluated it); stored are the PRE-clip gradients of both runs (the f32 reference's own,
    # recorded as clip_grad_norm_ received them) and the f64 grad norms. The gap f32 -> f64 is
    # the reference's own rounding, the yardstick of the GPU chain's per-tensor check.
    agent64 = PPObj(Envs((W, F), A), "cpu", (256, 512, 1024, 512), (512,)).double()
    f64 = lambda t: t.double()  # noqa: E731
    for i, start in enumerate((0, M)):
        agent64.load_state_dict({k: torch.from_numpy(v).double() for k, v in sds[i].items()})
        pre64 = []
        ns = dict(torch=torch, nn=_recording_nn(agent64, pre64), np=np, agent=agent64, args=args,
                  optimizer=optim.Adam(agent64.parameters(), lr=2.5e-4, eps=1e-5),
                  b_obs=f64(b_obs), b_actions=b_actions, b_logprobs=f64(b_logprobs),
                  b_advantages=f64(b_advantages), b_returns=f64(b_returns),
                  b_values=f64(b_values), mb_inds=perm[start:start + M], clipfracs=[],
                  start=start)
        exec(UPDATE_CODE, ns)
        out[f"grad_norm64_{i}"] = np.array(float(ns["gn"]))
        for k, v in pre64[0].items():
            out[f"gnorm64pre{i}::{k}"] = np.array([np.linalg.norm(v), np.abs(v).max()])
            pk = out.get(f"pick::{k}")
            out[f"grad64pre{i}::{k}"] = v.reshape(-1)[pk] if pk is not None else v
            v32 = pre32[i][k]
            out[f"gradpre{i}::{k}"] = v32.reshape(-1)[pk] if pk is not None else v32
    np.savez_compressed(OUT / f"{name}.npz", **out)


def _recording_nn(agent, record):
    """`nn` for an exec'd update block whose clip_grad_norm_ first records every parameter's
    gradient as it stands (pre-clip), then runs torch's own clip: numerics untouched."""
    def clip_grad_norm_(params, max_norm, *a, **kw):
        record.append({k: p.grad.detach().clone().numpy() for k, p in agent.named_parameters()})
        return nn.utils.clip_grad_norm_(params, max_norm, *a, **kw)

    return types.SimpleNamespace(utils=types.SimpleNamespace(clip_grad_norm_=clip_grad_norm_))


def config3_weights(agent, seed):
    """config2_weights for any layer shape: weight ~ N(0, 1) * gain / sqrt(fan_in), fan_in =
    in x kh x kw for a convolution (the NatureCNN of config 3), numpy PCG64, state_dict order."""
    rng = np.random.default_rng(seed)
    sd = {}
    for k, v in agent.state_dict().items():
        if k.endswith("weight"):
            gain = 0.01 if k.startswith("actor") else 1.0 if k.startswith("critic") else 2 ** 0.5
            w = rng.standard_normal(tuple(v.shape)) * (gain / np.sqrt(np.prod(v.shape[1:])))
        else:
            w = rng.standard_normal(tuple(v.shape)) * 0.05
        sd[k] = torch.from_numpy(w.astype(np.float32))
    return sd


def breakout_frames(rng, n):
    """n synthetic 84x84 u8 Breakout-like frames: a brick wall (rows of 6 gray levels, a random
    subset of bricks knocked out), a paddle and a ball at random places, black elsewhere."""
    f = np.zeros((n, 84, 84), np.uint8)
    levels = np.array([200, 180, 160, 140, 120, 100], np.uint8)
    for r in range(6):
        keep = rng.random((n, 14)) < 0.8
        row = np.repeat(np.where(keep, levels[r], 0).astype(np.uint8), 6, axis=1)
        f[:, 18 + 3 * r:21 + 3 * r, :] = row[:, None, :]
    px = rng.integers(0, 76, n)
    bx, by = rng.integers(0, 82, n), rng.integers(30, 76, n)
    for i in range(n):
        f[i, 78:80, px[i]:px[i] + 8] = 144
        f[i, by[i]:by[i] + 2, bx[i]:bx[i] + 2] = 236
    return f


def gen_update_config3(T=16, N=256, A=4, W=4, seed=27, name="update_config3"):
    """BASELINE config 3's network at its minibatch size: PPODefault (NatureCNN, 84x84x4,
    NormalizeImg) on a rollout-structured batch of T x N = 16 x 256 synthetic Breakout frame
    stacks (the frame-stack rule with resets, as in gen_update_config2), and two minibatch
    updates of 2048 through the reference's update block (ppo_atari_oc.py:566-610). Stored: the
    distinct frames [T+W, N, 84, 84] u8 and the dones (the test rebuilds the stacks), actions /
    log-probs / values / rewards, GAE advantages / returns from the reference block (:533-547),
    the permutation, per-minibatch loss scalars and grad norms, pre-clip gradients of the f32
    reference and of its float64 twin at the same parameters, and the parameters after each
    update (tensors above 16K elements as 4096 fixed samples)."""
    rng = np.random.default_rng(seed)
    # timeline row s + W - 1 = env n's frame of step s, s in [-(W-1), T]
    frames = breakout_frames(rng, (T + W) * N).reshape(T + W, N, 84, 84)
    dones = (rng.random((T + 1, N)) < 0.02).astype(np.float32)
    obs = np.zeros((T + 1, N, W, 84, 84), np.uint8)
    # obs[t] slot w = the frame of step t - (W-1) + w (timeline row t + w), clipped to the
    # latest reset: a reset at step t fills every slot with that step's frame
    last_reset = np.full(N, -10 ** 9)
    for t in range(T + 1):
        last_reset = np.where(dones[t] != 0, t, last_reset)
        for w in range(W):
            src = np.maximum(t - (W - 1) + w, last_reset)  # step whose frame fills the slot
            obs[t, :, w] = frames[src + W - 1, np.arange(N)]
    agent = PPODefault(Envs((W, 84, 84), A), "cpu")
    sd0 = config3_weights(agent, seed)
    agent.load_state_dict(sd0)
    B, M = T * N, T * N // 2
    b_obs = torch.from_numpy(obs[:T].reshape(B, W, 84, 84).astype(np.float32))
    torch.manual_seed(seed)
    with torch.no_grad():
        hid = agent.network(b_obs)
        dist = torch.distributions.Categorical(logits=agent.actor(hid))
        b_actions = dist.sample()
        lp = dist.log_prob(b_actions)
        val = agent.critic(hid).view(-1)
        next_value = agent.critic(agent.network(torch.from_numpy(
            obs[T].astype(np.float32)))).view(-1)
    u = rng.random((T, N))
    rewards = np.where(u < 0.02, 1.0, 0.0).astype(np.float32)
    values = (val + torch.from_numpy((rng.standard_normal(B) * 0.3).astype(np.float32)))
    values = values.view(T, N).contiguous()
    nv = next_value.reshape(N)
    ns = dict(torch=torch, agent=types.SimpleNamespace(get_value=lambda x: nv.reshape(1, N)),
              args=types.SimpleNamespace(num_steps=T, gamma=0.99, gae_lambda=0.95),
              device="cpu", next_obs=None, rewards=torch.from_numpy(rewards), values=values,
              dones=torch.from_numpy(dones[:T]), next_done=torch.from_numpy(dones[T]))
    exec(GAE_CODE, ns)
    b_advantages = ns["advantages"].reshape(-1)
    b_returns = ns["returns"].reshape(-1)
    b_values = values.reshape(-1)
    b_logprobs = lp + torch.from_numpy((rng.standard_normal(B) * 0.15).astype(np.float32))
    perm = rng.permutation(B)
    args = types.SimpleNamespace(clip_coef=0.1, norm_adv=True, clip_vloss=True, ent_coef=0.01,
                                 vf_coef=0.5, max_grad_norm=0.5, track=False, minibatch_size=M)
    optimizer = optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    sds = [{k: v.detach().clone().numpy() for k, v in agent.state_dict().items()}]
    gns, stats, pre32 = [], [], []
    for start in (0, M):
        mb_inds = perm[start:start + M]
        ns = dict(torch=torch, nn=_recording_nn(agent, pre32), np=np, agent=agent, args=args,
                  optimizer=optimizer, b_obs=b_obs, b_actions=b_actions, b_logprobs=b_logprobs,
                  b_advantages=b_advantages, b_returns=b_returns, b_values=b_values,
                  mb_inds=mb_inds, clipfracs=[], start=start)
        exec(UPDATE_CODE, ns)
        gns.append(float(ns["gn"]))
        mba = b_advantages[mb_inds]
        stats.append([ns["loss"].item(), ns["pg_loss"].item(), ns["v_loss"].item(),
                      ns["entropy_loss"].item(), ns["old_approx_kl"].item(),
                      ns["approx_kl"].item(), ns["clipfracs"][-1], mba.mean().item(),
                      mba.std().item()])
        sds.append({k: v.detach().clone().numpy() for k, v in agent.state_dict().items()})
    out = dict(frames=frames, dones=dones, actions=b_actions.numpy().astype(np.int64),
               logprobs=b_logprobs.numpy(), values=b_values.numpy(), rewards=rewards,
               next_value=nv.numpy(), advantages=b_advantages.numpy(),
               returns=b_returns.numpy(), perm=perm.astype(np.int64), M=M, seed=seed,
               grad_norms=np.array(gns, np.float64), stats=np.array(stats, np.float32),
               obs_sum=np.array(obs.astype(np.int64).sum()))
    pick_rng = np.random.default_rng(seed + 1)
    for k, v in sds[0].items():
        v64 = v.astype(np.float64)
        out[f"sum0::{k}"] = np.array([v64.sum(), (v64 ** 2).sum()])
        if v.size > (1 << 14):
            out[f"pick::{k}"] = np.sort(pick_rng.choice(v.size, 4096, replace=False))
    for i, sd in enumerate(sds[1:], 1):
        for k, v in sd.items():
            pk = out.get(f"pick::{k}")
            out[f"sd{i}::{k}"] = v.reshape(-1)[pk] if pk is not None else v
    agent64 = PPODefault(Envs((W, 84, 84), A), "cpu").double()
    f64 = lambda t: t.double()  # noqa: E731
    for i, start in enumerate((0, M)):
        agent64.load_state_dict({k: torch.from_numpy(v).double() for k, v in sds[i].items()})
        pre64 = []
        ns = dict(torch=torch, nn=_recording_nn(agent64, pre64), np=np, agent=agent64, args=args,
                  optimizer=optim.Adam(agent64.parameters(), lr=2.5e-4, eps=1e-5),
                  b_obs=f64(b_obs), b_actions=b_actions, b_logprobs=f64(b_logprobs),
                  b_advantages=f64(b_advantages), b_returns=f64(b_returns),
                  b_values=f64(b_values), mb_inds=perm[start:start + M], clipfracs=[],
                  start=start)
        exec(UPDATE_CODE, ns)
        out[f"grad_norm64_{i}"] = np.array(float(ns["gn"]))
        for k, v in pre64[0].items():
            out[f"gnorm64pre{i}::{k}"] = np.array([np.linalg.norm(v), np.abs(v).max()])
            pk = out.get(f"pick::{k}")
            out[f"grad64pre{i}::{k}"] = v.reshape(-1)[pk] if pk is not None else v
            v32 = pre32[i][k]
            out[f"gradpre{i}::{k}"] = v32.reshape(-1)[pk] if pk is not None else v32
    np.savez_compressed(OUT / f"{name}.npz", **out)


def gen_update_cartpole(B=512, M=128, seed=23, name="update_cartpole"):
    """Config 1: two minibatch updates of cleanrl/ppo.py's own update block (:250-290, clip 0.2)
    on its own Agent class (:94-126, exec'd), the whole learner step of ppo.py on CartPole-shaped
    observations."""
    from torch.distributions.categorical import Categorical

    ns_agent = dict(torch=torch, nn=nn, np=np, Categorical=Categorical)
    exec(PPO_AGENT_CODE, ns_agent)
    envs = types.SimpleNamespace(single_observation_space=Space(shape=(4,)),
                                 single_action_space=Space(shape=(), n=2))
    torch.manual_seed(seed)
    rng = np.random.default_rng(seed)
    agent = ns_agent["Agent"](envs)
    b_obs = torch.from_numpy((rng.uniform(-1, 1, (B, 4)) * [2.0, 1.5, 0.2, 1.5]).astype(np.float32))
    with torch.no_grad():
        b_actions, lp, _, val = agent.get_action_and_value(b_obs)
        val = val.view(-1)
    b_logprobs = lp + torch.from_numpy((rng.standard_normal(B) * 0.1).astype(np.float32))
    b_values = val + torch.from_numpy((rng.standard_normal(B) * 0.3).astype(np.float32))
    b_returns = val + torch.from_numpy((rng.standard_normal(B) * 2.0).astype(np.float32))
    b_advantages = torch.from_numpy((rng.standard_normal(B) * 1.5).astype(np.float32))
    perm = rng.permutation(B)
    args = types.SimpleNamespace(clip_coef=0.2, norm_adv=True, clip_vloss=True, ent_coef=0.01,
                                 vf_coef=0.5, max_grad_norm=0.5)
    optimizer = optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    sds = [{k: v.detach().clone().numpy() for k, v in agent.state_dict().items()}]
    stats = []
    for start in (0, M):
        ns = dict(torch=torch, nn=nn, np=np, agent=agent, args=args, optimizer=optimizer,
                  b_obs=b_obs, b_actions=b_actions.float(), b_logprobs=b_logprobs,
                  b_advantages=b_advantages, b_returns=b_returns, b_values=b_values,
                  mb_inds=perm[start:start + M], clipfracs=[])
        exec(PPO_UPDATE_CODE, ns)
        stats.append([ns["loss"].item(), ns["pg_loss"].item(), ns["v_loss"].item(),
                      ns["entropy_loss"].item(), ns["old_approx_kl"].item(),
                      ns["approx_kl"].item(), ns["clipfracs"][-1]])
        sds.append({k: v.detach().clone().numpy() for k, v in agent.state_dict().items()})
    out = dict(b_obs=b_obs.numpy(), b_actions=b_actions.numpy().astype(np.int64),
               b_logprobs=b_logprobs.numpy(), b_values=b_values.numpy(),
               b_returns=b_returns.numpy(), b_advantages=b_advantages.numpy(),
               perm=perm.astype(np.int64), M=M, stats=np.array(stats, np.float32))
    for i, sd in enumerate(sds):
        for k, v in sd.items():
            out[f"sd{i}::{k}"] = v
    np.savez_compressed(OUT / f"{name}.npz", **out)


def gen_replay(size=7, obs_shape=(4, 5), adds=10, seed=31, name="replay_sb3"):
    """SB3 ReplayBuffer(optimize_memory_usage=True) as the reference holds it
    (cleanrl_utils/buffers.py:379-431: add, sample, _get_samples), exec'd as the body of a class
    over a stub base that provides the state __init__ would build (:337-363; the module itself
    imports gym / SB3, absent here). Records the buffer after every add (wrap-around included),
    _get_samples for every slot, and the index support of sample() at a not-full and a full
    state (sample's own np.random.randint law, :412-415)."""
    import collections
    from typing import Optional

    lines = BUFFERS.read_text().splitlines()[REPLAY_METHOD_LINES[0] - 1:REPLAY_METHOD_LINES[1]]
    src = "class RB(Base):\n" + "\n".join(lines)

    class Base:
        def __init__(self, buffer_size, obs_shape, n_envs=1):
            self.buffer_size, self.n_envs, self.pos, self.full = buffer_size, n_envs, 0, False
            self.optimize_memory_usage = True
            self.observations = np.zeros((buffer_size, n_envs) + obs_shape, np.uint8)
            self.next_observations = None
            self.actions = np.zeros((buffer_size, n_envs, 1), np.int64)
            self.rewards = np.zeros((buffer_size, n_envs), np.float32)
            self.dones = np.zeros((buffer_size, n_envs), np.float32)

        @staticmethod
        def _normalize_obs(obs, env=None):
            return obs

        @staticmethod
        def _normalize_reward(reward, env=None):
            return reward

        def to_torch(self, array, copy=True):
            return np.array(array)

    Samples = collections.namedtuple("ReplayBufferSamples", "observations actions "
                                     "next_observations dones rewards")
    ns = dict(np=np, Optional=Optional, VecNormalize=object, ReplayBufferSamples=Samples,
              Base=Base)
    exec(compile(src, f"{BUFFERS}:{REPLAY_METHOD_LINES[0]}-{REPLAY_METHOD_LINES[1]}", "exec"), ns)
    rb = ns["RB"](size, obs_shape)
    rng = np.random.default_rng(seed)
    out = {"size": size}
    ins = {k: [] for k in ("obs", "next_obs", "action", "reward", "done")}
    snaps = {k: [] for k in ("pos", "full", "observations", "actions", "rewards", "dones")}
    support = {}
    for t in range(adds):
        o = rng.integers(0, 256, (1,) + obs_shape).astype(np.uint8)
        no = rng.integers(0, 256, (1,) + obs_shape).astype(np.uint8)
        a = rng.integers(0, 6, (1, 1))
        r = rng.standard_normal(1).astype(np.float32)
        d = (rng.random(1) < 0.3).astype(np.float32)
        rb.add(o, no, a, r, d)
        for k, v in zip(ins, (o, no, a, r, d)):
            ins[k].append(v)
        snaps["pos"].append(rb.pos)
        snaps["full"].append(rb.full)
        for k in ("observations", "actions", "rewards", "dones"):
            snaps[k].append(getattr(rb, k).copy())
        if t in (2, adds - 1):  # not full (pos = 3), full (pos = adds - size)
            get = rb._get_samples
            rb._get_samples = lambda inds, env=None: inds  # sample() returns its batch_inds
            np.random.seed(seed + t)
            inds = rb.sample(20000)
            del rb._get_samples
            assert get is not None
            support[t] = np.unique(inds)
    every = rb._get_samples(np.arange(size))
    for k, v in ins.items():
        out[f"in_{k}"] = np.stack(v)
    for k, v in snaps.items():
        out[f"after_{k}"] = np.array(v)
    for k in Samples._fields:
        out[f"get_{k}"] = getattr(every, k)
    for t, v in support.items():
        out[f"support_{t}"] = v
    np.savez_compressed(OUT / f"{name}.npz", **out)


def main():
    torch.set_num_threads(8)
    if sys.argv[1:]:  # just the named fixtures, e.g. update_config2 update_config3
        for n in sys.argv[1:]:
            globals()[f"gen_{n}"]()
        return
    gen_gae(16, 8, "synthetic", 1)
    gen_gae(123, 7, "jaxtest", 42)
    gen_gae(128, 128, "synthetic", 2)
    gen_loss("norm_clip", norm_adv=True, clip_vloss=True, seed=0)
    gen_loss("nonorm_clip", norm_adv=False, clip_vloss=True, seed=1)
    gen_loss("norm_noclip", norm_adv=True, clip_vloss=False, seed=2)
    gen_loss("nonorm_noclip", norm_adv=False, clip_vloss=False, seed=3)
    gen_loss("ties", norm_adv=True, clip_vloss=True, seed=4, ties=True)
    gen_loss("cartpole_c02", norm_adv=True, clip_vloss=True, seed=5, F=4, A=2, clip_coef=0.2,
             B=512, M=128)
    gen_loss("a18", norm_adv=True, clip_vloss=True, seed=6, A=18)
    gen_sample("n128_a6", 128, 6, 12, 42)
    gen_sample("n256_a4", 256, 4, 6, 43)
    gen_sample("n64_a18", 64, 18, 6, 44)
    gen_td("b32_a6", 32, 6, 11)
    gen_td("b256_a18", 256, 18, 12)
    gen_ppobj_small()
    gen_update()
    gen_update(B=32, M=16, A=4, seed=22, pixels=True, name="update_2mb_cnn")
    gen_update_cartpole()
    gen_replay()
    # decoder width 64: the fused heads + loss + heads-backward kernel's shapes (H % 64 == 0)
    gen_update(seed=24, name="update_2mb_h64", enc=(32, 64), dec=(64,))
    gen_init("ppobj_f12_a6", lambda e: PPObj(e, "cpu", (256, 512, 1024, 512), (512,)), (4, 12), 6,
             1, 160.0)
    gen_init("ppodefault_a4", lambda e: PPODefault(e, "cpu"), (4, 84, 84), 4, 1, 255.0)
    # config 2 at the real network dims, rollout-structured (the bench's update chain)
    gen_update_config2()
    # config 3's NatureCNN at a real minibatch size (2048), rollout-structured pixel stacks
    gen_update_config3()
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
