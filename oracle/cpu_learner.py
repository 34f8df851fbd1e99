"""ORACLE — CPU port of the reference PPO iteration (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Restates cleanrl/ppo_atari_oc.py:469-617 op for op on CPU torch (the reference's own device path
with device="cpu"): rollout storage tensors, per-step `agent.get_action_and_value` with
torch.distributions.Categorical, host float32 conversions of env outputs, the reverse GAE loop,
np.random.shuffle minibatches, the clipped PPO loss, backward, clip_grad_norm_ and Adam. The
agent is the PPObj / NatureCNN architecture of cleanrl/architectures/ppo.py:15-95 built from plain
torch.nn here; the env is the oracle restatement of the synthetic env (ocppo_oracle.synth_env_step)
with SB3-VecNormalize reward scaling (ocppo_oracle.vecnorm_reward).

Used by bench.py's `cpu_baseline` leg: it times this loop on the GPU box's host cores.
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn as nn
from torch.distributions.categorical import Categorical

from . import ocppo_oracle as O


def _init(layer, std=np.sqrt(2)):
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, 0.0)
    return layer


class CpuPPObj(nn.Module):
    def __init__(self, obs_shape, n_actions, enc=(256, 512, 1024, 512), dec=(512,)):
        super().__init__()
        layers, d = [], obs_shape[-1]
        for l in enc:
            layers += [_init(nn.Linear(d, l)), nn.ReLU()]
            d = l
        layers.append(nn.Flatten())
        d *= int(np.prod(obs_shape[:-1]))
        for l in dec:
            layers += [_init(nn.Linear(d, l)), nn.ReLU()]
            d = l
        self.network = nn.Sequential(*layers)
        self.actor = _init(nn.Linear(d, n_actions), 0.01)
        self.critic = _init(nn.Linear(d, 1), 1)

    def get_value(self, x):
        return self.critic(self.network(x))

    def get_action_and_value(self, x, action=None):
        h = self.network(x)
        probs = Categorical(logits=self.actor(h))
        if action is None:
            action = probs.sample()
        return action, probs.log_prob(action), probs.entropy(), self.critic(h)


class CpuNatureCNN(nn.Module):
    """PPODefault (cleanrl/architectures/ppo.py:15-57): x/255, 3 convs, Linear(3136, 512)."""

    def __init__(self, n_actions, window=4):
        super().__init__()
        self.network = nn.Sequential(
            _init(nn.Conv2d(window, 32, 8, stride=4)), nn.ReLU(),
            _init(nn.Conv2d(32, 64, 4, stride=2)), nn.ReLU(),
            _init(nn.Conv2d(64, 64, 3, stride=1)), nn.ReLU(), nn.Flatten(),
            _init(nn.Linear(64 * 7 * 7, 512)), nn.ReLU())
        self.actor = _init(nn.Linear(512, n_actions), 0.01)
        self.critic = _init(nn.Linear(512, 1), 1)

    def get_value(self, x):
        return self.critic(self.network(x / 255.0))

    def get_action_and_value(self, x, action=None):
        h = self.network(x / 255.0)
        probs = Categorical(logits=self.actor(h))
        if action is None:
            action = probs.sample()
        return action, probs.log_prob(action), probs.entropy(), self.critic(h)


class CpuLearner:
    """One process, `num_envs` synthetic envs (Pong obj vectors, or 84x84 pixel stacks with the
    NatureCNN when pixels=True), reference hyper-parameters."""

    def __init__(self, num_envs=128, num_steps=128, num_features=12, n_actions=6, seed=42,
                 num_minibatches=4, update_epochs=4, window=4, pixels=False):
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.pixels = pixels
        if pixels:
            num_features = 84 * 84
        self.N, self.T, self.F, self.A, self.W = num_envs, num_steps, num_features, n_actions, window
        self.obs_shape = (window, 84, 84) if pixels else (window, num_features)
        self.agent = CpuNatureCNN(n_actions, window) if pixels else \
            CpuPPObj(self.obs_shape, n_actions)
        self.opt = torch.optim.Adam(self.agent.parameters(), lr=2.5e-4, eps=1e-5)
        self.nmb, self.E = num_minibatches, update_epochs
        self.seed = seed
        self.step_id = 0
        f, _, _ = O.synth_env_step(seed, self.step_id, None, self.N, self.F, pixels)
        self.step_id += 1
        self.stack = np.repeat(f[:, None, :], window, 1)
        self.ret, self.rms = np.zeros(self.N), (0.0, 1.0, 1e-4)
        self.next_obs = self._obs_tensor()
        self.next_done = torch.zeros(self.N)

    def _obs_tensor(self):
        return torch.tensor(self.stack, dtype=torch.float32).view((self.N,) + self.obs_shape)

    def rollout_step(self, next_obs):
        """Act + env step + VecNormalize + frame stack of one rollout step (:502-514)."""
        with torch.no_grad():
            action, logprob, _, value = self.agent.get_action_and_value(next_obs)
        a = action.cpu().numpy()
        frame, r, d = O.synth_env_step(self.seed, self.step_id, a, self.N, self.F, self.pixels)
        self.step_id += 1
        r, self.ret, self.rms = O.vecnorm_reward(r, d, self.ret, self.rms)
        self.stack = np.concatenate([self.stack[:, 1:], frame[:, None]], 1)
        self.stack[d != 0] = frame[d != 0][:, None]
        return action, logprob, value, r, d

    def minibatch_update(self, b_obs, b_actions, b_logprobs, b_adv, b_ret, b_val, mb):
        """One minibatch of :566-610 (forward, loss, backward, clip_grad_norm_, Adam)."""
        _, newlp, ent, newv = self.agent.get_action_and_value(b_obs[mb], b_actions[mb])
        logratio = newlp - b_logprobs[mb]
        ratio = logratio.exp()
        mba = b_adv[mb]
        mba = (mba - mba.mean()) / (mba.std() + 1e-8)
        pg = torch.max(-mba * ratio, -mba * torch.clamp(ratio, 0.9, 1.1)).mean()
        newv = newv.view(-1)
        vu = (newv - b_ret[mb]) ** 2
        vc = (b_val[mb] + torch.clamp(newv - b_val[mb], -0.1, 0.1) - b_ret[mb]) ** 2
        v_loss = 0.5 * torch.max(vu, vc).mean()
        loss = pg - 0.01 * ent.mean() + v_loss * 0.5
        for p in self.agent.parameters():
            p.grad = None
        loss.backward()
        nn.utils.clip_grad_norm_(self.agent.parameters(), 0.5)
        self.opt.step()

    def iteration(self):
        T, N = self.T, self.N
        obs = torch.zeros((T, N) + self.obs_shape)
        actions = torch.zeros((T, N), dtype=torch.long)
        logprobs, rewards = torch.zeros((T, N)), torch.zeros((T, N))
        dones, values = torch.zeros((T, N)), torch.zeros((T, N))
        next_obs, next_done = self.next_obs, self.next_done
        for step in range(T):
            obs[step] = next_obs
            dones[step] = next_done
            action, logprob, value, r, d = self.rollout_step(next_obs)
            values[step] = value.flatten()
            actions[step] = action
            logprobs[step] = logprob
            rewards[step] = torch.tensor(r, dtype=torch.float32).view(-1)
            next_obs = self._obs_tensor()
            next_done = torch.tensor(d, dtype=torch.float32)
        with torch.no_grad():  # GAE, ppo_atari_oc.py:533-547
            next_value = self.agent.get_value(next_obs).reshape(1, -1)
            advantages, returns = gae_torch(rewards, values, dones, next_value, next_done)
        self.next_obs, self.next_done = next_obs, next_done
        B = T * N
        M = B // self.nmb
        b_obs = obs.reshape((-1,) + self.obs_shape)
        b_logprobs, b_actions = logprobs.reshape(-1), actions.reshape(-1)
        b_adv, b_ret, b_val = advantages.reshape(-1), returns.reshape(-1), values.reshape(-1)
        b_inds = np.arange(B)
        for _ in range(self.E):  # ppo_atari_oc.py:559-610
            np.random.shuffle(b_inds)
            for start in range(0, B, M):
                self.minibatch_update(b_obs, b_actions, b_logprobs, b_adv, b_ret, b_val,
                                      b_inds[start:start + M])
        return T * N


def gae_torch(rewards, values, dones, next_value, next_done, gamma=0.99, gae_lambda=0.95):
    """The reference's reverse GAE loop (ppo_atari_oc.py:533-547) on CPU torch tensors."""
    T = rewards.shape[0]
    advantages = torch.zeros_like(rewards)
    lastgaelam = 0.0
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nv = 1.0 - next_done, next_value
        else:
            nnt, nv = 1.0 - dones[t + 1], values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        lastgaelam = delta + gamma * gae_lambda * nnt * lastgaelam
        advantages[t] = lastgaelam
    return advantages, advantages + values


def host_info() -> dict:
    """CPU model, logical CPUs, the CPUs this process may run on and the cgroup CPU quota."""
    import os

    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"cpu_model": model, "cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def usable_threads() -> int:
    """All host cores this process may use: its CPU affinity, capped by the cgroup quota."""
    h = host_info()
    n = h["affinity_cpus"] or 1
    if h["cgroup_cpu_quota"]:
        n = min(n, max(1, int(h["cgroup_cpu_quota"])))
    return n


def _best(fn, reps):
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return best


def time_cpu_blocks(threads: int, c3: bool = True) -> dict:
    """Per-block CPU timings of the reference's own op sequences: GAE at T=128 for
    N in {128, 1024}; one PPObj minibatch forward + loss + backward + clip + Adam at M=4096;
    and a config-3 (NatureCNN, 256 pixel envs, minibatch 8192) iteration extrapolated from timed
    rollout steps and minibatch updates (128 x step + 16 x update)."""
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(0)
    out = {}
    for N in (128, 1024):
        r = torch.randn(128, N, generator=g)
        v = torch.randn(128, N, generator=g)
        d = (torch.rand(128, N, generator=g) < 0.01).float()
        nv, nd = torch.randn(1, N, generator=g), torch.zeros(N)
        out[f"gae_T128_N{N}_ms"] = round(1e3 * _best(lambda: gae_torch(r, v, d, nv, nd), 5), 3)
    lr = CpuLearner(num_envs=32, num_steps=128)
    B, M = 4096 * 4, 4096
    b_obs = torch.randint(0, 160, (B,) + lr.obs_shape, generator=g).float()
    b_act = torch.randint(0, 6, (B,), generator=g)
    b_lp, b_adv, b_ret, b_val = (torch.randn(B, generator=g) for _ in range(4))
    mb = np.random.RandomState(0).permutation(B)[:M]
    out["ppobj_minibatch_update_M4096_ms"] = round(1e3 * _best(
        lambda: lr.minibatch_update(b_obs, b_act, b_lp, b_adv, b_ret, b_val, mb), 3), 1)
    if c3:
        cl = CpuLearner(num_envs=256, num_steps=128, n_actions=4, pixels=True)
        x = cl._obs_tensor()
        step_s = _best(lambda: cl.rollout_step(x), 3)
        Bc, Mc = 256 * 128, 8192
        bo = torch.randint(0, 256, (Mc,) + cl.obs_shape, generator=g).float()
        ba = torch.randint(0, 4, (Mc,), generator=g)
        bl, bd, br, bv = (torch.randn(Mc, generator=g) for _ in range(4))
        upd_s = _best(lambda: cl.minibatch_update(bo, ba, bl, bd, br, bv, np.arange(Mc)), 1)
        it_s = 128 * step_s + 16 * upd_s
        out["c3_rollout_step_ms"] = round(1e3 * step_s, 1)
        out["c3_minibatch_update_M8192_ms"] = round(1e3 * upd_s, 1)
        out["c3_iteration_s_extrapolated"] = round(it_s, 2)
        out["c3_sps_extrapolated"] = round(Bc / it_s, 1)
    return out


class CpuCartPoleAgent(nn.Module):
    """cleanrl/ppo.py:100-126 restated: separate tanh-MLP critic / actor (64-64), orthogonal init
    (critic out std 1, actor out std 0.01)."""

    def __init__(self, obs_dim=4, n_actions=2):
        super().__init__()
        self.critic = nn.Sequential(_init(nn.Linear(obs_dim, 64)), nn.Tanh(),
                                    _init(nn.Linear(64, 64)), nn.Tanh(),
                                    _init(nn.Linear(64, 1), std=1.0))
        self.actor = nn.Sequential(_init(nn.Linear(obs_dim, 64)), nn.Tanh(),
                                   _init(nn.Linear(64, 64)), nn.Tanh(),
                                   _init(nn.Linear(64, n_actions), std=0.01))

    def get_value(self, x):
        return self.critic(x)

    def get_action_and_value(self, x, action=None):
        dist = torch.distributions.Categorical(logits=self.actor(x))
        if action is None:
            action = dist.sample()
        return action, dist.log_prob(action), dist.entropy(), self.critic(x)


def time_cpu_cartpole(iterations=20, threads=1, num_envs=4, num_steps=128, seed=1) -> dict:
    """BASELINE config 1 on the host: cleanrl/ppo.py's loop (:185-309; 4 CartPole-v1 envs,
    128 steps, 4 epochs x 4 minibatches of 128, clip 0.2, lr 2.5e-4 annealed off) with the
    oracle's CartPole dynamics (CartPoleOracle, gymnasium 0.28.1 restated) and the reference's
    agent on CPU torch with `threads` threads (ppo.py sets no thread count; 1 is its per-process
    share on a loaded host). Returns env steps/s and PPO updates/s over `iterations`."""
    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    np.random.seed(seed)
    env = O.CartPoleOracle(num_envs, seed)
    agent = CpuCartPoleAgent()
    opt = torch.optim.Adam(agent.parameters(), lr=2.5e-4, eps=1e-5)
    T, N, nmb, E = num_steps, num_envs, 4, 4
    B, M = T * N, T * N // nmb
    next_obs = torch.tensor(env.reset())
    next_done = torch.zeros(N)

    def iteration(next_obs, next_done):
        obs = torch.zeros((T, N, 4))
        actions = torch.zeros((T, N), dtype=torch.long)
        logprobs, rewards = torch.zeros((T, N)), torch.zeros((T, N))
        dones, values = torch.zeros((T, N)), torch.zeros((T, N))
        for step in range(T):
            obs[step] = next_obs
            dones[step] = next_done
            with torch.no_grad():
                action, logprob, _, value = agent.get_action_and_value(next_obs)
            values[step] = value.flatten()
            actions[step] = action
            logprobs[step] = logprob
            o, r, d = env.step(action.numpy())
            rewards[step] = torch.tensor(r)
            next_obs, next_done = torch.tensor(o), torch.tensor(d)
        with torch.no_grad():
            nv = agent.get_value(next_obs).reshape(1, -1)
            adv, ret = gae_torch(rewards, values, dones, nv, next_done)
        b_obs, b_lp, b_act = obs.reshape(-1, 4), logprobs.reshape(-1), actions.reshape(-1)
        b_adv, b_ret, b_val = adv.reshape(-1), ret.reshape(-1), values.reshape(-1)
        b_inds = np.arange(B)
        for _ in range(E):
            np.random.shuffle(b_inds)
            for start in range(0, B, M):
                mb = b_inds[start:start + M]
                _, newlp, ent, newv = agent.get_action_and_value(b_obs[mb], b_act[mb])
                logratio = newlp - b_lp[mb]
                ratio = logratio.exp()
                mba = b_adv[mb]
                mba = (mba - mba.mean()) / (mba.std() + 1e-8)
                pg = torch.max(-mba * ratio, -mba * torch.clamp(ratio, 0.8, 1.2)).mean()
                newv = newv.view(-1)
                vu = (newv - b_ret[mb]) ** 2
                vc = (b_val[mb] + torch.clamp(newv - b_val[mb], -0.2, 0.2) - b_ret[mb]) ** 2
                loss = pg - 0.01 * ent.mean() + 0.5 * torch.max(vu, vc).mean() * 0.5
                opt.zero_grad()
                loss.backward()
                nn.utils.clip_grad_norm_(agent.parameters(), 0.5)
                opt.step()
        return next_obs, next_done

    next_obs, next_done = iteration(next_obs, next_done)  # warm-up
    t0 = time.perf_counter()
    for _ in range(iterations):
        next_obs, next_done = iteration(next_obs, next_done)
    dt = time.perf_counter() - t0
    return {"sps": iterations * B / dt, "updates_per_sec": iterations * E * nmb / dt,
            "seconds": dt, "iterations": iterations, "threads": threads}


def time_cpu_baseline(iterations=2, threads=16, **kw) -> dict:
    """Time `iterations` CPU PPO iterations (after one untimed warm-up step of the network)."""
    torch.set_num_threads(threads)
    lr = CpuLearner(**kw)
    with torch.no_grad():
        lr.agent.get_action_and_value(lr.next_obs)
    t0 = time.perf_counter()
    steps = sum(lr.iteration() for _ in range(iterations))
    dt = time.perf_counter() - t0
    return {"env_steps": steps, "seconds": dt, "sps": steps / dt, "threads": threads,
            "updates_per_sec": iterations * lr.E * lr.nmb / dt}


class CpuQNetObj(nn.Module):
    """oc_cleanrl_amd.dqn.QNetworkObj in plain torch (per-frame Linear encoder, Flatten, Linear
    decoder, Q head; default PyTorch init like the reference's QNetwork, architectures/dqn.py)."""

    def __init__(self, obs_shape, n_actions, enc=(256, 512, 1024, 512), dec=(512,)):
        super().__init__()
        layers, d = [], obs_shape[-1]
        for n in enc:
            layers += [nn.Linear(d, n), nn.ReLU()]
            d = n
        layers.append(nn.Flatten())
        d *= obs_shape[0]
        for n in dec:
            layers += [nn.Linear(d, n), nn.ReLU()]
            d = n
        layers.append(nn.Linear(d, n_actions))
        self.network = nn.Sequential(*layers)

    def forward(self, x):
        return self.network(x)


def time_cpu_dqn(steps=4000, threads=16, num_envs=1, num_features=12, n_actions=6,
                 buffer_size=100_000, batch_size=32, train_frequency=4,
                 target_network_frequency=1000, seed=1) -> dict:
    """The training phase of cleanrl/dqn_atari_oc.py:341-400 on CPU torch, op for op: epsilon-
    greedy acting with the Q-network (:345-350), the synthetic env + VecNormalize reward, an SB3-
    style replay (optimize_memory_usage: next obs = the following row, cleanrl_utils/buffers.py),
    every `train_frequency` steps a batch of 32: target max, TD target, MSE, backward, Adam (:377-
    392), the target copy every `target_network_frequency` steps (:396-400). The buffer is filled
    with `batch_size` steps first (untimed): the timed steps are all past learning_starts."""
    import random

    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    random.seed(seed)
    rng = np.random.default_rng(seed)
    W, F, N = 4, num_features, num_envs
    obs_shape = (W, F)
    q, target = CpuQNetObj(obs_shape, n_actions), CpuQNetObj(obs_shape, n_actions)
    target.load_state_dict(q.state_dict())
    opt = torch.optim.Adam(q.parameters(), lr=1e-4)
    rows = max(buffer_size // N, 1)
    rb_obs = np.zeros((rows, N) + obs_shape, np.float32)
    rb_act = np.zeros((rows, N), np.int64)
    rb_rew = np.zeros((rows, N), np.float32)
    rb_done = np.zeros((rows, N), np.float32)
    pos, full = 0, False
    step_id = 0
    f, _, _ = O.synth_env_step(seed, step_id, None, N, F, False)
    stack = np.repeat(f[:, None, :], W, 1)
    ret, rms = np.zeros(N), (0.0, 1.0, 1e-4)
    epsilon = 0.05

    def one_step(global_step):
        nonlocal stack, ret, rms, pos, full, step_id
        if random.random() < epsilon:
            actions = rng.integers(0, n_actions, N)
        else:
            with torch.no_grad():
                actions = torch.argmax(q(torch.tensor(stack, dtype=torch.float32)), 1).numpy()
        frame, r, d = O.synth_env_step(seed, step_id, actions, N, F, False)
        step_id += 1
        r, ret, rms = O.vecnorm_reward(r, d, ret, rms)
        nxt = np.concatenate([stack[:, 1:], frame[:, None]], 1)
        nxt[d != 0] = frame[d != 0][:, None]
        rb_obs[pos], rb_act[pos], rb_rew[pos], rb_done[pos] = stack, actions, r, d
        rb_obs[(pos + 1) % rows] = nxt  # optimize_memory_usage: next obs lives in the next row
        pos = (pos + 1) % rows
        full = full or pos == 0
        stack = nxt
        if global_step % train_frequency == 0:
            hi = rows if full else pos
            b = (rng.integers(1, rows, batch_size) + pos) % rows if full else \
                rng.integers(0, hi, batch_size)
            e = rng.integers(0, N, batch_size)
            o = torch.tensor(rb_obs[b, e])
            no = torch.tensor(rb_obs[(b + 1) % rows, e])
            a = torch.tensor(rb_act[b, e]).view(-1, 1)
            rr = torch.tensor(rb_rew[b, e])
            dd = torch.tensor(rb_done[b, e])
            with torch.no_grad():
                target_max, _ = target(no).max(dim=1)
                td_target = rr + 0.99 * target_max * (1 - dd)
            old_val = q(o).gather(1, a).squeeze()
            loss = nn.functional.mse_loss(td_target, old_val)
            opt.zero_grad()
            loss.backward()
            opt.step()
        if global_step % target_network_frequency == 0:
            for tp, qp in zip(target.parameters(), q.parameters()):
                tp.data.copy_(1.0 * qp.data + 0.0 * tp.data)

    for g in range(1, batch_size + 1):  # fill past one batch (untimed)
        one_step(g * train_frequency + 1)
    t0 = time.perf_counter()
    for g in range(1, steps + 1):
        one_step(g)
    dt = time.perf_counter() - t0
    return {"sps": steps * N / dt, "updates_per_sec": steps / train_frequency / dt,
            "seconds": dt, "steps": steps, "threads": threads}
