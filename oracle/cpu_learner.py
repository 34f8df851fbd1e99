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


class CpuLearner:
    """One process, `num_envs` synthetic Pong-obj envs, reference hyper-parameters."""

    def __init__(self, num_envs=128, num_steps=128, num_features=12, n_actions=6, seed=42,
                 num_minibatches=4, update_epochs=4, window=4):
        torch.manual_seed(seed)
        np.random.seed(seed)
        self.N, self.T, self.F, self.A, self.W = num_envs, num_steps, num_features, n_actions, window
        self.obs_shape = (window, num_features)
        self.agent = CpuPPObj(self.obs_shape, n_actions)
        self.opt = torch.optim.Adam(self.agent.parameters(), lr=2.5e-4, eps=1e-5)
        self.nmb, self.E = num_minibatches, update_epochs
        self.seed = seed
        self.step_id = 0
        f, _, _ = O.synth_env_step(seed, self.step_id, None, self.N, self.F, False)
        self.step_id += 1
        self.stack = np.repeat(f[:, None, :], window, 1)
        self.ret, self.rms = np.zeros(self.N), (0.0, 1.0, 1e-4)
        self.next_obs = torch.tensor(self.stack, dtype=torch.float32)
        self.next_done = torch.zeros(self.N)

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
            with torch.no_grad():
                action, logprob, _, value = self.agent.get_action_and_value(next_obs)
                values[step] = value.flatten()
            actions[step] = action
            logprobs[step] = logprob
            a = action.cpu().numpy()
            frame, r, d = O.synth_env_step(self.seed, self.step_id, a, N, self.F, False)
            self.step_id += 1
            r, self.ret, self.rms = O.vecnorm_reward(r, d, self.ret, self.rms)
            self.stack = np.concatenate([self.stack[:, 1:], frame[:, None]], 1)
            self.stack[d != 0] = frame[d != 0][:, None]
            rewards[step] = torch.tensor(r, dtype=torch.float32).view(-1)
            next_obs = torch.tensor(self.stack, dtype=torch.float32)
            next_done = torch.tensor(d, dtype=torch.float32)
        with torch.no_grad():  # GAE, ppo_atari_oc.py:533-547
            next_value = self.agent.get_value(next_obs).reshape(1, -1)
            advantages = torch.zeros_like(rewards)
            lastgaelam = 0.0
            for t in reversed(range(T)):
                if t == T - 1:
                    nnt, nv = 1.0 - next_done, next_value
                else:
                    nnt, nv = 1.0 - dones[t + 1], values[t + 1]
                delta = rewards[t] + 0.99 * nv * nnt - values[t]
                lastgaelam = delta + 0.99 * 0.95 * nnt * lastgaelam
                advantages[t] = lastgaelam
            returns = advantages + values
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
                mb = b_inds[start:start + M]
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
        return T * N


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
