"""Evaluation harness with the reference's interface (cleanrl_utils/evals/generic_eval.py:7-29):

    rewards = evaluate(agent, make_env, eval_episodes, device, **env_kwargs)

runs `agent.get_action_and_value(obs)[0]` on ONE env until `eval_episodes` episodes have ended
and returns their episodic (raw, un-normalised) returns, as RecordEpisodeStatistics reports them
in `infos["final_info"]`. ppo_atari_oc.py:687-691 calls it with 10 episodes after training.

The env is the device-resident synthetic env (ALE / OCAtari are not available here), stacked by
the same HIP store kernel the learner uses (reset fill on episode end); the episode bookkeeping
is the env kernel's RecordEpisodeStatistics counters, read once per step (the reference syncs on
`actions.cpu()` every step as well).
"""
from __future__ import annotations

import torch

from . import ops
from .envs import SyntheticAtariEnv


class EvalEnv:
    """One synthetic env with frame stacking: reset() -> obs [1, W, ...] f32, step(actions) ->
    (obs, list of returns of the episodes that ended at this step)."""

    def __init__(self, env_id: str, obs_mode: str = "obj", num_features: int = 12, seed: int = 0,
                 device="cuda", window: int = 4):
        self.env = SyntheticAtariEnv(env_id, obs_mode, 1, num_features, seed, device, window)
        shape = (1,) + self.env.single_obs_shape
        dev = torch.device(device)
        self.stack = [torch.zeros(shape, dtype=torch.float32, device=dev) for _ in range(2)]
        self.obs = torch.zeros(shape, dtype=torch.float32, device=dev)
        self.cur = 0
        self.t = 0
        self.single_observation_space_shape = self.env.single_obs_shape
        self.n_actions = self.env.n_actions

    def reset(self):
        frame = self.env.reset()
        ops.obs_reset(frame, self.stack[self.cur], self.obs)
        self.t = 0
        return self.obs

    def step(self, actions):
        env = self.env
        env.step(actions.reshape(1).to(torch.int64), self.t)
        nxt = 1 - self.cur
        ops.rollout_store(env.frame, env.reward, env.done, self.stack[self.cur], self.stack[nxt],
                          self.obs)
        self.cur = nxt
        self.t += 1
        if self.t >= 1024:  # keep the env's step id in range of its counter base
            env.advance(self.t)
            self.t = 0
        ret_sum, _, count = env.pop_episode_stats()  # one host sync per step
        return self.obs, ([ret_sum] if count > 0 else [])


def make_env(idx: int = 0, env_id: str = "ALE/Pong-v5", obs_mode: str = "obj",
             num_features: int = 12, seed: int = 0, device="cuda", **_):
    """The reference's `make_env(idx=0, **env_kwargs)` factory shape (capture_video, run_dir
    and other gym-only kwargs are accepted and ignored)."""
    return EvalEnv(env_id, obs_mode, num_features, seed + idx, device)


def evaluate(agent, make_env, eval_episodes: int, device, **env_kwargs):
    """generic_eval.py:7-29 semantics: episodic returns of `eval_episodes` finished episodes."""
    env = make_env(idx=0, device=device, **env_kwargs)
    agent.eval()
    obs = env.reset()
    episodic_returns: list = []
    with torch.no_grad():
        while len(episodic_returns) < eval_episodes:
            actions = agent.get_action_and_value(obs)[0]
            obs, finished = env.step(actions)
            episodic_returns += finished
    return episodic_returns[:eval_episodes] if len(episodic_returns) > eval_episodes \
        else episodic_returns
