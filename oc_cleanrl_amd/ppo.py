"""`python -m oc_cleanrl_amd.ppo [cleanrl/ppo.py flags]` — config 1: PPO on CartPole-v1.

The same learner as `python -m oc_cleanrl_amd` (trainer.PPOTrainer) with cleanrl/ppo.py's
defaults (Args :17-78: seed 1, 4 envs, 500k steps, clip_coef 0.2, no VecNormalize) and its agent
(separate tanh-MLP actor / critic, :100-126 = agents.CartPoleAgent), fed by the device CartPole-v1
vector env (envs.CartPoleVecEnv: gymnasium 0.28.1 dynamics, one HIP launch per step) instead of
gym.vector.SyncVectorEnv (:162). GAE, the fused loss, clip + Adam are the HIP kernels of the
Atari path; metrics go to runs/<run>/metrics.jsonl under ppo.py's scalar names."""
from __future__ import annotations

from .__main__ import main as _main

# cleanrl/ppo.py:17-78 where it differs from ppo_atari_oc.py's Args
PPO_DEFAULTS = dict(exp_name="ppo", seed=1, env_id="CartPole-v1", total_timesteps=500_000,
                    num_envs=4, clip_coef=0.2, architecture="CARTPOLE_MLP", obs_mode="obj",
                    buffer_window_size=1, vecnorm_reward=False, wandb_project_name="cleanRL")


def main(argv=None):
    return _main(argv, defaults=PPO_DEFAULTS)


if __name__ == "__main__":
    main()
