"""Device-resident vectorised environments.

ALE / OCAtari / HackAtari are not available (no emulator, no network), so the learner is driven
by a synthetic env that lives in HBM and steps with one HIP kernel (ocppo_synth_env_step):
object-vector frames with OCAtari obj-mode statistics or 84x84 u8 pixel frames, Pong-like sparse
rewards and episode ends. It replaces the SubprocVecEnv + per-step host round trip
of cleanrl/ppo_atari_oc.py:411-414, 511-514; its dynamics are NOT Pong's (parity of returns
against real ALE is unpinned).

The env produces the NEWEST frame per env; frame stacking and storage happen in the rollout store
kernel (ops.rollout_store).
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .args import ACTION_COUNTS


class SyntheticAtariEnv:
    """num_envs synthetic Atari envs on one device.

    obs_mode "obj": frames [N, F] f32 (F = num_features); "dqn": frames [N, 84*84] u8.
    """

    integer_obs = True  # integer coordinates <= 210 / u8 pixels: bf16 / u8 storage is exact
    synthetic = True    # its step is ocppo_synth_env_step's (the policy head may fuse it)

    def __init__(self, env_id: str, obs_mode: str, num_envs: int, num_features: int, seed: int,
                 device, window: int = 4):
        self.env_id = env_id
        self.pixels = obs_mode == "dqn"
        self.num_envs = num_envs
        self.n_actions = ACTION_COUNTS.get(env_id, 6)
        self.window = window
        self.frame_elems = 84 * 84 if self.pixels else num_features
        self.single_obs_shape = (window, 84, 84) if self.pixels else (window, num_features)
        self.frame_dtype = torch.uint8 if self.pixels else torch.float32
        self.seed = int(seed)
        self.device = torch.device(device)
        N = num_envs
        self.frame = torch.zeros((N, self.frame_elems), dtype=self.frame_dtype, device=device)
        self.reward = torch.zeros(N, dtype=torch.float32, device=device)
        self.done = torch.zeros(N, dtype=torch.float32, device=device)
        # RecordEpisodeStatistics counters: run_ret, run_len, fin_ret_sum, fin_len_sum, fin_count
        self.ep_state = torch.zeros((N, 5), dtype=torch.float32, device=device)
        self.step_base = torch.zeros(1, dtype=torch.int64, device=device)

    def reset(self):
        """Initial frames (step id = step_base); advances step_base by one."""
        ops.synth_env_step(self.seed, self.step_base, 0, None, self.frame, self.reward, self.done,
                           None)
        self.step_base.add_(1)
        return self.frame

    def step(self, actions, step_offset: int):
        """Writes frame/reward/done for step id step_base + step_offset (graph-replay safe)."""
        ops.synth_env_step(self.seed, self.step_base, step_offset, actions, self.frame,
                           self.reward, self.done, self.ep_state)

    def advance(self, n: int):
        self.step_base.add_(n)

    def pop_episode_stats(self):
        """(sum of finished-episode returns, sum of lengths, count) since the last call."""
        s = self.ep_state[:, 2:5].sum(0, dtype=torch.float64).tolist()
        self.ep_state[:, 2:5].zero_()
        return s


class CartPoleVecEnv:
    """num_envs CartPole-v1 envs on one device (config 1: cleanrl/ppo.py:162's SyncVectorEnv of
    RecordEpisodeStatistics(gym.make("CartPole-v1"))), stepped by one HIP kernel
    (ops.cartpole_step: gymnasium 0.28.1 dynamics in f64, TimeLimit 500, same-step auto-reset).

    Same interface as SyntheticAtariEnv: frame [N, 4] f32 is the whole observation (no frame
    stack: window 1, single_obs_shape (1, 4); CartPoleAgent flattens it), reward / done [N] f32,
    RecordEpisodeStatistics counters in ep_state."""

    pixels = False
    integer_obs = False  # fractional state: stored in f32

    def __init__(self, num_envs: int, seed: int, device):
        self.env_id = "CartPole-v1"
        self.num_envs = N = num_envs
        self.n_actions = 2
        self.window = 1
        self.frame_elems = 4
        self.single_obs_shape = (1, 4)
        self.frame_dtype = torch.float32
        self.seed = int(seed)
        self.device = torch.device(device)
        self.state = torch.zeros((N, 4), dtype=torch.float64, device=device)
        self.counters = torch.zeros((N, 2), dtype=torch.int64, device=device)
        self.frame = torch.zeros((N, 4), dtype=torch.float32, device=device)
        self.reward = torch.zeros(N, dtype=torch.float32, device=device)
        self.done = torch.zeros(N, dtype=torch.float32, device=device)
        self.ep_state = torch.zeros((N, 5), dtype=torch.float32, device=device)

    def reset(self):
        ops.cartpole_step(self.seed, None, self.state, self.counters, self.frame)
        return self.frame

    def step(self, actions, step_offset: int = 0):
        ops.cartpole_step(self.seed, actions, self.state, self.counters, self.frame, self.reward,
                          self.done, self.ep_state)

    def advance(self, n: int):
        pass

    def pop_episode_stats(self):
        s = self.ep_state[:, 2:5].sum(0, dtype=torch.float64).tolist()
        self.ep_state[:, 2:5].zero_()
        return s


def make_device_env(env_id: str, obs_mode: str, num_envs: int, num_features: int, seed: int,
                    device, window: int = 4):
    """The device-resident vector env for `env_id`: CartPole-v1 (config 1) or the synthetic
    Atari env (configs 2-5; ALE / OCAtari are not available)."""
    if env_id == "CartPole-v1":
        return CartPoleVecEnv(num_envs, seed, device)
    return SyntheticAtariEnv(env_id, obs_mode, num_envs, num_features, seed, device, window)


class HostVecEnv:
    """Host (CPU) vector env → the device rollout path: the env-step boundary of
    cleanrl/ppo_atari_oc.py:506-514 for real emulators (OCAtari / ALE through
    gymnasium's vector API, which this image lacks).

    `envs` is the reference's SubprocVecEnv of make_env thunks (:411-413) WITHOUT the VecNormalize
    of :414 (reward normalisation runs on the device, fused into the store kernel; a
    reward-normalising wrapper is rejected), or any gymnasium vector env with the same frame
    stack. Both APIs are accepted:
      SB3 VecEnv (the reference's): reset() -> obs [N, W, *frame];
        step(actions np.int64 [N]) -> (obs, reward [N], done [N], infos)   (:511)
      gymnasium: reset(seed=...) -> (obs, info);
        step(actions) -> (obs, reward, terminated, truncated, info)
    Only the NEWEST frame obs[:, -1] crosses PCIe per step; the device store kernel rebuilds the
    stack. On a done the env's own returned stack is the authority: the reference's NoopResetEnv /
    FireResetEnv step the inner frame stack after reset and EpisodicLifeEnv signals done on a life
    loss without resetting it (ppo_atari_oc.py:278-282), so the older W-1 frames of every done row
    are uploaded too (one small async copy per done row, outside the captured step graph) and the
    store copies them instead of FrameStack's fill. An env that declares
    `frame_stack_fill_rule = True` (its reset stacks are W copies of the first frame) skips that.

    Per step: actions D2H into pinned memory (one stream sync: the env needs them), env.step on
    the host, newest frame / reward / done (= terminated | truncated, :514) written into pinned
    staging, then ONE async H2D copy of the staging block on the current stream, ordered before
    the store kernel that consumes .frame / .reward / .done. The trainer captures the device work
    between two host steps (upload + store of step t-1, act of step t, action copy) as one
    hipGraph per step, so a rollout step costs one graph launch + one sync + the env's own step.

    Episode statistics (charts/Episodic_Original_Reward / Episodic_Length, :516-529) come from the
    envs' RecordEpisodeStatistics reports (`info["episode"]` of SB3's per-env info dicts, or
    gymnasium's `final_info` / `episode` + `_episode` entries): whole games even when
    EpisodicLifeEnv ends an "episode" per life. Only an env that never reports them falls back to
    summing raw rewards between dones (episode_info=None: automatic; True/False: force).
    """

    def __init__(self, envs, env_id: str, obs_mode: str, num_envs: int, seed: int, device,
                 window: int = 4, episode_info: bool | None = None):
        if getattr(envs, "norm_reward", False):
            raise ValueError("pass the vector env without VecNormalize(norm_reward=True): the "
                             "device store kernel applies the reward normalisation (:414)")
        self.envs = envs
        self.env_id = env_id
        self.pixels = obs_mode == "dqn"
        self.num_envs = N = int(num_envs)
        self.n_actions = ACTION_COUNTS.get(env_id, 6)
        na = getattr(getattr(envs, "single_action_space", None), "n", None)
        if na is not None:
            self.n_actions = int(na)
        self.window = window
        self.seed = int(seed)
        self.device = torch.device(device)
        self.frame_dtype = torch.uint8 if self.pixels else torch.float32
        self._frame_shape = None
        self.single_obs_shape = None
        pin = self.device.type == "cuda"
        self._act_host = torch.empty(N, dtype=torch.int64, pin_memory=pin)
        self._run_ret = np.zeros(N, np.float64)
        self._run_len = np.zeros(N, np.int64)
        self._fin = [0.0, 0.0, 0.0]
        self._fin_info = [0.0, 0.0, 0.0]
        self.episode_info = episode_info
        self._info_seen = False
        self._pin = pin
        self.frame = self.reward = self.done = None
        self.reset_stacks = window > 1 and not getattr(envs, "frame_stack_fill_rule", False)
        self.reset_prev = None
        self._reset_rows = np.zeros(0, np.int64)

    def _alloc(self, obs):
        obs = np.asarray(obs)
        if obs.shape[0] != self.num_envs or obs.ndim < 3:
            raise ValueError(f"host env obs must be [N={self.num_envs}, W, *frame], got {obs.shape}")
        self.single_obs_shape = tuple(obs.shape[1:])
        self._frame_shape = tuple(obs.shape[2:])
        fe = int(np.prod(self._frame_shape))
        self.frame_elems = fe
        N = self.num_envs
        # one pinned staging block: [frame bytes | reward f32 | done f32], one H2D per step
        fb = N * fe * (1 if self.pixels else 4)
        self._off_r = (fb + 255) // 256 * 256
        self._off_d = self._off_r + 4 * N
        nbytes = self._off_d + 4 * N
        self._stage_host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=self._pin)
        self._stage_dev = torch.empty(nbytes, dtype=torch.uint8, device=self.device)

        def views(buf):
            fr = buf[:fb].view(self.frame_dtype).view(N, fe)
            rw = buf[self._off_r:self._off_r + 4 * N].view(torch.float32)
            dn = buf[self._off_d:self._off_d + 4 * N].view(torch.float32)
            return fr, rw, dn

        self._h_frame, self._h_reward, self._h_done = views(self._stage_host)
        self.frame, self.reward, self.done = views(self._stage_dev)
        if self.reset_stacks:
            W = self.single_obs_shape[0]
            self._h_reset = torch.zeros((N, W - 1, fe), dtype=self.frame_dtype,
                                        pin_memory=self._pin)
            self.reset_prev = torch.zeros((N, W - 1, fe), dtype=self.frame_dtype,
                                          device=self.device)

    def _stage(self, obs, reward, done, reset_rows=None):
        obs = np.asarray(obs)
        flat = obs.reshape(self.num_envs, obs.shape[1], -1)
        np.copyto(self._h_frame.numpy(), flat[:, -1], casting="unsafe")
        if self.reset_stacks:
            rows = np.flatnonzero(np.asarray(done)) if reset_rows is None else reset_rows
            if len(rows):
                hr = self._h_reset.numpy()
                hr[rows] = flat[rows, :-1]
            self._reset_rows = rows
        np.copyto(self._h_reward.numpy(), np.asarray(reward, dtype=np.float64), casting="unsafe")
        np.copyto(self._h_done.numpy(), np.asarray(done), casting="unsafe")

    def upload(self):
        """Staging block → device, async on the current stream (graph-capturable)."""
        self._stage_dev.copy_(self._stage_host, non_blocking=True)

    def upload_resets(self):
        """The done rows' older W-1 frames → reset_prev, async on the current stream. Issued
        eagerly before the (captured) step that stores them: only done rows are copied."""
        rows = self._reset_rows
        if not self.reset_stacks or not len(rows):
            return
        if len(rows) * 4 >= self.num_envs:
            self.reset_prev.copy_(self._h_reset, non_blocking=True)
        else:
            for r in rows.tolist():
                self.reset_prev[r].copy_(self._h_reset[r], non_blocking=True)
        self._reset_rows = rows[:0]

    def fetch_actions(self, actions):
        """Actions → pinned host memory, async on the current stream (graph-capturable)."""
        self._act_host.copy_(actions, non_blocking=True)

    def reset(self):
        try:
            r = self.envs.reset(seed=self.seed)
        except TypeError:  # SB3 VecEnv: reset() takes no seed (seeded per worker, :412)
            r = self.envs.reset()
        obs = r[0] if isinstance(r, tuple) and len(r) == 2 and isinstance(r[1], dict) else r
        if self.frame is None:
            self._alloc(obs)
        # every row's whole stack is staged (the initial obs is the env's own reset stack)
        self._stage(obs, np.zeros(self.num_envs), np.zeros(self.num_envs),
                    reset_rows=np.arange(self.num_envs))
        self.upload()
        self.upload_resets()
        return self.frame

    def host_step(self):
        """Wait for the queued action copy, step the host env, fill the staging block. The wait
        also drains the previous upload (same stream, queued earlier), so the block is free."""
        if self._pin:
            torch.cuda.current_stream(self.device).synchronize()
        act = self._act_host.numpy().copy()
        out = self.envs.step(act)
        if len(out) == 5:  # gymnasium: terminated | truncated (:514)
            obs, reward, term, trunc, infos = out
            done = np.logical_or(term, trunc)
        else:  # SB3 VecEnv: done already folds both, the env auto-resets
            obs, reward, done, infos = out
            done = np.asarray(done, dtype=bool)
        r = np.asarray(reward, dtype=np.float64)
        self._run_ret += r
        self._run_len += 1
        if done.any():
            self._fin[0] += float(self._run_ret[done].sum())
            self._fin[1] += float(self._run_len[done].sum())
            self._fin[2] += float(done.sum())
            self._run_ret[done] = 0.0
            self._run_len[done] = 0
        if self.episode_info is not False:
            self._episode_infos(infos)
        self._stage(obs, r, done)

    def step(self, actions, step_offset: int = 0):
        """Eager form of one env step: fetch_actions + host_step + upload."""
        self.fetch_actions(actions)
        self.host_step()
        self.upload()

    def advance(self, n: int):
        pass

    def _episode_infos(self, infos):
        """RecordEpisodeStatistics reports of one step: SB3 per-env dicts (info["episode"] =
        {"r", "l", ...}, what ppo_atari_oc.py:518-523 reads) or gymnasium's vector-info dict."""
        eps = []
        if isinstance(infos, (list, tuple)):
            eps = [i["episode"] for i in infos if isinstance(i, dict) and "episode" in i]
        elif isinstance(infos, dict):
            if "final_info" in infos:
                eps = [i["episode"] for i in infos["final_info"]
                       if isinstance(i, dict) and "episode" in i]
            elif "episode" in infos and "_episode" in infos:
                ep, mask = infos["episode"], np.asarray(infos["_episode"], bool)
                eps = [{"r": np.asarray(ep["r"])[i], "l": np.asarray(ep["l"])[i]}
                       for i in np.flatnonzero(mask)]
        for e in eps:
            self._info_seen = True
            self._fin_info[0] += float(np.asarray(e["r"]).reshape(-1)[0])
            self._fin_info[1] += float(np.asarray(e["l"]).reshape(-1)[0])
            self._fin_info[2] += 1.0

    def pop_episode_stats(self):
        use_info = self.episode_info if self.episode_info is not None else self._info_seen
        s = self._fin_info if use_info else self._fin
        self._fin, self._fin_info = [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]
        return s
