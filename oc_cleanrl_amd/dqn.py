"""DQN learner of cleanrl/dqn_atari_oc.py (BASELINE config 5) on HBM-resident state.

The reference loop (dqn_atari_oc.py:341-400) per global step: epsilon-greedy action (:345-350),
env step, `rb.add` into an SB3 ReplayBuffer(optimize_memory_usage=True) (:369), then after
`learning_starts` every `train_frequency` steps a batch of 32 is sampled (:377), the TD target
r + gamma * max_a Q_target(s') * (1 - d) and the MSE against Q(s)[a] are formed (:378-382), Adam
steps (:390-392), and every `target_network_frequency` steps the target net is soft-updated with
tau (:396-400).

Here every piece of that loop runs on the GPU without a host round trip:
  ops.epsilon_greedy        one coin per global step for all envs (the reference's
                            `random.random() < epsilon` decides for the whole vector), greedy
                            argmax or uniform actions, epsilon = linear_schedule(step)
  SyntheticAtariEnv.step    device env (ALE / OCAtari are not available)
  ops.rollout_store_vecnorm frame stack + VecNormalize(norm_reward=True) reward (:317)
  ops.ReplayBuffer          1M-transition HBM replay, SB3 optimize_memory_usage layout
  ops.td_loss_fwd_bwd       fused TD target + MSE forward and d loss / d Q
  ops.FlatAdam              Adam (torch defaults: eps 1e-8, no clipping) over one flat buffer
and `train_frequency` env steps + the train step are captured as ONE hipGraph (a second graph
without the train step covers the steps before `learning_starts`).

Q-networks: `QNetwork` is architectures/dqn.py:8-31 (module layout and state-dict keys equal, the
reference's default PyTorch init). The reference's QNetwork is convolution-only, so obs_mode
"obj" cannot run in the reference at all (its Args.architecture is never used to pick another
net); `QNetworkObj` is this build's declared extension for object vectors: the PPObj trunk
(per-frame Linear encoder, Flatten, Linear decoder, architectures/ppo.py:60-84) with a Q head.
"""
from __future__ import annotations

import json
import time
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import gemm_table, ops
from .agents import Predictor, fused_trunk, q_head
from .args import OBS_MODES, parse_dataclass
from .envs import SyntheticAtariEnv


@dataclass
class DQNArgs:
    """The flags of dqn_atari_oc.py:53-140 (same names and defaults) + this build's additions."""
    exp_name: str = "dqn_atari_oc"
    seed: int = 42
    torch_deterministic: bool = True
    cuda: bool = True
    env_id: str = "ALE/Pong-v5"
    obs_mode: str = "dqn"
    feature_func: str = ""
    buffer_window_size: int = 4
    backend: str = "Synthetic"  # reference: OCAtari (ALE not available here)
    modifs: str = ""
    new_rf: str = ""
    frameskip: int = 4
    track: bool = False
    wandb_project_name: str = "OCAtari"
    wandb_entity: str = "AIML_OC"
    wandb_dir: Optional[str] = None
    capture_video: bool = False
    ckpt: str = ""
    logging_level: int = 40
    author: str = "JB"
    architecture: str = "DQN"
    total_timesteps: int = 10_000_000
    learning_rate: float = 1e-4
    num_envs: int = 1
    buffer_size: int = 1_000_000
    gamma: float = 0.99
    tau: float = 1.0
    target_network_frequency: int = 1000
    batch_size: int = 32
    start_e: float = 1.0
    end_e: float = 0.01
    exploration_fraction: float = 0.10
    learning_starts: int = 80_000
    train_frequency: int = 4
    test_modifs: str = ""
    masked_wrapper: str = ""

    # [oc_cleanrl_amd] additions
    num_features: int = 12      # object-vector width F per frame (synthetic obj env)
    obs_storage: str = "auto"   # replay obs dtype: auto (u8 pixels / bf16 objects) | f32 | bf16 | u8
    encoder_dims: tuple = (256, 512, 1024, 512)  # QNetworkObj (obs_mode obj)
    decoder_dims: tuple = (512,)
    cuda_graphs: bool = True
    gemm_table: bool = False  # the shipped hipBLASLt solution table (gemm_table.py): no gain measured here
    vecnorm_reward: bool = True  # VecNormalize(norm_reward=True) of dqn_atari_oc.py:286
    log_dir: str = "runs"
    save_model: bool = True
    log_every: int = 100        # the reference logs td_loss / q_values every 100 steps


class QNetwork(Predictor):
    """architectures/dqn.py:8-31: NatureCNN Q-network, forward = network(x / 255)."""

    def __init__(self, obs_shape, n_actions):
        super().__init__()
        self.network = nn.Sequential(
            nn.Conv2d(obs_shape[0], 32, 8, stride=4), nn.ReLU(),
            nn.Conv2d(32, 64, 4, stride=2), nn.ReLU(),
            nn.Conv2d(64, 64, 3, stride=1), nn.ReLU(),
            nn.Flatten(), nn.Linear(3136, 512), nn.ReLU(),
            nn.Linear(512, n_actions))

    def forward(self, x):
        return self.network(x / 255.0)

    def q_values(self, x):
        return q_head(fused_trunk(self.network[:-1], x / 255.0), self.network[-1])

    def get_action_and_value(self, x):
        """architectures/dqn.py:28-31 (greedy action; the eval harness uses element 0)."""
        q = self.forward(x)
        action = torch.argmax(q, 1)
        return action, q[:, action], None, None

    def predict(self, x, states=None, **_):
        with torch.no_grad():
            dev = next(self.parameters()).device
            q = self.forward(torch.as_tensor(np.asarray(x), dtype=torch.float32, device=dev))
            return np.argmax(q.cpu().numpy(), axis=1), states


class QNetworkObj(Predictor):
    """[oc_cleanrl_amd extension] object-vector Q-network: PPObj's trunk + a Q head."""

    def __init__(self, obs_shape, n_actions, encoder_dims=(256, 512, 1024, 512),
                 decoder_dims=(512,)):
        super().__init__()
        layers, d = [], obs_shape[-1]
        for l in encoder_dims:
            layers += [nn.Linear(d, l), nn.ReLU()]
            d = l
        layers.append(nn.Flatten())
        d *= int(np.prod(obs_shape[:-1]))
        for l in decoder_dims:
            layers += [nn.Linear(d, l), nn.ReLU()]
            d = l
        layers.append(nn.Linear(d, n_actions))
        self.network = nn.Sequential(*layers)

    def forward(self, x):
        return self.network(x)

    def q_values(self, x):
        return q_head(fused_trunk(self.network[:-1], x), self.network[-1])

    get_action_and_value = QNetwork.get_action_and_value
    predict = QNetwork.predict


# The train step's target-network forward on a side stream, concurrent with the online forward
# (DQNTrainer._train_step; captured into the chunk's hipGraph as a fork / join): measured slower
# (config 5 11.3k vs 12.4k env steps/s, profiles/r06/config5_side_stream/), so off
TARGET_SIDE_STREAM = False

# The acting step's Q head + epsilon-greedy choice as one HIP launch (ops.q_head_epsilon_greedy).
FUSED_ACT = True
# ... and with an object-frame synthetic env, the whole rest of the step (env, store +
# VecNormalize, replay add) in the same launch (ops.dqn_act_step)
FUSED_ACT_STEP = True


def make_qnet(args: DQNArgs, obs_shape, n_actions) -> nn.Module:
    if args.obs_mode == "obj":
        return QNetworkObj(obs_shape, n_actions, args.encoder_dims, args.decoder_dims)
    return QNetwork(obs_shape, n_actions)


def _q_forward(net, x):
    """Q(x) through the fused Linear(+ReLU) path (same math as net(x))."""
    return net.q_values(x)


class DQNTrainer:
    def __init__(self, args: DQNArgs, device, log: bool = True):
        a = args
        if a.backend != "Synthetic":
            raise NotImplementedError("ALE / OCAtari are not available; use --backend Synthetic")
        if a.obs_mode not in ("dqn", "obj"):
            raise NotImplementedError(f"obs_mode {a.obs_mode!r}: only dqn and obj are supported")
        self.args = a
        self.dev = torch.device(device)
        torch.use_deterministic_algorithms(a.torch_deterministic)
        # deterministic mode also NaN-fills every torch.empty (a debugging aid: ~300 fill launches per
        # iteration here); nothing reads uninitialised memory, so results are unaffected
        torch.utils.deterministic.fill_uninitialized_memory = False
        torch.backends.cudnn.deterministic = a.torch_deterministic
        torch.backends.cudnn.benchmark = False
        self.gemm_table = a.gemm_table and gemm_table.use(device)
        torch.manual_seed(a.seed)
        self.E = a.num_envs
        self.env = SyntheticAtariEnv(a.env_id, a.obs_mode, self.E, a.num_features, a.seed,
                                     self.dev, a.buffer_window_size)
        self.pixels = self.env.pixels
        self.A = self.env.n_actions
        self.obs_shape = self.env.single_obs_shape
        self.q = make_qnet(a, self.obs_shape, self.A).to(self.dev)
        self.target = make_qnet(a, self.obs_shape, self.A).to(self.dev)
        self.target.load_state_dict(self.q.state_dict())  # :315
        self.opt = ops.FlatAdam(self.q.parameters(), lr=a.learning_rate, eps=1e-8)
        # the target net's parameters as views of one flat buffer too (soft update = 2 ops)
        t_params = [p for p in self.target.parameters()]
        offs, n = ops.flat_offsets(t_params)
        self.t_flat = torch.zeros(n, dtype=torch.float32, device=self.dev)
        for p, off in zip(t_params, offs):
            self.t_flat[off:off + p.numel()].copy_(p.detach().reshape(-1))
            p.data = self.t_flat[off:off + p.numel()].view_as(p)
            p.requires_grad_(False)
        self.direct_grads = all(isinstance(m, (nn.Linear, nn.ReLU, nn.Flatten))
                                for m in self.q.network)

        if a.obs_storage == "auto":
            st = torch.uint8 if self.pixels else torch.bfloat16
        else:
            st = {"f32": torch.float32, "bf16": torch.bfloat16, "u8": torch.uint8}[a.obs_storage]
        self.obs_dtype = st
        dev, f32 = self.dev, torch.float32
        W = self.obs_shape[0]
        self.stacks = [torch.zeros((self.E,) + self.obs_shape, dtype=st, device=dev)
                       for _ in range(2)]
        self.net_obs = torch.zeros((self.E,) + self.obs_shape, dtype=f32, device=dev)
        # SB3 keeps buffer_size // n_envs rows of n_envs transitions (buffers.py:185)
        self.rb = ops.ReplayBuffer(max(a.buffer_size // self.E, 1), self.E, self.obs_shape, dev,
                                   obs_dtype=st,
                                   seed=a.seed)
        self.actions = torch.zeros(self.E, dtype=torch.int64, device=dev)
        self.rew_out = torch.zeros(self.E, dtype=f32, device=dev)
        self.done_out = torch.zeros(self.E, dtype=f32, device=dev)
        self.ret_state = torch.zeros(self.E, dtype=torch.float64, device=dev)
        self.rms_state = torch.tensor([0.0, 1.0, 1e-4], dtype=torch.float64, device=dev)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)  # global_step
        self.epsilon = torch.zeros(1, dtype=f32, device=dev)
        B = a.batch_size
        self.batch = {"observations": torch.zeros((B,) + self.obs_shape, device=dev),
                      "next_observations": torch.zeros((B,) + self.obs_shape, device=dev),
                      "actions": torch.zeros((B, 1), dtype=torch.int64, device=dev),
                      "rewards": torch.zeros((B, 1), device=dev),
                      "dones": torch.zeros((B, 1), device=dev)}
        self.dq = torch.zeros((B, self.A), dtype=f32, device=dev)
        self.side = torch.cuda.Stream(self.dev) if self.dev.type == "cuda" else None
        self.td_stats = torch.zeros(2, dtype=f32, device=dev)
        self.duration = a.exploration_fraction * a.total_timesteps
        # acting: the Q head and the epsilon-greedy choice in one launch
        head = self.q.network[-1]
        self.fused_act = (FUSED_ACT and isinstance(head, nn.Linear) and head.bias is not None and
                          self.A <= 8 and head.in_features % 256 == 0 and
                          head.in_features <= 1024)
        self.cur = 0  # index of the stack holding the current obs
        self.global_step = 0
        self.log_enabled = log
        self.graphs: dict = {}
        # reset (:333): obs = initial frame stack
        frame = self.env.reset()
        ops.obs_reset(frame, self.stacks[0], self.net_obs)

    # ------------------------------------------------------------------------------------------
    def _env_step(self, k: int, advance: int = 0) -> bool:
        """One global step (:345-372): act, step, store + VecNormalize, replay add. With the
        fused launch (ops.dqn_act_step), `advance` moves the chunk counters in it: True then."""
        a = self.args
        prev, nxt = self.stacks[self.cur], self.stacks[1 - self.cur]
        # global step = chunk base (step_dev, advanced once per chunk) + k + 1
        with torch.no_grad():
            if self.fused_act:
                net = self.q.network
                x = self.net_obs / 255.0 if self.pixels else self.net_obs
                h = fused_trunk(net[:-1], x)
                if FUSED_ACT_STEP and not self.pixels and ops.dqn_act_step_ok(
                        h, net[-1].weight, self.env, prev, self.rb):
                    vn = (self.ret_state, self.rms_state) if a.vecnorm_reward else None
                    ops.dqn_act_step(h, net[-1].weight, net[-1].bias, a.seed, self.step_dev,
                                     a.start_e, a.end_e, self.duration, self.actions,
                                     self.epsilon, k + 1, self.env, k, prev, nxt, self.net_obs,
                                     self.done_out, self.rew_out, self.rb, vecnorm_state=vn,
                                     advance=advance)
                    self.cur = 1 - self.cur
                    return bool(advance)
                ops.q_head_epsilon_greedy(h, net[-1].weight, net[-1].bias, a.seed, self.step_dev,
                                          a.start_e, a.end_e, self.duration, self.actions,
                                          self.epsilon, step_offset=k + 1)
            else:
                q = _q_forward(self.q, self.net_obs)
                ops.epsilon_greedy(q, a.seed, self.step_dev, a.start_e, a.end_e, self.duration,
                                   self.actions, self.epsilon, step_offset=k + 1)
        self.env.step(self.actions, k)
        if a.vecnorm_reward:
            # VecNormalize(envs, norm_obs=False, norm_reward=True) (:298) keeps SB3's default
            # gamma = 0.99 whatever --gamma says (ops' default)
            ops.rollout_store_vecnorm(self.env.frame, self.env.reward, self.env.done, prev, nxt,
                                      self.net_obs, self.done_out, self.ret_state,
                                      self.rms_state, self.rew_out)
        else:
            ops.rollout_store(self.env.frame, self.env.reward, self.env.done, prev, nxt,
                              self.net_obs, self.rew_out, self.done_out)
        self.rb.add(prev, nxt, self.actions, self.rew_out, self.done_out)
        self.cur = 1 - self.cur
        return False

    def _train_step(self):
        """:377-392 — sample, TD target + MSE (fused), backward, Adam."""
        a = self.args
        d = self.rb.sample(a.batch_size, out=self.batch)
        if TARGET_SIDE_STREAM and self.side is not None:
            # the target network's forward on a side stream beside the online forward: two
            # independent launch chains (5 launches each) of one sampled batch, joined before the
            # TD loss -- the same kernels on the same operands, so the same values
            main = torch.cuda.current_stream(self.dev)
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side), torch.no_grad():
                q_next = _q_forward(self.target, d["next_observations"])
            q = _q_forward(self.q, d["observations"])
            main.wait_stream(self.side)
            q_next.record_stream(main)
        else:
            with torch.no_grad():
                q_next = _q_forward(self.target, d["next_observations"])
            q = _q_forward(self.q, d["observations"])
        ops.td_loss_fwd_bwd(q.detach(), q_next, d["actions"], d["rewards"], d["dones"], a.gamma,
                            dq=self.dq, stats=self.td_stats)
        if not self.direct_grads:
            self.opt.zero_grad()
        q.backward(self.dq)
        self.opt.step()

    def _target_update(self):
        """:396-400 — target = tau * q + (1 - tau) * target, parameter by parameter (elementwise:
        the flat buffers hold the same values)."""
        tau = self.args.tau
        self.t_flat.copy_(tau * self.opt.params + (1.0 - tau) * self.t_flat)

    def _chunk(self, train: bool):
        tf = self.args.train_frequency
        moved = False
        for k in range(tf):
            moved = self._env_step(k, advance=tf if k == tf - 1 else 0)
        if not moved:
            self.env.advance(tf)
            self.step_dev.add_(tf)
        if train:
            self._train_step()

    # ------------------------------------------------------------------------------------------
    def _graphable(self) -> bool:
        a = self.args
        return (a.cuda_graphs and a.learning_starts % a.train_frequency == 0 and
                a.target_network_frequency % a.train_frequency == 0 and a.train_frequency % 2 == 0)

    def _run_chunk(self, train: bool):
        key = "train" if train else "fill"
        if not self._graphable():
            return self._chunk(train)
        g = self.graphs.get(key)
        if g is None:
            # warm up eagerly once (creates Adam state / workspaces), then capture
            self._chunk(train)
            torch.cuda.synchronize(self.dev)
            g = torch.cuda.CUDAGraph()
            cur = self.cur
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._chunk(train)
            # capture recorded the work without running it: restore the host-side stack parity
            self.cur = cur
            self.graphs[key] = g
            return
        g.replay()  # train_frequency is even: the stack parity is back where it started

    def steps(self, n: int):
        """Advance `n` global steps (a multiple of train_frequency when graphs are used)."""
        a = self.args
        tf = a.train_frequency
        if self._graphable():
            if n % tf:
                raise ValueError(f"n={n} must be a multiple of train_frequency={tf}")
            for _ in range(n // tf):
                end = self.global_step + tf
                self._run_chunk(train=end > a.learning_starts)
                self.global_step = end
                if end > a.learning_starts and end % a.target_network_frequency == 0:
                    self._target_update()
            return
        for _ in range(n):  # general path: the reference's order step by step
            self.global_step += 1
            self._env_step(0)
            self.env.advance(1)
            self.step_dev.add_(1)
            gs = self.global_step
            if gs > a.learning_starts:
                if gs % tf == 0:
                    self._train_step()
                if gs % a.target_network_frequency == 0:
                    self._target_update()

    def metrics(self) -> dict:
        st = self.td_stats.tolist()
        ep_ret, ep_len, ep_n = self.env.pop_episode_stats()
        m = {"losses/td_loss": st[0], "losses/q_values": st[1],
             "charts/epsilon": float(self.epsilon)}
        if ep_n > 0:
            m["charts/Episodic_Original_Reward"] = ep_ret / ep_n
            m["charts/Episodic_Length"] = ep_len / ep_n
        return m

    def checkpoint(self) -> dict:
        """The `.cleanrl_model` payload of dqn_atari_oc.py:418-423."""
        return {"model_weights": {k: v.detach().clone() for k, v in self.q.state_dict().items()},
                "args": asdict(self.args)}


def run_dqn(args: DQNArgs, device=None) -> DQNTrainer:
    device = device or torch.device("cuda:0")
    tr = DQNTrainer(args, device)
    run_name = f"{args.env_id}__{args.exp_name}__{args.seed}__{int(time.time())}".replace("/", "_")
    run_dir = Path(args.log_dir) / run_name
    run_dir.mkdir(parents=True, exist_ok=True)
    (run_dir / "args.json").write_text(json.dumps(asdict(args), indent=1, default=str))
    start = time.time()
    chunk = max(args.train_frequency, args.log_every - args.log_every % args.train_frequency)
    with open(run_dir / "metrics.jsonl", "w") as w:
        while tr.global_step < args.total_timesteps:
            n = min(chunk, args.total_timesteps - tr.global_step)
            n -= n % args.train_frequency if tr._graphable() else 0
            if n <= 0:
                break
            tr.steps(n)
            m = tr.metrics()
            m["charts/SPS"] = int(tr.global_step * args.num_envs / (time.time() - start))
            m["global_step"] = tr.global_step
            w.write(json.dumps(m) + "\n")
    if args.save_model:
        torch.save(tr.checkpoint(), run_dir / f"{args.exp_name}.cleanrl_model")
    return tr


def main(argv=None):
    args = parse_dataclass(DQNArgs, argv, None, "oc_cleanrl_amd DQN (dqn_atari_oc.py surface)")
    if args.obs_mode not in OBS_MODES:
        raise SystemExit(f"bad obs_mode {args.obs_mode}")
    tr = run_dqn(args)
    print({k: round(v, 5) for k, v in tr.metrics().items()})


if __name__ == "__main__":
    main()
