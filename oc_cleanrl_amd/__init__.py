"""oc_cleanrl_amd — MI355X-native PPO actor-learner for OC-CleanRL (BluemlJ/oc_cleanrl).

The hot path of cleanrl/ppo_atari_oc.py (rollout storage fill → GAE → fused minibatch PPO loss →
PyTorch network fwd/bwd + Adam → RCCL gradient all-reduce) with its memory-bound glue as HIP
kernels for gfx950 behind the C-ABI of include/ocppo.h (libocppo_hip.so, loaded by `_lib`).

Submodules are imported lazily: `ops` and `agents` need the built HIP library.
"""
__all__ = ["ops", "agents", "args", "envs", "trainer"]
__version__ = "0.1.0"
