"""ctypes binding of libocppo_hip.so (the C-ABI declared in include/ocppo.h).

torch is imported first on purpose: torch ships libamdhip64.so with soname libamdhip64.so.7, and
libocppo_hip.so's NEEDED entry is that soname, so loading ours after torch reuses torch's HIP
runtime (one runtime per process, shared streams and graph capture).

There is no CPU fallback: if the library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

PKG = Path(__file__).resolve().parent
# OCPPO_LIB: load another build of the same C-ABI (experiments, e.g. a probe variant); default
# is the in-tree build
LIB_PATH = Path(os.environ.get("OCPPO_LIB", PKG / "lib" / "libocppo_hip.so"))
HEADER = PKG.parent / "include" / "ocppo.h"

# constants mirrored from include/ocppo.h (checked against the header by tests/test_abi.py)
OCPPO_ABI_VERSION = 28
OCPPO_OK, OCPPO_E_INVALID, OCPPO_E_LAUNCH, OCPPO_E_WORKSPACE = 0, 1, 2, 3
OCPPO_F32, OCPPO_BF16, OCPPO_U8 = 0, 1, 2
OCPPO_X6_MBITS_ROWS = 2
STAT_NAMES = ("loss", "pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac",
              "adv_mean", "adv_std")
OCPPO_NUM_STATS = len(STAT_NAMES)

P, I64, U64, D, I, SZ = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double,
                         ctypes.c_int, ctypes.c_size_t)

SIGNATURES: dict[str, tuple[type, list]] = {
    "ocppo_abi_version": (I, []),
    "ocppo_last_error": (ctypes.c_char_p, []),
    "ocppo_gae": (I, [P, P, P, P, P, P, I64, I64, D, D, P, P]),
    "ocppo_minibatch_adv_stats": (I, [P, P, P, I64, I64, P]),
    "ocppo_minibatch_prepare": (I, [P, P, I64, I64, P, P, P, P, P, P, P, P, P, P, P]),
    "ocppo_ppo_loss_workspace_bytes": (SZ, [I64, I64]),
    "ocppo_ppo_loss_fwd_bwd": (I, [P, P, P, I64, I64, P, P, P, P, P, P, P, D, D, D, I, I, P, P, P,
                                   P, SZ]),
    "ocppo_clip_adam_workspace_bytes": (SZ, [I64]),
    "ocppo_clip_adam_step": (I, [P, P, P, P, P, I64, P, D, D, D, D, D, P, P, SZ, I, P, P, P, P,
                                 P]),
    "ocppo_categorical_sample": (I, [P, P, P, P, I64, I64, I64, I64, P, P, P, P, P]),
    "ocppo_policy_head_sample": (I, [P, P, I64, I64, P, P, P, P, P, P, I64, I64, I64, P, P, P, P,
                                     P]),
    "ocppo_torch_exponential_geometry": (I, [I64, I64, I64, P, P]),
    "ocppo_philox_exponential": (I, [P, P, I64, P, I64, I64]),
    "ocppo_philox_exponential_steps": (I, [P, P, I64, I64, P, I64, I64, I64]),
    "ocppo_categorical_logprob_entropy": (I, [P, P, P, I64, I64, P, P]),
    "ocppo_categorical_logprob_entropy_bwd": (I, [P, P, P, P, P, I64, I64, P]),
    "ocppo_rollout_store": (I, [P, P, I, P, P, I64, I64, I64, P, P, I, P, P, P, I, P]),
    "ocppo_obs_reset": (I, [P, P, I, I64, I64, I64, P, I, P, I]),
    "ocppo_gather_rows": (I, [P, P, I, P, I64, I64, P]),
    "ocppo_gather_rows_cl": (I, [P, P, I, P, I64, I64, I64, P, I]),
    "ocppo_frame_cache_shift": (I, [P, P, P, I64, P, I64, I64, I64]),
    "ocppo_linear_act": (I, [P, P, I64, P, P, P, I64, I64, I64, I64, I]),
    "ocppo_linear2_act": (I, [P, P, I64, P, P, P, P, P, I64, I64, I64, I64, I64, I, I]),
    "ocppo_relu_bias_grad_workspace_bytes": (SZ, [I64, I64]),
    "ocppo_relu_bias_grad": (I, [P, P, P, P, P, I64, I64, P, SZ]),
    "ocppo_relu_bias_grad_bits": (I, [P, P, P, P, P, I64, I64, P, SZ]),
    "ocppo_relu_bias_grad_chunks": (I64, [I64, I64]),
    "ocppo_relu_bias_grad_partial": (I, [P, P, P, P, P, I64, I64]),
    "ocppo_sum_splits_db": (I, [P, P, I64, I64, P, P, I64, I64, P]),
    "ocppo_relu_bias_wgrad_workspace_bytes": (SZ, [I64, I64, I64]),
    "ocppo_relu_bias_wgrad": (I, [P, P, P, P, I64, P, P, I64, I64, I64, P, SZ]),
    "ocppo_relu_bias_wgrad_rows": (I, [P, P, P, P, I64, P, P, I64, I64, I64, P, SZ, P]),
    "ocppo_sum_splits_db_finish": (I, [P, P, I64, I64, P, P, I64, I64, P, P]),
    "ocppo_heads_bwd_workspace_bytes": (SZ, [I64, I64, I64]),
    "ocppo_heads_bwd": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I64, I64, I64, I, P, SZ]),
    "ocppo_bias_act": (I, [P, P, P, I64, I64, I]),
    "ocppo_bias_act_nchw": (I, [P, P, P, I64, I64, I64, I, P]),
    "ocppo_sum_splits": (I, [P, P, I64, I64, P]),
    "ocppo_frames_gather": (I, [P, P, I, I64, I64, I64, I64, P, I64, P]),
    "ocppo_frames_expand": (I, [P, P, I64, I64, P, P, I64, P, I64, I64, I64, P]),
    "ocppo_frames_scatter": (I, [P, P, I64, I64, P, I64, P, I64, P, I64, I64, I64, P]),
    "ocppo_vecnorm_reward": (I, [P, P, P, I64, D, D, D, P, P, P]),
    "ocppo_rollout_store_vecnorm": (I, [P, P, I, P, P, I64, I64, I64, P, P, I, P, P, D, D, D, P,
                                        P, P, I, P]),
    "ocppo_replay_workspace_bytes": (SZ, []),
    "ocppo_replay_add": (I, [P, P, P, I, P, P, P, I64, I64, P, I64, P, I, P, P, P, P]),
    "ocppo_replay_sample": (I, [P, U64, P, P, I64, I64, I64, P, I, P, P, P, I64, P, P, P, P, P,
                                P]),
    "ocppo_epsilon_greedy": (I, [P, P, I64, I64, U64, P, I64, D, D, D, P, P]),
    "ocppo_td_loss_fwd_bwd": (I, [P, P, P, P, P, P, I64, I64, D, P, P]),
    "ocppo_synth_env_step": (I, [P, U64, P, I64, P, I64, I64, I, P, P, P, P]),
    "ocppo_policy_head_env_step": (I, [P, P, I64, I64, P, P, P, P, P, P, I64, I64, I64, P, P, P,
                                       U64, P, I64, I64, P, P, P, P]),
    "ocppo_cartpole_step": (I, [P, U64, P, I64, P, P, P, P, P, P]),
    "ocppo_heads_loss_workspace_bytes": (SZ, [I64, I64, I64]),
    "ocppo_heads_loss_fwd_bwd": (I, [P, P, I64, I64, P, P, P, P, I64, P, P, P, P, P, P, D, D, D, I,
                                     I, P, P, P, P, P, P, P, P, P, P, SZ]),
    "ocppo_heads_loss_rows": (I, [P, P, I64, I64, P, P, P, P, I64, P, P, P, P, P, P, D, D, D, I,
                                  I, P, P, P, P, P, P, P, P, P, P, SZ, P]),
    "ocppo_sum_splits_finish": (I, [P, P, I64, I64, P, P]),
    "ocppo_sum_splits_act": (I, [P, P, I64, I64, I64, P, I, P]),
    "ocppo_gemm_x6_gather": (I, [P, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64, P,
                                 I, P, P, I64, I64, I]),
    "ocppo_frames_expand_index": (I, [P, P, P, I64, P, I64, I64, I64, P]),
    "ocppo_gemm_x6_wgrad": (I, [P, P, I64, I64, P, I64, I64, I64, I64, I64, P, I64, P, I64, I64,
                                P, P, P, I64, I, P]),
    "ocppo_conv_x6": (I, [P, I, P, P, P, I64, P, I64, I64, I64, I64, I64, P, I, P, I, P, P, P,
                          P, P, P]),
    "ocppo_conv_x6_u8": (I, [P, I, P, P, I64, I64, I64, I64, I64, I64, P, I64, P, I64, I64, I64,
                             I64, P, I, ctypes.c_float, I, P, P, P, P]),
    "ocppo_deferred_finish_run": (I, [P, P]),
    "ocppo_linear_cache_shift": (I, [P, P, I64, P, P, P, P, I64, I64, I64, I64, I]),
    "ocppo_linear_cache_ring": (I, [P, P, I64, P, P, P, P, I64, I64, I64, I64, I64, I]),
    "ocppo_linear_act_ring": (I, [P, P, I64, P, P, P, I64, I64, I64, I64, I64, I64, I]),
    "ocppo_conv2d_act": (I, [P, P, I64, I64, I64, I64, P, P, I64, I64, I64, I64, P, I]),
    "ocppo_frames_scatter_chunks": (I64, [I64]),
    "ocppo_frames_gather_linear": (I, [P, P, I, I64, I64, I64, I64, P, I64, P, P, I64, I, P, P, P,
                                       P, I64, P, P]),
    "ocppo_q_head_epsilon_greedy": (I, [P, P, I64, I64, P, P, I64, U64, P, I64, D, D, D, P, P, P]),
    "ocppo_dqn_act_step": (I, [P, P, I64, I64, P, P, I64, U64, P, I64, D, D, D, P, P, U64, P, I64,
                               I64, P, P, P, P, I64, P, P, I, P, P, P, I, D, D, D, P, P, P, I64, P,
                               P, P, P, I64]),
    "ocppo_frames_scatter_relu": (I, [P, P, I64, I64, P, I64, P, I64, P, I64, I64, I64, P, P, P,
                                      P]),
    "ocppo_gemm_x6": (I, [P, P, I64, I64, P, I64, I64, P, I64, I64, I64, I64, I64, I64, P, I, P,
                          I64, P, P, P, I, I, P, I64, I64, P, SZ]),
    "ocppo_gemm_x6_sk_workspace_bytes": (SZ, [I]),
    "ocppo_split_planes": (I, [P, I, P, P, P, P, P, P]),
    "ocppo_gae_records": (I, [P, P, P, P, P, P, I64, I64, D, D, P, P, P, P, P]),
    "ocppo_minibatch_prepare_records": (I, [P, P, I64, I64, P, P, P, P, P, P, P]),
    "ocppo_store_linear2": (I, [P, P, P, P, I64, I64, I64, P, P, I, P, P, P, I, D, D, D, P, P, P,
                                P, P, P, P, I64, I64, I64]),
}


class OcppoError(RuntimeError):
    """A C-ABI call returned a non-zero status."""


def header_functions() -> list[str]:
    """Names of every function the header declares (the ABI contract)."""
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]*?\b(ocppo_\w+)\s*\(", text, re.M)))


def _load() -> ctypes.CDLL:
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} is missing: the HIP extension is required (no CPU fallback). "
            "Build it with `python -m oc_cleanrl_amd.build`.")
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (restype, argtypes) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    ver = lib.ocppo_abi_version()
    if ver != OCPPO_ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {ver}, expected {OCPPO_ABI_VERSION}; rebuild")
    return lib


LIB = _load()


def call(name: str, *args) -> None:
    """Invoke a status-returning entry point and raise OcppoError on failure."""
    rc = getattr(LIB, name)(*args)
    if rc != OCPPO_OK:
        msg = LIB.ocppo_last_error().decode(errors="replace")
        raise OcppoError(f"{name} failed (status {rc}): {msg}")
