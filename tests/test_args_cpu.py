"""The Args surface mirrors cleanrl/ppo_atari_oc.py:63-190 (names + defaults) with a tyro-like
CLI, and the derived DP sizes follow ppo_atari_multigpu.py:166-173."""
import ast
from pathlib import Path

import pytest

REF_SCRIPT = Path("/root/reference/cleanrl/ppo_atari_oc.py")


def test_defaults_match_reference_fields():
    from oc_cleanrl_amd.args import Args

    a = Args()
    # hyper-parameters of the hot path (ppo_atari_oc.py:119-168)
    assert (a.learning_rate, a.num_steps, a.gamma, a.gae_lambda) == (2.5e-4, 128, 0.99, 0.95)
    assert (a.num_minibatches, a.update_epochs, a.clip_coef, a.ent_coef) == (4, 4, 0.1, 0.01)
    assert (a.vf_coef, a.max_grad_norm, a.target_kl, a.norm_adv, a.clip_vloss) == \
        (0.5, 0.5, None, True, True)
    assert a.encoder_dims == (256, 512, 1024, 512) and a.decoder_dims == (512,)
    assert (a.seed, a.num_envs, a.total_timesteps, a.buffer_window_size) == (42, 10, 10_000_000, 4)


@pytest.mark.skipif(not REF_SCRIPT.exists(), reason="reference checkout not mounted")
def test_every_reference_field_exists():
    from oc_cleanrl_amd.args import Args

    tree = ast.parse(REF_SCRIPT.read_text())
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "Args")
    names = [s.target.id for s in cls.body if isinstance(s, ast.AnnAssign)]
    missing = [n for n in names if not hasattr(Args(), n)]
    assert not missing, missing


def test_cli_forms():
    from oc_cleanrl_amd.args import parse_args

    a = parse_args(["--num-envs", "8", "--num_steps", "32", "--no-anneal-lr", "--norm_adv", "False",
                    "--encoder-dims", "32", "64", "--target-kl", "0.02", "--obs_mode", "obj"])
    assert (a.num_envs, a.num_steps, a.anneal_lr, a.norm_adv) == (8, 32, False, False)
    assert a.encoder_dims == (32, 64) and a.target_kl == 0.02 and a.obs_mode == "obj"
    assert parse_args(["--cuda"]).cuda is True
    with pytest.raises(SystemExit):
        parse_args(["--obs_mode", "rgb"])


def test_derived_sizes_single_and_dp():
    from oc_cleanrl_amd.args import Args, finalize

    a = finalize(Args(num_envs=128, architecture="PPO_OBJ", obs_mode="obj"), 1)
    assert (a.batch_size, a.minibatch_size, a.num_iterations) == (16384, 4096, 610)
    assert a.local_num_envs == 128 and a.local_minibatch_size == 4096
    b = finalize(Args(num_envs=1024, architecture="PPO_OBJ", obs_mode="obj"), 8)
    assert (b.local_num_envs, b.local_batch_size, b.local_minibatch_size) == (128, 16384, 4096)
    assert (b.batch_size, b.minibatch_size) == (131072, 32768)
    with pytest.raises(AssertionError):
        finalize(Args(obs_mode="obj", architecture="PPO"), 1)
    with pytest.raises(NotImplementedError):
        finalize(Args(obs_mode="masked_dqn_bin"), 1)
