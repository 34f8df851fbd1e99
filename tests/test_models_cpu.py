"""Agents mirror cleanrl/architectures/ppo.py: state-dict keys/shapes, seeded init (same RNG
consumption order → same weights), forward outputs (against tests/golden/init_*.json and
ppobj_small.npz made from the reference modules)."""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden


def _agent(name):
    from oc_cleanrl_amd.agents import make_agent

    info = json.loads((GOLDEN / f"init_{name}.json").read_text())
    torch.manual_seed(info["seed"])
    if name.startswith("ppobj"):
        ag = make_agent("PPO_OBJ", tuple(info["obs_shape"]), info["n_actions"])
    else:
        ag = make_agent("PPO", tuple(info["obs_shape"]), info["n_actions"])
    return ag, info


@pytest.mark.parametrize("name", ["ppobj_f12_a6", "ppodefault_a4"])
def test_state_dict_layout_and_seeded_init(name):
    ag, info = _agent(name)
    sd = ag.state_dict()
    assert list(sd) == list(info["params"])  # same keys, same order
    assert sum(p.numel() for p in ag.parameters()) == info["num_params"]
    for k, v in sd.items():
        ref = info["params"][k]
        assert list(v.shape) == ref["shape"]
        np.testing.assert_allclose(float(v.double().sum()), ref["sum"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(float(v.double().abs().sum()), ref["abs_sum"], rtol=1e-6)


@pytest.mark.parametrize("name", ["ppobj_f12_a6", "ppodefault_a4"])
def test_seeded_forward_matches_reference(name):
    ag, info = _agent(name)
    rng = np.random.default_rng(info["seed"])
    x = torch.from_numpy((rng.random((4,) + tuple(info["obs_shape"])) * info["x_scale"])
                         .astype(np.float32).round())
    with torch.no_grad():
        logits, value = ag.logits_and_value(x)
    np.testing.assert_allclose(logits.double().numpy(), np.array(info["logits"]), rtol=1e-4,
                               atol=1e-6)
    np.testing.assert_allclose(value.double().numpy(), np.array(info["value"]), rtol=1e-4,
                               atol=1e-5)


def test_reference_state_dict_loads_and_matches():
    from oc_cleanrl_amd.agents import make_agent

    z = golden("ppobj_small.npz")
    ag = make_agent("PPO_OBJ", (4, 6), 6, None, tuple(z["encoder_dims"]), tuple(z["decoder_dims"]))
    sd = {k[4:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("sd::")}
    ag.load_state_dict(sd, strict=True)
    with torch.no_grad():
        x = torch.from_numpy(z["x"])
        logits, _ = ag.logits_and_value(x)
        np.testing.assert_allclose(logits.numpy(), z["logits"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(ag.get_value(x).numpy(), z["value"], rtol=1e-6, atol=1e-6)


def test_action_api_fails_loudly_on_cpu():
    from oc_cleanrl_amd.agents import make_agent

    ag = make_agent("PPO_OBJ", (4, 6), 6, None, (8,), (8,))
    with pytest.raises(ValueError, match="GPU"):
        ag.get_action_and_value(torch.zeros(2, 4, 6))


def test_unsupported_architecture():
    from oc_cleanrl_amd.agents import make_agent

    with pytest.raises(NotImplementedError):
        make_agent("OCT", (4, 6), 6)


def test_predict_greedy():
    from oc_cleanrl_amd.agents import make_agent

    torch.manual_seed(0)
    ag = make_agent("PPO_OBJ", (4, 6), 6, None, (8,), (8,))
    x = np.random.default_rng(0).random((5, 4, 6)).astype(np.float32)
    a, _ = ag.predict(x)
    with torch.no_grad():
        ref = ag.actor(ag.network(torch.from_numpy(x))).argmax(1).numpy()
    assert np.array_equal(a, ref)


def test_gemm_table_file_is_a_tunableop_table():
    """The shipped hipBLASLt solution table (gemm_table.py): TunableOp's CSV with its validators
    (PyTorch version of this image, gfx950) and one solution per GEMM signature, hipBLASLt
    solutions or the default only (no rocBLAS entries: those lose under hipGraph replay)."""
    import csv

    import torch

    from oc_cleanrl_amd import gemm_table

    rows = list(csv.reader(open(gemm_table.TABLE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["PT_VERSION"] == torch.__version__.split("+")[0]
    assert val["GCN_ARCH_NAME"].startswith("gfx950")
    entries = [r for r in rows if r[0] != "Validator"]
    assert len(entries) == len({(r[0], r[1]) for r in entries}) > 0
    assert all(r[2] == "Default" or r[2].startswith("Gemm_Hipblaslt_") for r in entries)
    # config 2's encoder / decoder GEMM shapes are in it
    sigs = {r[1] for r in entries}
    assert "tn_1024_11520_512_ld_512_512_1024" in sigs and "nn_2048_4096_512_ld_2048_512_2048" in sigs


def test_gemm_table_not_used_off_gpu():
    from oc_cleanrl_amd import gemm_table

    gemm_table._state.clear()
    try:
        assert gemm_table.use("cpu") is False
    finally:
        gemm_table._state.clear()
