"""Experiment (CPU): how many ReLU decisions does an f32 forward of the config-2 fixture's first
minibatch take unlike float64's, and how many pre-activations lie within rounding distance of 0?

The config-2 golden test (tests/test_config2_golden_gpu.py) reports that this package's chain takes
2-4 ReLU decisions per minibatch unlike the float64 twin and that those flips set its end-to-end
gradient distance from f64. This restates the reference's own f32 forward (torch CPU, the
fixture's seeded weights and the minibatch's observations, PPObj's layer order) next to an f64
forward, and counts per layer
  * the f32 forward's flips against f64 (what the reference's f32 run did on this minibatch),
  * the pre-activations with |z64| < k * 2^-24 * S (S = sum |w||x| + |b|, the scale of the
    rounding error of ANY f32 evaluation of that dot product) for k = 1, 8, 64: the expected
    number of flips of an f32 forward whose error is about k units of that scale.

    python tools/exp_relu_flips.py
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    from conftest import golden
    from test_config2_golden_gpu import config2_weights

    from oc_cleanrl_amd.agents import PPObj

    z = golden("update_config2.npz")
    from types import SimpleNamespace

    torch.manual_seed(0)
    envs = SimpleNamespace(observation_space=SimpleNamespace(shape=(4, 12)),
                           action_space=SimpleNamespace(n=6))
    agent = PPObj(envs, encoder_dims=(256, 512, 1024, 512), decoder_dims=(512,))
    agent.load_state_dict(config2_weights(agent, int(z["seed"])))
    M = int(z["M"])
    idx = z["perm"][:M].astype(np.int64)
    obs = torch.from_numpy(z["obs"][:128].reshape(-1, 4, 12)[idx]).float()
    lins = [m for m in agent.network if isinstance(m, torch.nn.Linear)]
    out = {"minibatch": 0, "rows": M, "layers": []}
    x32 = obs.reshape(-1, 12)
    x64 = x32.double()
    for i, lin in enumerate(lins):
        if i == len(lins) - 1:  # the decoder: on the flattened stack of W frame encodings
            x32 = x32.reshape(M, -1)
            x64 = x64.reshape(M, -1)
        w, b = lin.weight.detach(), lin.bias.detach()
        z32 = torch.addmm(b, x32, w.t())
        z64 = torch.addmm(b.double(), x64, w.double().t())
        S = x64.abs() @ w.double().abs().t() + b.double().abs()
        rel = (z64.abs() / S)
        rec = {"layer": i, "shape": list(z64.shape), "f32_flips": int(((z32 > 0) != (z64 > 0)).sum()),
               "f32_err_over_S_max": float(((z32.double() - z64).abs() / S).max()),
               "f32_err_over_S_p99": float(torch.quantile(((z32.double() - z64).abs() / S).flatten()[:1 << 24], 0.99))}
        both = (z32 > 0) & (z64 > 0)
        e = ((z32.double() - z64).abs() / S)[both] / 2.0 ** -24
        rec["err_units_p99_max_where_both_positive"] = (round(float(torch.quantile(e[:1 << 24], 0.99)), 2),
                                                        round(float(e.max()), 2))
        for k in (1, 8, 64):
            rec[f"near0_{k}u"] = int((rel < k * 2.0 ** -24).sum())
        out["layers"].append(rec)
        x32 = torch.relu(z32)
        x64 = torch.relu(z64)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
