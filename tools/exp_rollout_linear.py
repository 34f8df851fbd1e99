"""Rollout-step Linear(+ReLU) layers: hipBLASLt (torch._addmm_activation) vs ocppo_linear_act,
each captured 50x in a hipGraph; max |diff| against an f64 reference relative to sum |a*b|."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd import ops  # noqa: E402
from tools.exp_rollout_gemms import t  # noqa: E402

dev = torch.device("cuda:0")
# (M, K, N): encoder layers at 512 rows (4 frames x 128 envs) and at 128 rows (frame cache),
# decoder 2048 -> 512 and the NatureCNN head 3136 -> 512 at 128 / 256 rows
shapes = [(512, 12, 256), (512, 256, 512), (512, 512, 1024), (512, 1024, 512),
          (128, 12, 256), (128, 256, 512), (128, 512, 1024), (128, 1024, 512), (128, 2048, 512),
          (256, 3136, 512), (1024, 2048, 512)]
for m, k, n in shapes:
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev) * 0.05
    b = torch.randn(n, device=dev)
    out = torch.empty(m, n, device=dev)
    us_t = t(lambda: torch._addmm_activation(b, x, w.t(), use_gelu=False))
    us_h = t(lambda: ops.linear_act(x, w, b, True, out))
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    scale = (x.double().abs() @ w.double().abs().t()).max().item()
    ref_t = torch._addmm_activation(b, x, w.t(), use_gelu=False)
    print(json.dumps({"m": m, "k": k, "n": n, "torch_us": round(us_t, 2), "hip_us": round(us_h, 2),
                      "hip_TFs": round(2 * m * k * n / us_h / 1e6, 1),
                      "err_hip": (out.double() - ref).abs().max().item() / scale,
                      "err_torch": (ref_t.double() - ref).abs().max().item() / scale}), flush=True)
