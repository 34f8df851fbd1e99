"""Experiment: NatureCNN (architectures/ppo.py:15-46) fwd+bwd at the config-3 update minibatch
(8192 x 4 x 84 x 84) and rollout forward (256), NCHW vs channels_last (NHWC) memory format on
MIOpen, plus the input conversion cost."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd.agents import make_agent  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = "--bench" in sys.argv


def timeit(fn, reps=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for fmt in (torch.contiguous_format, torch.channels_last):
    torch.manual_seed(0)
    ag = make_agent("PPO", (4, 84, 84), 4, dev).to(dev).to(memory_format=fmt)
    xb = torch.randint(0, 256, (8192, 4, 84, 84), device=dev, dtype=torch.uint8).float()
    xr = torch.randint(0, 256, (256, 4, 84, 84), device=dev, dtype=torch.uint8).float()
    xb_f, xr_f = xb.contiguous(memory_format=fmt), xr.contiguous(memory_format=fmt)

    def upd():
        lg, v = ag.logits_and_value(xb_f)
        torch.autograd.backward([lg, v], [torch.ones_like(lg), torch.ones_like(v)])

    def roll():
        with torch.no_grad():
            ag.logits_and_value(xr_f)

    def roll_nchw():
        with torch.no_grad():
            ag.logits_and_value(xr)

    print(f"  rollout fwd with an NCHW input: {timeit(roll_nchw, 20):7.3f} ms", flush=True)
    t_conv = timeit(lambda: xb.contiguous(memory_format=fmt).sum()) if fmt != torch.contiguous_format else 0.0
    print(f"{str(fmt):28s} update fwd+bwd {timeit(upd):8.2f} ms   rollout fwd {timeit(roll, 20):7.3f} ms"
          f"   input convert+sum {t_conv:.2f} ms", flush=True)
