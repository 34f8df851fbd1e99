"""Experiment: PPObj encoder fwd+bwd time vs row count (the frame-dedup capacity C per minibatch;
16384 = M x W without dedup). hipBLASLt tile quantisation makes time non-monotone in rows."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oc_cleanrl_amd.agents import make_agent  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
ag = make_agent("PPO_OBJ", (4, 12), 6, dev).to(dev)
for p in ag.parameters():
    p.grad = torch.zeros_like(p)
    p._ocppo_direct_grad = True


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


rows = [int(r) for r in sys.argv[1:]] or [10240, 10752, 11264, 11520, 11776, 12032, 12288, 12544,
                                           12800, 13312, 14336, 15360, 16384]
for R in rows:
    x = torch.randn(R, 12, device=dev)
    g = torch.randn(R, 512, device=dev)

    def step():
        enc = ag.encode(x)
        torch.autograd.backward(enc, g)

    def fwd():
        with torch.no_grad():
            ag.encode(x)

    t, tf = timeit(step), timeit(fwd)
    fl = 3 * 2 * R * (12 * 256 + 256 * 512 + 512 * 1024 + 1024 * 512) / 1e12
    print(f"rows={R}: fwd+bwd {t:.1f}us ({fl / (t * 1e-6):.0f} TF)  fwd {tf:.1f}us  "
          f"per-row {t / R * 1e3:.2f}ns", flush=True)
