"""Experiment: per-layer time of the NatureCNN update at the config-3 minibatch (8192) in NHWC on
MIOpen: forward, backward-data and backward-weights of each convolution, plus the 3136->512 head."""
import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
CL = torch.channels_last
B = 8192


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
    return a.elapsed_time(b) / reps * 1e3


layers = [(4, 32, 8, 4, 84), (32, 64, 4, 2, 20), (64, 64, 3, 1, 9)]  # cin, cout, k, s, in size
total = 0.0
for cin, cout, k, s, hw in layers:
    x = torch.rand(B, cin, hw, hw, device=dev).contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=CL)
    conv = lambda: torch.ops.aten.convolution(x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1)  # noqa: E731
    y = conv()
    g = torch.randn_like(y).contiguous(memory_format=CL)
    tf = timeit(conv)
    tx = timeit(lambda: torch.ops.aten.convolution_backward(
        g, x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)))
    tw = timeit(lambda: torch.ops.aten.convolution_backward(
        g, x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)))
    ho = y.shape[2]
    fl = 2 * B * ho * ho * cout * cin * k * k / 1e9
    total += tf + tw + (tx if cin != 4 else 0)
    print(f"conv {cin}->{cout} k{k} s{s} ({fl:.1f} GFLOP): fwd {tf:7.1f} us ({fl / tf * 1e-3:5.0f} TF)"
          f"  dX {tx:7.1f} us ({fl / tx * 1e-3:5.0f} TF)  dW {tw:7.1f} us ({fl / tw * 1e-3:5.0f} TF)",
          flush=True)
print(f"conv total per minibatch (no dX for conv1): {total:.0f} us", flush=True)
