"""Experiment: NatureCNN conv1 (4 -> 32, 8x8, stride 4 on 84x84) as-is vs as a space-to-depth
conv (64 -> 32, 2x2, stride 1 on 21x21: the same products, the 4x4 phase moved into channels),
NHWC on MIOpen; rollout batch 256 forward and update batch 8192 forward + weight grad."""
import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
CL = torch.channels_last


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def s2d(x):  # [B, 4, 84, 84] -> [B, 64, 21, 21], channel = c*16 + dy*4 + dx
    B = x.shape[0]
    return x.view(B, 4, 21, 4, 21, 4).permute(0, 1, 3, 5, 2, 4).reshape(B, 64, 21, 21)


def w_s2d(w):  # [32, 4, 8, 8] -> [32, 64, 2, 2]
    return w.view(32, 4, 2, 4, 2, 4).permute(0, 1, 3, 5, 2, 4).reshape(32, 64, 2, 2)


w = torch.randn(32, 4, 8, 8, device=dev) * 0.05
ws = w_s2d(w).contiguous(memory_format=CL)
wc = w.contiguous(memory_format=CL)
for B in (256, 8192):
    x = torch.randint(0, 256, (B, 4, 84, 84), device=dev).float() / 255
    xc = x.contiguous(memory_format=CL)
    xs = s2d(x).contiguous(memory_format=CL)
    y1 = torch.ops.aten.convolution(xc, wc, None, (4, 4), (0, 0), (1, 1), False, (0, 0), 1)
    y2 = torch.ops.aten.convolution(xs, ws, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1)
    err = ((y1 - y2).abs().max() / y1.abs().max()).item()
    t1 = timeit(lambda: torch.ops.aten.convolution(xc, wc, None, (4, 4), (0, 0), (1, 1), False,
                                                   (0, 0), 1))
    t2 = timeit(lambda: torch.ops.aten.convolution(xs, ws, None, (1, 1), (0, 0), (1, 1), False,
                                                   (0, 0), 1))
    g = torch.randn_like(y1).contiguous(memory_format=CL)
    tw1 = timeit(lambda: torch.ops.aten.convolution_backward(
        g, xc, wc, None, (4, 4), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)))
    tw2 = timeit(lambda: torch.ops.aten.convolution_backward(
        g, xs, ws, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)))
    print(f"B={B}: fwd 8x8/s4 {t1:8.1f} us  s2d 2x2/s1 {t2:8.1f} us  (rel diff {err:.1e});"
          f"  dW {tw1:8.1f} vs {tw2:8.1f} us", flush=True)

# conv1 at the rollout batch: eager launches vs the same launch replayed from a hipGraph
x = (torch.randint(0, 256, (256, 4, 84, 84), device=dev).float() / 255).contiguous(memory_format=CL)
f = lambda: torch.ops.aten.convolution(x, wc, None, (4, 4), (0, 0), (1, 1), False, (0, 0), 1)  # noqa: E731
t_eager = timeit(f, 50)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    f()
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    for _ in range(20):
        f()
t_graph = timeit(gr.replay, 5) / 20
print(f"rollout conv1 B=256: eager {t_eager:.1f} us, graph-replayed {t_graph:.1f} us", flush=True)
