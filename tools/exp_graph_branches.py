"""Do parallel branches of a captured hipGraph run concurrently? Two streams forked/joined inside
capture, each with a chain of small kernels, vs the same kernels on one stream."""
import json
import torch

dev = torch.device("cuda:0")
a = torch.randn(128, 512, device=dev)
b = torch.randn(128, 512, device=dev)
w = torch.randn(512, 512, device=dev)


def chain(x, n=6):
    for _ in range(n):
        x = torch.relu(x @ w)
    return x


def timed(g, reps=200):
    g.replay(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record(); torch.cuda.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


chain(a); chain(b); torch.cuda.synchronize()
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1):
    chain(a); chain(b)
s2 = torch.cuda.Stream()
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    cur = torch.cuda.current_stream()
    s2.wait_stream(cur)
    chain(a)
    with torch.cuda.stream(s2):
        chain(b)
    cur.wait_stream(s2)
g0 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g0):
    chain(a)
print(json.dumps({"one_chain_us": round(timed(g0), 2), "serial_two_chains_us": round(timed(g1), 2),
                  "forked_two_chains_us": round(timed(g2), 2)}))
