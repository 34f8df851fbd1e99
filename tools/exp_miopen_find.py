"""Experiment: MIOpen's default (immediate-mode) convolution solutions for the NatureCNN update vs
the ones its Find search picks (torch.backends.cudnn.benchmark), recorded into a user find-db
under MIOPEN_USER_DB_PATH so that later runs reuse them without searching.

    MIOPEN_USER_DB_PATH=<dir> python tools/exp_miopen_find.py [B]
"""
import json
import os
import sys
import time

import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
CL = torch.channels_last
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
LAYERS = [(4, 32, 8, 4, 84), (32, 64, 4, 2, 20), (64, 64, 3, 1, 9)]  # Cin, Cout, k, stride, H


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def ops_for(Cin, Cout, k, s, H):
    x = torch.rand(B, Cin, H, H, device=dev).contiguous(memory_format=CL)
    w = (torch.randn(Cout, Cin, k, k, device=dev) * 0.05).contiguous(memory_format=CL)
    y = torch.ops.aten.convolution(x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1)
    g = torch.randn_like(y).contiguous(memory_format=CL)
    conv = lambda: torch.ops.aten.convolution(x, w, None, (s, s), (0, 0), (1, 1), False,  # noqa
                                              (0, 0), 1)
    bwd = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
        g, x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1, (Cin != 4, True, False))
    return conv, bwd


print(json.dumps({"db": os.environ.get("MIOPEN_USER_DB_PATH"), "B": B}), flush=True)
res = {}
for bench in (False, True):
    torch.backends.cudnn.benchmark = bench
    for L in LAYERS:
        conv, bwd = ops_for(*L)
        t0 = time.time()
        conv()
        bwd()
        torch.cuda.synchronize()
        first = time.time() - t0
        res[(bench, L)] = (timeit(conv), timeit(bwd), first)
        print(json.dumps({"benchmark": bench, "layer": f"{L[0]}->{L[1]} {L[2]}x{L[2]}/{L[3]}",
                          "fwd_us": round(res[(bench, L)][0], 1),
                          "bwd_us": round(res[(bench, L)][1], 1),
                          "first_call_s": round(first, 2)}), flush=True)
