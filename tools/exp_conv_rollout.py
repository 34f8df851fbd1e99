"""Experiment: the NatureCNN convolutions of the rollout forward (channels_last, batch = envs) --
ops.conv2d_act (implicit GEMM on the f32 MFMA, bias + ReLU fused) vs the _ConvAct forward it would
replace (MIOpen NHWC convolution + channels_last copy + ops.bias_act), each timed in a hipGraph of
back-to-back launches; correctness vs an f64 conv.

    python tools/exp_conv_rollout.py [B ...]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from oc_cleanrl_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
torch.backends.cudnn.deterministic = False
torch.backends.cudnn.benchmark = os.environ.get("CONV_BENCHMARK", "0") == "1"  # MIOpen Find
CL = torch.channels_last
LAYERS = [(4, 32, 8, 4, 84), (32, 64, 4, 2, 20), (64, 64, 3, 1, 9)]  # Cin, Cout, k, stride, H


def timeit(fn, reps=20):
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
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3


def miopen_path(x, w, b, stride):
    y = torch.ops.aten.convolution(x, w, None, (stride, stride), (0, 0), (1, 1), False, (0, 0), 1)
    y = y.contiguous(memory_format=CL)
    ops.bias_act(y.permute(0, 2, 3, 1).reshape(-1, y.shape[1]), b, True)
    return y


for B in [int(v) for v in sys.argv[1:]] or [256, 128]:
    for Cin, Cout, k, s, H in LAYERS:
        x = torch.rand(B, Cin, H, H, device=dev).contiguous(memory_format=CL)
        w = (torch.randn(Cout, Cin, k, k, device=dev) * (Cin * k * k) ** -0.5).contiguous(
            memory_format=CL)
        b = torch.randn(Cout, device=dev) * 0.1
        ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), stride=s))
        y = ops.conv2d_act(x, w, b, s)
        err = float((y.double() - ref).abs().max() / ref.abs().max())
        y2 = miopen_path(x, w, b, s)
        err2 = float((y2.double() - ref).abs().max() / ref.abs().max())
        t_ours = timeit(lambda: ops.conv2d_act(x, w, b, s, out=y))
        t_mi = timeit(lambda: miopen_path(x, w, b, s))
        OH = (H - k) // s + 1
        fl = 2 * B * OH * OH * Cout * Cin * k * k
        print(json.dumps({"B": B, "layer": f"{Cin}->{Cout} {k}x{k}/{s} on {H}x{H}",
                          "ours_us": round(t_ours, 2), "ours_tf": round(fl / t_ours / 1e6, 1),
                          "miopen_path_us": round(t_mi, 2), "err": f"{err:.1e}",
                          "err_miopen": f"{err2:.1e}"}), flush=True)
