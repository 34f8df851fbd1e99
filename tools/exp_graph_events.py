"""Experiment: can hipEventRecordWithFlags(..., hipEventRecordExternal) bracket a kernel inside a
captured hipGraph on this ROCm (torch refuses external events on ROCm)?"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from oc_cleanrl_amd import ops  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipEventRecordWithFlags.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
hip.hipEventRecordWithFlags.restype = ctypes.c_int
hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]

dev = torch.device("cuda:0")
M, A = 4096, 6
logits = torch.randn(M, A, device=dev)
v = torch.randn(M, device=dev)
B = 16384
acts = torch.randint(0, A, (B,), device=dev)
lp, adv, ret, val = (torch.randn(B, device=dev) for _ in range(4))
idx = torch.randperm(B, device=dev)[:M]
ws = ops.LossWorkspace(M, A, dev)
st = torch.empty(9, device=dev)
dl = torch.empty(M, A, device=dev)
dv = torch.empty(M, device=dev)


def call():
    ops.ppo_loss_fwd_bwd(logits, v, acts, lp, adv, ret, val, mb_inds=idx, clip_coef=0.1,
                         ent_coef=0.01, vf_coef=0.5, norm_adv=True, clip_vloss=True,
                         dlogits=dl, dvalue=dv, stats=st, workspace=ws)


call()
torch.cuda.synchronize()
evs = []
for _ in range(2):
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 0) == 0
    evs.append(e)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    s = torch.cuda.current_stream().cuda_stream
    r0 = hip.hipEventRecordWithFlags(evs[0], s, 1)
    for _ in range(16):
        call()
    r1 = hip.hipEventRecordWithFlags(evs[1], s, 1)
print("record rc", r0, r1)
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    rc = hip.hipEventElapsedTime(ctypes.byref(ms), evs[0], evs[1])
    print("replay", i, "rc", rc, "16 launches ms", ms.value, "per launch us", ms.value * 1e3 / 16)
# eager reference timing
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(16):
    call()
e1.record()
torch.cuda.synchronize()
print("eager 16 launches ms", e0.elapsed_time(e1))
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0.record()
g.replay()
t1.record()
torch.cuda.synchronize()
print("graph replay (16 launches) ms", t0.elapsed_time(t1))
