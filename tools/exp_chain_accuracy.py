"""Per-op accuracy of the update GEMMs on the config-2 golden's REAL operands (experiment).

The reference's update (ppo_atari_oc.py:566-606) on update_config2.npz's minibatch 0 is run in
float64 on the GPU with autograd (PPObj module order, architectures/ppo.py:60-95), keeping every
layer's input, pre-activation, and their gradients. Each Linear's three products are then redone
from the f32-rounded f64 operands by: the f32 CPU GEMM (what the reference ran), hipBLASLt f32,
and ocppo_gemm_x6 — and compared with the f64 result, relative to the result's largest element
(the golden's metric) and to |A||B| (the GEMM tests' metric), plus the sign bias of the error.

    python tools/exp_chain_accuracy.py > gpurun_out/chain_acc.jsonl
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from oc_cleanrl_amd import ops  # noqa: E402
from oc_cleanrl_amd.agents import make_agent  # noqa: E402
from test_config2_golden_gpu import config2_weights  # noqa: E402

DEV = torch.device("cuda:0")


def stats(c, ref, sab):
    d = c.double().to(ref.device) - ref
    return {"err_max": float(d.abs().max() / ref.abs().max()),
            "err_sab": float((d.abs() / sab.clamp_min(1e-300)).max()),
            "bias": float((torch.sign(ref) * d).mean() / d.abs().mean().clamp_min(1e-300))}


def main():
    z = np.load(ROOT / "tests" / "golden" / "update_config2.npz")
    T, N, W, F, A = 128, 128, 4, 12, 6
    M = int(z["M"])
    agent = make_agent("PPO_OBJ", (W, F), A)
    agent.load_state_dict(config2_weights(agent, int(z["seed"])))
    agent = agent.double().to(DEV)
    obs = torch.from_numpy(z["obs"][:T].reshape(T * N, W, F).astype(np.float64)).to(DEV)
    mb = torch.from_numpy(z["perm"][:M]).to(DEV)
    x = obs[mb]
    lins = [m for m in agent.network if isinstance(m, torch.nn.Linear)]
    # forward, keeping each Linear's input and output (pre-activation)
    acts = []
    h = x
    for m in agent.network:
        if isinstance(m, torch.nn.Linear):
            inp = h.reshape(-1, h.shape[-1])
            h = m(h)
            h.retain_grad()
            acts.append((inp, h))
        else:
            h = m(h)
    logits, value = agent.actor(h), agent.critic(h)
    act = torch.from_numpy(z["actions"]).to(DEV)[mb]
    lp_old = torch.from_numpy(z["logprobs"]).double().to(DEV)[mb]
    adv = torch.from_numpy(z["advantages"]).double().to(DEV)[mb]
    ret = torch.from_numpy(z["returns"]).double().to(DEV)[mb]
    val_old = torch.from_numpy(z["values"]).double().to(DEV)[mb]
    dist = torch.distributions.Categorical(logits=logits)
    ratio = (dist.log_prob(act) - lp_old).exp()
    adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    pg = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 0.9, 1.1)).mean()
    v = value.view(-1)
    vc = val_old + torch.clamp(v - val_old, -0.1, 0.1)
    vl = 0.5 * torch.max((v - ret) ** 2, (vc - ret) ** 2).mean()
    loss = pg - 0.01 * dist.entropy().mean() + 0.5 * vl
    loss.backward()
    names = [n for n, m in agent.network.named_children() if isinstance(m, torch.nn.Linear)]
    for name, lin, (inp, out) in zip(names, lins, acts):
        gz = out.grad.reshape(-1, out.shape[-1])  # d loss / d pre-activation (f64)
        Wt = lin.weight.detach()
        x64 = inp.detach()
        R, K = x64.shape
        Nn = Wt.shape[0]
        x32, w32, g32 = x64.float(), Wt.float(), gz.float()
        rec = {"layer": f"network.{name}", "rows": R, "in": K, "out": Nn}
        # dW = g^T x
        ref = gz.t() @ x64
        sab = gz.abs().t() @ x64.abs()
        rec["dW"] = {"cpu_f32": stats(g32.cpu().t() @ x32.cpu(), ref, sab),
                     "hipblaslt": stats(g32.t() @ x32, ref, sab)}
        S = 16 if R % (32 * 16) == 0 else 8
        if R % 32 == 0 and ops.x6_tile(Nn, K, S) is not None and K % 4 == 0 and Nn % 4 == 0:
            part = torch.empty(S, Nn, K, device=DEV)
            c = torch.empty(Nn, K, device=DEV)
            t = ops.x6_tile(Nn, K, S)
            ops.gemm_x6(g32, 1, Nn, x32, 1, K, part, K, Nn, K, R, splits=S, split_c=Nn * K,
                        tile=t)
            ops.sum_splits(part, c)
            rec["dW"][f"x6_s{S}"] = stats(c, ref, sab)
        # dX = g W
        if name != "0":
            ref = gz @ Wt
            sab = gz.abs() @ Wt.abs()
            rec["dX"] = {"cpu_f32": stats(g32.cpu() @ w32.cpu(), ref, sab),
                         "hipblaslt": stats(g32 @ w32, ref, sab)}
            if Nn % 32 == 0 and ops.x6_tile(R, K) is not None:
                c = torch.empty(R, K, device=DEV)
                ops.gemm_x6(g32, Nn, 1, w32, 1, K, c, K, R, K, Nn)
                rec["dX"]["x6"] = stats(c, ref, sab)
        # forward z = x W^T (no bias)
        ref = x64 @ Wt.t()
        sab = x64.abs() @ Wt.abs().t()
        rec["fwd"] = {"cpu_f32": stats(x32.cpu() @ w32.cpu().t(), ref, sab),
                      "hipblaslt": stats(x32 @ w32.t(), ref, sab)}
        if K % 32 == 0 and ops.x6_tile(R, Nn) is not None:
            c = torch.empty(R, Nn, device=DEV)
            ops.gemm_x6(x32, K, 1, w32, K, 1, c, Nn, R, Nn, K)
            rec["fwd"]["x6"] = stats(c, ref, sab)
        print(json.dumps(rec), flush=True)


def flips():
    """The f32 forward of each route CHAINED through the encoder + decoder (each layer fed the
    route's own previous output, as in training): ReLU decisions that differ from f64, per layer,
    and how much gradient they carry (sum of |d loss / d z| over the flipped elements, relative
    to the largest column sum of |g| — an upper bound of the bias-gradient error they cause)."""
    z = np.load(ROOT / "tests" / "golden" / "update_config2.npz")
    T, N, W, F, A = 128, 128, 4, 12, 6
    M = int(z["M"])
    agent = make_agent("PPO_OBJ", (W, F), A)
    agent.load_state_dict(config2_weights(agent, int(z["seed"])))
    a64 = make_agent("PPO_OBJ", (W, F), A)
    a64.load_state_dict(agent.state_dict())
    a64 = a64.double().to(DEV)
    obs = torch.from_numpy(z["obs"][:T].reshape(T * N, W, F).astype(np.float64))
    mb = torch.from_numpy(z["perm"][:M])
    x = obs[mb]
    lins64 = [m for m in a64.network if isinstance(m, torch.nn.Linear)]

    def chain(route):
        h = x.float().to(DEV) if route != "cpu_f32" else x.float()
        zs = []
        for m in a64.network:
            if isinstance(m, torch.nn.Linear):
                w = m.weight.detach().float()
                b = m.bias.detach().float()
                h2 = h.reshape(-1, h.shape[-1])
                if route == "cpu_f32":
                    zz = torch.addmm(b.cpu(), h2, w.cpu().t())
                elif route == "x6" and h2.shape[1] % 32 == 0 and ops.x6_tile(h2.shape[0], w.shape[0]) is not None:
                    zz = torch.empty(h2.shape[0], w.shape[0], device=DEV)
                    ops.gemm_x6(h2, h2.shape[1], 1, w, w.shape[1], 1, zz, w.shape[0],
                                h2.shape[0], w.shape[0], h2.shape[1], bias=b)
                else:
                    zz = torch.addmm(b, h2, w.t())
                zs.append(zz.cpu().double())
                h = zz.reshape(*h.shape[:-1], zz.shape[-1])
            elif isinstance(m, torch.nn.ReLU):
                h = torch.relu(h)
            else:
                h = m(h)
        return zs

    # f64 forward + gradients of the pre-activations
    h = x.to(DEV)
    zs64 = []
    for m in a64.network:
        if isinstance(m, torch.nn.Linear):
            h = m(h)
            h.retain_grad()
            zs64.append(h)
        else:
            h = m(h)
    logits, value = a64.actor(h), a64.critic(h)
    dist = torch.distributions.Categorical(logits=logits)
    act = torch.from_numpy(z["actions"]).to(DEV)[mb.to(DEV)]
    loss = -(dist.log_prob(act)).mean() + 0.5 * (value.view(-1) ** 2).mean()
    loss.backward()
    for route in ("cpu_f32", "hipblaslt", "x6"):
        zs = chain(route)
        rec = {"route": route, "layers": []}
        for l, (zr, z64) in enumerate(zip(zs, zs64)):
            z64c = z64.detach().reshape(zr.shape).cpu()
            g = z64.grad.reshape(zr.shape).cpu()
            flip = (zr > 0) != (z64c > 0)
            colmax = float(g.abs().sum(0).max())
            rec["layers"].append({"n": int(flip.sum()), "g_flipped": float(g[flip].abs().sum()) / colmax,
                                  "zerr_max": float((zr - z64c).abs().max() / z64c.abs().max())})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
    flips()
