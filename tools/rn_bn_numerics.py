"""CPU emulation of the train-mode BatchNorm numerics of the ResNet-50 training path, to find which
rounding step puts the HIP fp32 gradients 3-4x further from fp64 than torch fp32.

The oracle ResNet-50 (oracle/resnet_cpu.py) runs with every BatchNorm2d replaced by an
autograd.Function that reproduces one arithmetic form in fp32:

  torch   F.batch_norm (reference)
  hip     the round-3 kernels: forward statistics from fp32 per-64-row (sum y, sum y^2) partials,
          var = E[y^2] - m^2 in fp64, out = y*scale + shift (scale = g*is, shift = b - m*scale, fp32);
          backward sums fp32 per chunk, dy = k1*g + k2*y + k3 (k3 = -g*is*s/n - k2*m)
  cen     centred forms: statistics from per-chunk (sum, M2 about the chunk mean) merged in fp64
          (Chan), out = (y - m)*scale + b, dy = k1*g + k2*(y - m) + k3'   (k3' = -g*is*s/n)
  fwd     only the forward centred (backward as hip)
  bwd     only the backward centred (forward as hip)
  st / ap only the centred statistics / only the centred apply
  ex      exact fp64 statistics, centred apply and backward
  impl    round 4's kernels: one-pass statistics (conv epilogue), centred apply and backward
  c64     every conv in fp64 rounded to fp32 (the floor set by the BatchNorm arithmetic alone)

usage: python tools/rn_bn_numerics.py [frames] [hw] | state.pt   (env MODES=impl,ex,...  WATCH=param name)
"""
import re
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.resnet_cpu import ResNet50TrunkCPU, resnet_features  # noqa: E402

CH = 64  # rows per partial (the conv epilogue's tile)


def chunk_stats(y2d, centred):
    """y2d (M, C) fp32 -> mean, var (fp64) from fp32 per-chunk partials merged in fp64."""
    M, C = y2d.shape
    n = (M + CH - 1) // CH
    pad = n * CH - M
    yp = torch.cat([y2d, y2d.new_zeros(pad, C)]) if pad else y2d
    yc = yp.view(n, CH, C)
    cnt = torch.full((n, 1), float(CH), dtype=torch.float64)
    if pad:
        cnt[-1] = CH - pad
    s = yc.sum(1)  # fp32
    if not centred:
        q = (yc * yc).sum(1)
        S, Q = s.double().sum(0), q.double().sum(0)
        m = S / M
        return m, (Q / M - m * m).clamp_min(0)
    mt = s / cnt.float()
    d = yc - mt.unsqueeze(1)
    if pad:
        d[-1, CH - pad:] = 0
    m2 = (d * d).sum(1)
    mean = s.double().sum(0) / M
    var = (m2.double().sum(0) + (cnt * (mt.double() - mean) ** 2).sum(0)) / M
    return mean, var


class BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, w, b, mode):
        N, C, H, W = y.shape
        y2 = y.permute(0, 2, 3, 1).reshape(-1, C)
        cf = mode in ("cen", "fwd", "ap", "ex", "impl")
        if mode == "ex":
            m64, v64 = y2.double().mean(0), y2.double().var(0, unbiased=False)
        else:
            m64, v64 = chunk_stats(y2, mode in ("cen", "fwd", "st"))
        mu = m64.float()
        is_ = (1.0 / torch.sqrt(v64 + 1e-5)).float()
        sc = w * is_
        if cf:
            out = (y2 - mu) * sc + b
        else:
            sh = b - mu * sc
            out = torch.addcmul(sh, y2, sc)  # y*sc + sh
        ctx.save_for_backward(y2, w, mu, is_)
        ctx.mode, ctx.shape = mode, (N, C, H, W)
        return out.view(N, H, W, C).permute(0, 3, 1, 2).contiguous()

    @staticmethod
    def backward(ctx, go):
        y2, w, mu, is_ = ctx.saved_tensors
        N, C, H, W = ctx.shape
        g = go.permute(0, 2, 3, 1).reshape(-1, C).float()
        M = g.shape[0]
        xh = (y2 - mu) * is_
        n = (M + CH - 1) // CH
        pad = n * CH - M
        gp = torch.cat([g, g.new_zeros(pad, C)]) if pad else g
        xp = torch.cat([xh, xh.new_zeros(pad, C)]) if pad else xh
        s = gp.view(n, CH, C).sum(1).double().sum(0)
        q = (gp * xp).view(n, CH, C).sum(1).double().sum(0)
        gm, isd = w.double(), is_.double()
        k1 = (gm * isd).float()
        k2 = (-gm * isd * isd * q / M)
        if ctx.mode in ("cen", "bwd", "ex", "impl"):
            k3 = (-gm * isd * s / M).float()
            dy = k1 * g + k2.float() * (y2 - mu) + k3
        else:
            k3 = (-gm * isd * s / M + gm * isd * isd * mu.double() * q / M).float()
            dy = k1 * g + k2.float() * y2 + k3
        return dy.view(N, H, W, C).permute(0, 3, 1, 2), q.float(), s.float(), None


class BNMod(nn.Module):
    def __init__(self, bn, mode):
        super().__init__()
        self.bn, self.mode = bn, mode

    def forward(self, x):
        if self.mode == "torch":
            return self.bn(x)
        return BNFn.apply(x, self.bn.weight, self.bn.bias, self.mode)


class Conv64(nn.Module):
    """a conv computed in fp64 and rounded to fp32 (forward and, through autograd, backward)"""

    def __init__(self, conv):
        super().__init__()
        self.conv = conv

    def forward(self, x):
        c = self.conv
        return F.conv2d(x.double(), c.weight.double(), None, c.stride, c.padding).float()


def swap_conv(m):
    for name, ch in m.named_children():
        if isinstance(ch, nn.Conv2d):
            setattr(m, name, Conv64(ch))
        else:
            swap_conv(ch)


def swap_bn(m, mode):
    for name, ch in m.named_children():
        if isinstance(ch, nn.BatchNorm2d):
            setattr(m, name, BNMod(ch, mode))
        else:
            swap_bn(ch, mode)


def head_loss(f, head, y, w, l0):
    a1, a2, f1, f2 = head
    B = y.shape[0]
    f = f.view(B, -1, f.shape[-1])
    hh = torch.relu(f @ a1.weight.T.to(f.dtype) + a1.bias.to(f.dtype))
    a = torch.sigmoid(hh @ a2.weight.T.to(f.dtype) + a2.bias.to(f.dtype)).squeeze(-1)
    a = torch.softmax(a, dim=1)
    gg = (f * a.unsqueeze(-1)).sum(1)
    z = torch.relu(gg @ f1.weight.T.to(f.dtype) + f1.bias.to(f.dtype)) @ f2.weight.T.to(f.dtype) + f2.bias.to(f.dtype)
    return F.cross_entropy((l0.to(f.dtype) + z) / 2, y, weight=w.to(f.dtype))


def rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


def main():
    if len(sys.argv) > 1 and sys.argv[1].endswith(".pt"):
        # the state of tests/test_resnet_train_gpu.py::test_ensemble_training_step (member + clips), saved by
        # constructing EnsembleDetector on the CPU with the test's seed
        st = torch.load(sys.argv[1], weights_only=True)
        full, x = st["sd"], st["x"]
        B = x.shape[0]
        x = x.reshape(-1, *x.shape[2:])
        sd = {k[len("backbone."):]: v for k, v in full.items() if k.startswith("backbone.")}
        head = (nn.Linear(2048, 64), nn.Linear(64, 1), nn.Linear(2048, 256), nn.Linear(256, 2))
        for mod, key in zip(head, ("temporal_attention.0", "temporal_attention.2", "fc1", "fc2")):
            mod.weight.data.copy_(full[key + ".weight"])
            mod.bias.data.copy_(full[key + ".bias"])
        y = torch.tensor([0, 1] * (B // 2) + [0] * (B % 2))
        l0 = torch.zeros(B, 2)
    else:
        frames = int(sys.argv[1]) if len(sys.argv) > 1 else 4
        hw = int(sys.argv[2]) if len(sys.argv) > 2 else 128
        torch.manual_seed(0)
        base = ResNet50TrunkCPU().train()
        for mod in base.modules():
            if isinstance(mod, nn.Conv2d):
                nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
        head = (nn.Linear(2048, 64), nn.Linear(64, 1), nn.Linear(2048, 256), nn.Linear(256, 2))
        nn.init.kaiming_normal_(head[2].weight, mode="fan_out", nonlinearity="relu")
        nn.init.normal_(head[3].weight, 0, 0.01)
        x = torch.randn(frames, 3, hw, hw)
        B = frames // 2
        y = torch.tensor([0, 1] * (B // 2) + [0] * (B % 2))
        l0 = torch.randn(B, 2) * 0.1
        sd = base.state_dict()
    w = torch.tensor([0.7, 1.3])
    grads = {}
    import os
    modes = os.environ.get("MODES", "hip,fwd,bwd,cen,st,ap,ex,impl,c64,c64ap").split(",")
    watch = os.environ.get("WATCH", "")  # a parameter name to report per mode
    for mode in ["f64", "torch"] + modes:
        t = ResNet50TrunkCPU().train()
        t.load_state_dict(sd)
        dt = torch.float64 if mode == "f64" else torch.float32
        t = t.to(dt)
        if mode == "c64":
            swap_conv(t)
        elif mode == "c64ap":
            swap_conv(t)
            swap_bn(t, "ap")
        elif mode not in ("f64", "torch"):
            swap_bn(t, mode)
        f = resnet_features(t, x.to(dt))
        loss = head_loss(f, head, y, w, l0)
        loss.backward()
        grads[mode] = ({re.sub(r"\.(conv|bn)\.(weight|bias)$", r".\2", n): p.grad.detach().clone() for n, p in t.named_parameters()}, f.detach())
    g64, f64 = grads["f64"]
    for mode in ["torch"] + modes:
        g, f = grads[mode]
        if watch:
            print(f"{mode:6s} {watch}: rel err {rel(g[watch], g64[watch]):.3e}")
        errs = sorted(((rel(g[n], g64[n]), n) for n in g64), reverse=True)
        l4 = [e for e, n in errs if n.startswith("7.2")]
        print(f"{mode:6s} feat {rel(f, f64):.2e}  worst {errs[0][0]:.4f} ({errs[0][1]})  median "
              f"{errs[len(errs) // 2][0]:.4f}  7.2.* max {max(l4):.4f}")
        if mode == "torch":
            e32 = {n: rel(g[n], g64[n]) for n in g64}
        else:
            ratio = sorted(((rel(g[n], g64[n]) / max(e32[n], 1e-30), n) for n in g64 if rel(g[n], g64[n]) > 1e-4),
                           reverse=True)
            print(f"        worst ratio to torch-cpu fp32: {ratio[0][0]:.2f} ({ratio[0][1]}), "
                  f"over 3x: {sum(r > 3 for r, _ in ratio)}")


if __name__ == "__main__":
    main()
