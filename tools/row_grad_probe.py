#!/usr/bin/env python3
"""Which part of the config-3 loss gives a wrong per-node gradient at one row? The model's gate gradients at
B(20,4), dims [128,128,128], split into the nll term and the L2 term, against the oracle (fp32 and float64)
at the rows where they disagree most.
usage: python tools/row_grad_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import torch.nn.functional as Fn  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from oracle import directgcn_cpu as oc  # noqa: E402
from test_gpu_configs import _csr_coo, _labels, _model  # noqa: E402

dev = torch.device("cuda:0")
n, dims, LAM = 4, [128, 128, 128], 1e-7
N, s, d, c = pkg.synth.de_bruijn_edges(n)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
m = _model(pkg, dims, N, n).to(dev).eval()
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1234))
y = _labels(N, n)


def gpu_grads(term):
    m.zero_grad(set_to_none=True)
    h, masks = x.to(dev), []
    for conv in m.convs:
        h = conv.fused_forward(h, g, None, res_x=h, act=True)
        masks.append((h > 0).detach().cpu())
    lp, _ = m.head(h)
    loss = Fn.nll_loss(lp, y.to(dev)) if term == "nll" else LAM * sum(p.norm(2).pow(2) for p in m.parameters())
    loss.backward()
    return {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}, masks


ei, w = _csr_coo(g)
if len(sys.argv) > 1 and sys.argv[1] == "sequence":
    # the config-3 test's exact sequence: x requires grad, nll + l2 in one backward, then a no-grad forward
    xd = x.to(dev).requires_grad_(True)
    h, masks = xd, []
    for conv in m.convs:
        h = conv.fused_forward(h, g, None, res_x=h, act=True)
        masks.append((h > 0).detach().cpu())
    lp, _ = m.head(h)
    (Fn.nll_loss(lp, y.to(dev)) + LAM * sum(p.norm(2).pow(2) for p in m.parameters())).backward()
    torch.cuda.synchronize()
    keys = ("convs.0.C_in_vec", "convs.1.C_all_vec", "convs.0.bias_main_in", "convs.0.bias_directed_shared_in")
    snap = {k: dict(m.named_parameters())[k].grad.detach().cpu().clone() for k in keys}
    with torch.no_grad():
        m(pkg.Data(x=xd, graph=g))
    torch.cuda.synchronize()
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    lp_r, _ = oc.model_forward(p, dims, x, ei, w[0], ei, w[1], ei, w[2], n_gram_len=n, prop=oc.propagate_chunked,
                               act_masks=masks)
    (Fn.nll_loss(lp_r, y) + LAM * sum(v.norm(2).pow(2) for v in p.values())).backward()
    prm = dict(m.named_parameters())
    for k in keys:
        after = prm[k].grad.detach().cpu()
        e0 = (snap[k].double() - p[k].grad.double()).abs()
        e1 = (after.double() - p[k].grad.double()).abs()
        print(f"{k}: before the no-grad forward max |d| {float(e0.max()):.3e} (row {int(e0.flatten().argmax())}), "
              f"after {float(e1.max()):.3e} (row {int(e1.flatten().argmax())}); changed by the forward: "
              f"{not torch.equal(snap[k], after)}; grad storage shared with another parameter: "
              f"{[o for o in prm if o != k and prm[o].grad is not None and prm[o].grad.untyped_storage().data_ptr() == prm[k].grad.untyped_storage().data_ptr()]}")
    sys.exit(0)

gn, masks = gpu_grads("nll")
gl, _ = gpu_grads("l2")
for term, gg in (("nll", gn), ("l2", gl)):
    for dt in (torch.float32, torch.float64):
        p = {k: v.detach().cpu().to(dt).clone().requires_grad_(True) for k, v in m.state_dict().items()}
        if term == "nll":
            lp_r, _ = oc.model_forward(p, dims, x.to(dt), ei, w[0], ei, w[1], ei, w[2], n_gram_len=n,
                                       prop=oc.propagate_chunked, act_masks=masks)
            Fn.nll_loss(lp_r, y).backward()
        else:
            (LAM * sum(v.norm(2).pow(2) for v in p.values())).backward()
        print(f"== {term} vs oracle {dt}")
        for k in ("convs.0.C_in_vec", "convs.0.constant", "convs.1.C_all_vec", "convs.1.constant"):
            err = (gg[k].double() - p[k].grad.double()).abs()
            flat = int(err.flatten().argmax())
            row = flat // gg[k].shape[1] if gg[k].dim() == 2 else flat
            print(f"  {k}: max |d| {float(err.max()):.3e} at row {row} (max |ref| {float(p[k].grad.abs().max()):.3e}); "
                  f"row 52642 |d| {float(err[52642].max()):.3e}")
