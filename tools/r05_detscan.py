#!/usr/bin/env python3
"""Round-5 determinism scan (cold caches): every hot-path kernel that mixes MFMA with packed-FP32 VALU math, run
repeatedly on fixed inputs with a 2 GiB cache flush before each call; reports the outputs that differ bitwise from
the first call. Motivated by the bf16 dense backward, whose lead-tile bias dots (v_pk_fma_f32 next to bf16 MFMAs)
varied in ~half of such runs and became reproducible when the translation unit was built with -fno-slp-vectorize.
  python tools/r05_detscan.py [reps=10]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402

from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
from protgram_directgcn_amd import ops  # noqa: E402
import test_gpu_parity as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
flush = torch.empty(1 << 29, device=dev)


def scan(name, fn):
    ref, bad = None, []
    for r in range(reps):
        flush.fill_(float(r))
        torch.cuda.synchronize()
        out = fn()
        out = out if isinstance(out, (tuple, list)) else [out]
        out = [o.detach().clone() for o in out if torch.is_tensor(o)]
        torch.cuda.synchronize()
        if ref is None:
            ref = out
            continue
        for i, (a, b) in enumerate(zip(ref, out)):
            if not torch.equal(a, b):
                bad.append((r, i, int((a != b).sum())))
    print(json.dumps({"op": name, "reps": reps, "differing": bad[:8], "n_bad_reps": len({b[0] for b in bad})}),
          flush=True)


Z, xres, prm, const, rr, W_res, b_res, dY = T._dense_case(20000, 128, 128, False, True, False, 3)
dv = {k: v.to(dev) for k, v in prm.items()}
Zg, dYg, xg, cg = Z.to(dev), dY.to(dev), xres.to(dev), const.to(dev) if const is not None else None
scan("dense_f32_fwd", lambda: ops.layer_dense(Zg, dv, 0, constant=cg, res_x=xg, act=True))
scan("dense_f32_fwd_pregated", lambda: ops.layer_dense(Zg, dv, 0, constant=cg, res_x=xg, act=True, pregated=True))
Y = ops.layer_dense(Zg, dv, 0, res_x=xg, act=True)
scan("dense_f32_bwd", lambda: list(v for v in ops.layer_dense_backward(dYg, Zg, Y, dv, 0, res_x=xg, act=True)
                                   .values() if v is not None))
Zb, xb, dYb = Zg.to(torch.bfloat16), xg.to(torch.bfloat16), dYg.to(torch.bfloat16)
packs = []
scan("dense_bf16_fwd", lambda: ops.layer_dense(Zb, dv, 0, constant=cg, res_x=xb, act=True, packs=packs))
Yb = ops.layer_dense(Zb, dv, 0, res_x=xb, act=True, packs=packs)
scan("dense_bf16_bwd", lambda: list(v for v in ops.layer_dense_backward(dYb, Zb, Yb, dv, 0, res_x=xb, act=True,
                                                                         packs=packs).values() if v is not None))
# head (decoder + log_softmax + L2), the middle-tile forward / transposed / scatter kernels at 4-gram
N, s, d, c = pkg.synth.de_bruijn_edges(4)
g = pkg.build_propagation_csr(N, s, d, c, device=dev)
x = torch.randn(N, 128, generator=torch.Generator().manual_seed(1)).to(dev)
W1, b1 = torch.randn(64, 128, device=dev) * 0.1, torch.randn(64, device=dev) * 0.1
W2, b2 = torch.randn(20, 64, device=dev) * 0.1, torch.randn(20, device=dev) * 0.1
scan("head_f32", lambda: ops.head(x, W1, b1, W2, b2, 1e-12))
scan("spmm3_mid_f32", lambda: ops.spmm3(g, x))
G = torch.randn(N, 384, generator=torch.Generator().manual_seed(2)).to(dev)
scan("spmm3t_f32", lambda: ops.spmm3_t(g, G))
scan("spmm3t_offdiag_f32", lambda: ops.spmm3t_offdiag(g, G))
sp = ops.ngram_scatter_plan(g, 0, 50)
Gm = torch.randn(50 * 400, 384, generator=torch.Generator().manual_seed(3)).to(dev)
scan("scatter_f32", lambda: ops.spmm3t_scatter(sp, Gm))
scan("scatter_bf16", lambda: ops.spmm3t_scatter(sp, Gm.to(torch.bfloat16)))
A_, B_ = torch.randn(160000, 64, device=dev), torch.randn(160000, 128, device=dev)
scan("gemm_at_b", lambda: ops.gemm_at_b(A_, B_))
