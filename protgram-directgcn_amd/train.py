"""The reference trainer's step with the model-independent work fused.

``protgram_directgcn_trainer.py:91-100`` (full batch) and ``:129-140`` (per cluster) run, every step:
zero_grad -> autocast forward -> ``F.nll_loss`` (x the cluster weight) + ``l2_lambda * sum(p.norm(2).pow(2))``
over ALL parameters -> GradScaler backward -> step -> update, and ``loss.item()``. ``train_step`` computes the
same loss and gradients with:

* the L2 value from ONE multi-tensor launch (``pg_multi_sqsum_f32``) and its gradient ``2 * l2_lambda * p``
  added to every ``p.grad`` after backward by ONE launch (``pg_multi_axpy_f32``; under a GradScaler scaled by
  its device-side scale, no host sync) -- instead of ~110 per-parameter norm / pow / add launches forward and
  backward;
* the nll term as a gather + mean (``-logp[i, y_i]`` averaged; torch's nll_loss kernels are single-block);
* no host sync: the loss comes back as a device scalar (call ``.item()`` when you need it, as the reference
  does once per step).

Gradients equal the reference step's up to float summation order (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

from ._lib import check, load_library


class TensorList:
    """Device descriptors ({x, y, numel}) + chunk offsets for a fixed list of fp32 tensors."""

    def __init__(self, xs: List[torch.Tensor], ys: Optional[List[torch.Tensor]] = None):
        lib = load_library()
        if not xs:
            raise ValueError("empty tensor list")
        dev = xs[0].device
        for t in xs + (ys or []):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
                raise ValueError("tensors must be contiguous fp32 on one device")
        self.xs, self.ys = xs, ys
        desc = np.zeros((len(xs), 3), dtype=np.int64)
        chunks = np.zeros(len(xs) + 1, dtype=np.int64)
        for i, x in enumerate(xs):
            desc[i, 0] = x.data_ptr()
            desc[i, 1] = ys[i].data_ptr() if ys is not None else 0
            desc[i, 2] = x.numel()
            chunks[i + 1] = chunks[i] + lib.pg_multi_chunks(x.numel())
        self.key = tuple(int(v) for v in desc[:, :2].reshape(-1))
        self.desc = torch.from_numpy(desc).to(dev)
        self.chunk_ptr = torch.from_numpy(chunks).to(dev)
        self.nchunks = int(chunks[-1])
        self.partial = torch.empty(max(self.nchunks, 1), dtype=torch.float32, device=dev)


_LISTS: dict = {}


def _tensor_list(xs, ys=None) -> TensorList:
    key = tuple(t.data_ptr() for t in xs) + (tuple(t.data_ptr() for t in ys) if ys is not None else ())
    tl = _LISTS.get(key)
    if tl is None:
        if len(_LISTS) > 64:
            _LISTS.clear()
        tl = TensorList(xs, ys)
        _LISTS[key] = tl
    return tl


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def l2_sqsum(params: Iterable[torch.Tensor]) -> torch.Tensor:
    """sum_p ||p||_2^2 over the tensors (no autograd), one launch: the value of the trainer's L2 term."""
    xs = [p.detach() for p in params]
    tl = _tensor_list(xs)
    out = torch.empty((), dtype=torch.float32, device=xs[0].device)
    check(load_library().pg_multi_sqsum_f32(len(xs), ctypes.c_void_p(tl.desc.data_ptr()),
                                            ctypes.c_void_p(tl.chunk_ptr.data_ptr()), tl.nchunks,
                                            ctypes.c_void_p(tl.partial.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                            _stream(out.device)), "pg_multi_sqsum_f32")
    return out


def add_l2_grad(params: List[torch.Tensor], l2_lambda: float, scale: Optional[torch.Tensor] = None):
    """p.grad += 2 * l2_lambda * (scale) * p for every parameter (missing grads become zeros first): the
    gradient of l2_lambda * sum_p ||p||^2, one launch."""
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    xs = [p.detach() for p in params]
    ys = [p.grad for p in params]
    tl = _tensor_list(xs, ys)
    sp = ctypes.c_void_p(scale.data_ptr()) if scale is not None else None
    check(load_library().pg_multi_axpy_f32(len(xs), ctypes.c_void_p(tl.desc.data_ptr()),
                                           ctypes.c_void_p(tl.chunk_ptr.data_ptr()), tl.nchunks,
                                           float(2.0 * l2_lambda), sp, _stream(xs[0].device)), "pg_multi_axpy_f32")


def nll_mean(logp: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """F.nll_loss(logp, y) (mean reduction, no class weights) as gather + mean."""
    return -logp.gather(1, y.view(-1, 1)).mean()


def train_step(model, data, y: torch.Tensor, optimizer, l2_lambda: float = 0.0, scaler=None, weight: float = 1.0,
               autocast: bool = True) -> torch.Tensor:
    """One step of the reference loop (trainer :91-100, or :129-140 with weight = batch nodes / total nodes).
    Returns the total loss (nll * weight + l2_lambda * sum ||p||^2) as a device scalar."""
    params = [p for p in model.parameters() if p.requires_grad]
    optimizer.zero_grad(set_to_none=False)
    use_amp = autocast and scaler is not None and scaler.is_enabled()
    with torch.amp.autocast("cuda", enabled=use_amp):
        lp, _ = model(data=data)
        loss = nll_mean(lp.float(), y) * weight
    l2 = l2_sqsum(params) if l2_lambda else None
    scaled = scaler is not None and scaler.is_enabled()
    (scaler.scale(loss) if scaled else loss).backward()
    if l2_lambda:
        add_l2_grad(params, l2_lambda, scale=scaler._scale if scaled else None)  # device-side scale: no sync
    else:  # the reference's 0 * l2 term still gives every parameter a (zero) gradient, so it is stepped
        for p in params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
    if scaled:
        scaler.step(optimizer)
        scaler.update()
    else:
        optimizer.step()
    total = loss.detach()
    return total + l2_lambda * l2 if l2 is not None else total
