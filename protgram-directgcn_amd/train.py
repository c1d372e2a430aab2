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

from . import ops
from ._lib import check, load_library


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


_DEFERRED: list = []  # (device tensor, host array) uploads of a capture in progress, written after it ends
_ARENA: dict = {}     # device -> [int64 tensor, next free index]: where a capture's uploads live (prepare_capture)


def prepare_capture(dev, n: int = 1 << 16) -> torch.Tensor:
    """A fresh device arena (n int64) for the descriptor tables built inside the next HIP-graph capture on `dev`.
    Allocated here, outside the capture, so the graph's own memory pool never hands those bytes to a captured
    kernel (a table in pool memory would be clobbered at every replay by the kernels that reused its bytes during
    the capture). The graph's owner keeps the returned tensor as long as the graph."""
    t = torch.zeros(n, dtype=torch.int64, device=dev)
    _ARENA[torch.device(dev)] = [t, 0]
    return t


def _upload(a: np.ndarray, dev, keep: Optional[list] = None, nptr: Optional[int] = None) -> torch.Tensor:
    """Host array (int64) -> device without a host sync (pinned staging, stream-ordered copy). `keep` receives the
    pinned staging tensor: a copy captured into a HIP graph re-reads it at every replay, so its owner must keep it
    alive. Inside a HIP-graph capture (no pinned allocation is allowed there) the table takes a slice of the arena
    of prepare_capture(), and its contents -- static for every replay: addresses and chunk offsets -- are written by
    flush_deferred() after the capture ends."""
    if torch.cuda.is_current_stream_capturing():
        if a.dtype != np.int64:
            raise TypeError("capture-time uploads are int64 tables")
        slot = _ARENA.get(torch.device(dev))
        n = int(a.size)
        if slot is None or slot[1] + n > slot[0].numel():
            raise RuntimeError("no room for a descriptor table in this capture: call train.prepare_capture(dev) "
                               "before capturing")
        t = slot[0][slot[1]:slot[1] + n].view(a.shape)
        slot[1] += (n + 1) // 2 * 2  # 16-B aligned slices
        # nptr: the table's leading address columns (check_deferred); None: all but the last
        _DEFERRED.append((t, np.array(a, copy=True), a.shape[1] - 1 if nptr is None and a.ndim == 2 else nptr))
        return t
    h = torch.from_numpy(a).pin_memory()
    if keep is not None:
        keep.append(h)
    return h.to(dev, non_blocking=True)


class TensorList:
    """Device descriptors + chunk offsets for a list of fp32 tensor groups: field k of descriptor t is the data
    pointer of fields[k][t]; the last int64 is numel (of fields[0][t])."""

    def __init__(self, *fields: List[torch.Tensor], gtype: bool = False):
        """gtype: pg_adam_desc_t's trailing gradient-type column (field 1 may then hold bf16 tensors: 1)."""
        lib = load_library()
        xs = fields[0]
        if not xs:
            raise ValueError("empty tensor list")
        dev = xs[0].device
        for k, f in enumerate(fields):
            for t in f:
                ok = t.dtype == torch.float32 or (gtype and k == 1 and t.dtype == torch.bfloat16)
                if not ok or not t.is_contiguous() or t.device != dev:
                    raise ValueError("tensors must be contiguous fp32 on one device")
        desc = np.zeros((len(xs), len(fields) + 1 + int(gtype)), dtype=np.int64)
        chunks = np.zeros(len(xs) + 1, dtype=np.int64)
        for i, x in enumerate(xs):
            for k, f in enumerate(fields):
                desc[i, k] = f[i].data_ptr()
            desc[i, len(fields)] = x.numel()
            if gtype:
                if any(f[i].numel() != x.numel() for f in fields):
                    raise ValueError("tensor list fields differ in size")
                desc[i, -1] = 1 if fields[1][i].dtype == torch.bfloat16 else 0
            chunks[i + 1] = chunks[i] + lib.pg_multi_chunks(x.numel())
        self.fields = fields  # keep the tensors alive while the descriptors may be in use (dropped when cached)
        self.host = []  # the pinned staging copies (see _upload)
        self.desc = _upload(desc, dev, self.host, nptr=len(fields))
        self.chunk_ptr = _upload(chunks, dev, self.host)
        self.nchunks = int(chunks[-1])
        self.partial = torch.empty(max(self.nchunks, 1), dtype=torch.float32, device=dev)
        if torch.cuda.is_current_stream_capturing():
            _CAPTURED_LISTS.append(self)  # fields kept: a replay reads them by address


_CAPTURED_LISTS: list = []  # TensorLists built inside a capture: kept (with the tensors they point to) by its owner


def flush_deferred() -> list:
    """Write the uploads deferred during a capture (see _upload); call after the capture, before the first replay.
    Returns what the captured launches read by address -- the written tensors and the TensorLists built during the
    capture, with the tensors their descriptors point to: the owner of the graph keeps them as long as the graph."""
    keep = []
    for t, a, nptr in _DEFERRED:
        t.copy_(torch.from_numpy(a))
        keep.append((t, a, nptr))
    _DEFERRED.clear()
    keep += _CAPTURED_LISTS
    _CAPTURED_LISTS.clear()
    keep += [slot[0] for slot in _ARENA.values()]
    _ARENA.clear()
    return keep


def check_deferred(keep: list):
    """Debug check of flush_deferred's result before a first replay: every written table reads back as built, and
    every address in a descriptor table (its leading address columns) lies inside a live allocation of the caching
    allocator. Raises instead of letting a replay dereference a stale address."""
    live = []
    for seg in torch.cuda.memory_snapshot():
        addr = seg["address"]
        for b in seg["blocks"]:
            if b["state"] == "active_allocated":
                live.append((addr, addr + b["size"]))
            addr += b["size"]
    live.sort()
    import bisect
    starts = [a for a, _ in live]
    for item in keep:
        if not isinstance(item, tuple):
            continue
        t, a, nptr = item
        if not torch.equal(t.cpu(), torch.from_numpy(a)):
            raise RuntimeError("a deferred descriptor table does not read back as written")
        if a.ndim == 2 and nptr:
            for ptr in a[:, :nptr].reshape(-1).tolist():
                i = bisect.bisect_right(starts, ptr) - 1
                if i < 0 or not (live[i][0] <= ptr < live[i][1]):
                    raise RuntimeError(f"descriptor address {ptr:#x} is not inside a live allocation")


_LISTS: dict = {}


def _tensor_list(xs, ys=None) -> TensorList:
    """Parameter-only lists are cached (parameters keep their storage); lists with gradients are rebuilt per
    call -- caching them would keep every step's freed gradients alive."""
    if ys is not None:
        return TensorList(xs, ys)
    key = tuple(t.data_ptr() for t in xs)
    tl = _LISTS.get(key)
    if tl is None:
        if len(_LISTS) > 64:
            _LISTS.clear()
        tl = TensorList(xs, xs)  # pg_tensor_desc_t = {x, y, numel}: y unused by the sum of squares
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


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad = maximize = False; L2-style weight_decay) as ONE HIP launch per step for all
    parameters of a group (``pg_adam_f32``), instead of the foreach path's ~8 multi-tensor passes.

    GradScaler-aware without host syncs (``_step_supports_amp_scaling``): the scaler hands over its device
    scale and inf flag (``grad_scale`` / ``found_inf``); gradients are unscaled in-kernel and the whole update
    (including the step count) is skipped on inf, as torch's fused optimizers do. State per parameter has
    torch's keys (``step``, ``exp_avg``, ``exp_avg_sq``)."""

    _step_supports_amp_scaling = True

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        # device descriptor lists by the (address, numel) of every field: a step whose parameters, gradients and
        # moments sit where they sat before (persistent gradient buffers, or the caching allocator handing the same
        # blocks back) reuses the uploaded descriptors -- no host-side table and no host-to-device copy per step
        self._tl_cache: dict = {}
        # per parameter group: [device float64 {lr, weight_decay}, the host values last written into it]. The kernel
        # reads the learning rate from there at run time, so a HIP-graph replay of the step follows a schedule that
        # changes group["lr"] between replays (ReduceLROnPlateau, protgram_directgcn_trainer.py:84, :102)
        self._hyper: dict = {}

    def refresh_hyper(self):
        """Write every group's current ``lr`` / ``weight_decay`` into its device scalars (one fill launch per changed
        value, stream-ordered, no host sync). Eager steps call it themselves; the owner of a captured step calls it
        before every replay (GraphedTrainStep, shard.MiddleTrainer). betas and eps stay as captured."""
        if _capturing():
            raise RuntimeError("train.Adam.refresh_hyper inside a HIP-graph capture would bake the values into it")
        for gi, group in enumerate(self.param_groups):
            h = self._hyper.get(gi)
            if h is None:
                continue
            want = (float(group["lr"]), float(group["weight_decay"]))
            if want[0] < 0 or want[1] < 0:
                raise ValueError("invalid Adam hyper-parameters")
            for k in range(2):
                if h[1] is None or h[1][k] != want[k]:
                    h[0][k].fill_(want[k])
            h[1] = want

    def _hyper_ptr(self, gi: int, dev) -> ctypes.c_void_p:
        h = self._hyper.get(gi)
        if h is None or h[0].device != dev:
            if _capturing():
                raise RuntimeError("train.Adam: a parameter group's first step cannot be inside a HIP-graph capture")
            self._hyper[gi] = [torch.zeros(2, dtype=torch.float64, device=dev), None]
        if not _capturing():
            self.refresh_hyper()
        elif self._hyper[gi][1] != (float(self.param_groups[gi]["lr"]), float(self.param_groups[gi]["weight_decay"])):
            raise RuntimeError("train.Adam: lr / weight_decay changed without refresh_hyper() before this capture")
        return ctypes.c_void_p(self._hyper[gi][0].data_ptr())

    def _tensor_list(self, fields) -> TensorList:
        key = tuple((t.data_ptr(), t.numel(), t.dtype) for f in fields for t in f)
        tl = self._tl_cache.get(key)
        if tl is None:
            tl = TensorList(*fields, gtype=True)  # pg_adam_desc_t: field 1 (the gradient) may be bf16
            if not _capturing():  # a capture's lists keep their tensors (deferred bf16 gradients have no other owner)
                tl.fields = None  # the descriptors hold addresses only; the key guarantees they are current
            if len(self._tl_cache) >= 16:
                self._tl_cache.pop(next(iter(self._tl_cache)))
            self._tl_cache[key] = tl
        return tl

    def _cohorts(self, ps: List[torch.Tensor]) -> List[tuple]:
        """Group the parameters being stepped by their step counter (one pg_adam_f32 launch per counter).

        torch.optim.Adam counts steps per parameter: a parameter without a gradient is not stepped and its
        count stays behind. Here parameters that are always stepped together share ONE device scalar (so the
        usual case is one launch per group); a counter shared with a parameter that is not stepped this time
        is split off first (a device-side clone: no host sync). Counters that are not fp32 scalars on the
        parameter's device -- e.g. after ``load_state_dict`` from a checkpoint mapped to the CPU, which also
        un-shares them -- are rebuilt on the device, one shared scalar per distinct host value."""
        dev = ps[0].device
        rebuilt: dict = {}
        for p in ps:
            st = self.state[p]
            s = st["step"]
            if not (torch.is_tensor(s) and s.device == dev and s.dtype == torch.float32 and s.dim() == 0):
                if torch.is_tensor(s) and s.device.type != "cpu":
                    s = s.to(device=dev, dtype=torch.float32).reshape(())  # another device: stream-ordered copy
                    st["step"] = s
                else:
                    v = float(s)  # host value (CPU tensor or number): no device sync
                    if v not in rebuilt:
                        rebuilt[v] = torch.full((), v, dtype=torch.float32, device=dev)
                    st["step"] = rebuilt[v]
        users: dict = {}  # counter -> number of parameters (in any group) that share it
        for st in self.state.values():
            s = st.get("step")
            if torch.is_tensor(s):
                users[id(s)] = users.get(id(s), 0) + 1
        groups: dict = {}
        for p in ps:
            groups.setdefault(id(self.state[p]["step"]), []).append(p)
        out = []
        for members in groups.values():
            s = self.state[members[0]]["step"]
            if users[id(s)] > len(members):  # shared with parameters that are not stepped now: split
                s = s.clone()
                for p in members:
                    self.state[p]["step"] = s
            out.append((members, s))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        grad_scale = getattr(self, "grad_scale", None)
        found_inf = getattr(self, "found_inf", None)
        lib = load_library()
        # train_step's fused L2 value: per-chunk sums of p^2 (pre-update) from every launch, added at the end
        # (_want_sqsum == "groups": one value per parameter group, in _last_sqsum_groups)
        want_sq = getattr(self, "_want_sqsum", False)
        sq_parts = []
        group_parts: List[list] = []
        for gi, group in enumerate(self.param_groups):
            group_parts.append([])
            ps = [p for p in group["params"] if p.grad is not None or ops.deferred_grad(p) is not None]
            if not ps:
                continue
            fresh = None
            for p in ps:
                if (p.grad is not None and p.grad.is_sparse) or p.dtype != torch.float32:
                    raise RuntimeError("train.Adam takes dense fp32 parameters")
                if p.grad is not None and ops.deferred_grad(p) is not None:
                    raise RuntimeError("train.Adam: a parameter has both .grad and a deferred bf16 gradient")
                if p.device != ps[0].device:
                    raise RuntimeError("train.Adam: the parameters of a group must share one device")
                st = self.state[p]
                if not st:
                    if fresh is None:  # new parameters of this step share one counter
                        fresh = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["step"] = fresh
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            b1, b2 = group["betas"]
            dev = ps[0].device
            gs = grad_scale.to(dev) if grad_scale is not None else None
            fi = found_inf.to(dev, dtype=torch.float32) if found_inf is not None else None
            hyper = self._hyper_ptr(gi, dev)
            for members, step in self._cohorts(ps):
                grads = [p.grad.contiguous() if p.grad is not None else ops.deferred_grad(p) for p in members]
                tl = self._tensor_list((members, grads, [self.state[p]["exp_avg"] for p in members],
                                        [self.state[p]["exp_avg_sq"] for p in members]))
                if want_sq:
                    sq_parts.append(tl.partial[:tl.nchunks])
                    group_parts[-1].append(tl.partial[:tl.nchunks])
                check(lib.pg_adam_f32(len(members), ctypes.c_void_p(tl.desc.data_ptr()),
                                      ctypes.c_void_p(tl.chunk_ptr.data_ptr()), tl.nchunks, float(group["lr"]),
                                      float(b1), float(b2), float(group["eps"]),
                                      float(getattr(self, "_l2_extra", 0.0)),  # added to hyper[1] in-kernel
                                      ctypes.c_void_p(step.data_ptr()),
                                      ctypes.c_void_p(gs.data_ptr()) if gs is not None else None,
                                      ctypes.c_void_p(fi.data_ptr()) if fi is not None else None,
                                      ctypes.c_void_p(tl.partial.data_ptr()) if want_sq else None, hyper,
                                      _stream(dev)),
                      "pg_adam_f32")
            for p in ps:  # written in place by the kernel: let autograd / version-keyed caches see it
                torch.autograd.graph.increment_version(p)
        def fixed_order_sum(chunks):
            parts = torch.cat(chunks) if len(chunks) > 1 else chunks[0]
            out = torch.empty((), dtype=torch.float32, device=parts.device)
            check(lib.pg_multi_sum_f32(parts.numel(), ctypes.c_void_p(parts.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                       _stream(parts.device)), "pg_multi_sum_f32")
            return out

        if want_sq == "groups":
            self._last_sqsum_groups = [fixed_order_sum(gp) if gp else None for gp in group_parts]
        elif want_sq and sq_parts:
            self._last_sqsum = fixed_order_sum(sq_parts)
        return loss


# train_step runs the prediction head through ops.head_train (one kernel for its forward and backward) when the model
# offers it (ProtGramDirectGCN.head_train_args) and the kernel takes the shape; False: the framework ops
HEAD_FUSED = True


# bf16 mode with train.Adam and no GradScaler: the per-node constants' gradients stay the layers' bf16 dpre, read by
# Adam directly (ops.deferred_grad; the parameters' .grad stay None in this step); False: fp32 .grad as usual
DEFER_CONST_GRAD = True


def train_step(model, data, y: torch.Tensor, optimizer, l2_lambda: float = 0.0, scaler=None, weight: float = 1.0,
               autocast: bool = True) -> torch.Tensor:
    """One step of the reference loop (trainer :91-100, or :129-140 with weight = batch nodes / total nodes).
    Returns the total loss (nll * weight + l2_lambda * sum ||p||^2) as a device scalar."""
    defer = DEFER_CONST_GRAD and isinstance(optimizer, Adam) and not (scaler is not None and scaler.is_enabled())
    prev = ops._DEFER_CONST_GRAD
    ops._DEFER_CONST_GRAD = defer
    try:
        return _train_step(model, data, y, optimizer, l2_lambda, scaler, weight, autocast)
    finally:
        ops._DEFER_CONST_GRAD = prev
        ops._DEFERRED_GRADS.clear()


def _train_step(model, data, y, optimizer, l2_lambda, scaler, weight, autocast):
    params = [p for p in model.parameters() if p.requires_grad]
    optimizer.zero_grad(set_to_none=True)  # autograd then assigns gradients instead of adding into zeros
    use_amp = autocast and scaler is not None and scaler.is_enabled()
    scaled = scaler is not None and scaler.is_enabled()
    head = model.head_train_args() if HEAD_FUSED and hasattr(model, "head_train_args") else None
    if head is not None:
        # the prediction head's forward and backward in one kernel (ops.head_train): the layers' output h gets its
        # gradient (already scaled by the GradScaler's scale) from the kernel, the decoder parameters theirs
        with torch.amp.autocast("cuda", enabled=use_amp):
            h = model.body(data)
        W1, b1, W2, b2, p_drop = head
        seed = torch.randint(0, 2 ** 62, (1,), device=h.device, dtype=torch.int64) if p_drop > 0 else None
        scale = None
        if scaled:
            scaler.scale(torch.zeros((), device=h.device))  # the scale tensor exists from here on
            scale = scaler._scale
        # bf16 mode at F = 256 (config 5): the kernel reads the bf16 h and returns its bf16 gradient (no widened copy
        # either way); else the fp32 kernel on h.float() (F = 128)
        r = None
        if h.is_cuda and h.dtype == torch.bfloat16:
            r = ops.head_train_bf16(h, W1, b1, W2, b2, y, weight, p_drop, seed, scale)
            hf = h
        if r is None:
            hf = h.float()
            r = ops.head_train(hf, W1, b1, W2, b2, y, weight, p_drop, seed, scale) if hf.is_cuda else None
        if r is not None:
            loss, dh, grads = r
            for prm, gr in zip((W1, b1, W2, b2), grads):
                if prm.requires_grad:
                    prm.grad = gr
            torch.autograd.backward(hf, grad_tensors=dh)
            return _finish_step(model, params, optimizer, loss, l2_lambda, scaler, scaled, backward=False)
        lp, _ = model.head(hf, need_emb=False)
        loss = nll_mean(lp.float(), y) * weight
    else:
        with torch.amp.autocast("cuda", enabled=use_amp):
            lp, _ = model(data=data)
            loss = nll_mean(lp.float(), y) * weight
    return _finish_step(model, params, optimizer, loss, l2_lambda, scaler, scaled, backward=True)


def _finish_step(model, params, optimizer, loss, l2_lambda, scaler, scaled, backward: bool):
    """train_step after the forward: backward (unless done), the L2 term, the optimizer step; returns the loss."""
    # train.Adam takes the L2 gradient 2 * l2_lambda * p as extra weight decay inside its one launch (added to
    # the unscaled gradient before the moments, exactly where the gradient sum would put it), and -- when it steps
    # exactly these parameters -- the L2 value too, from the pre-update parameters it reads anyway; other
    # optimizers get the gradient added to p.grad by one pg_multi_axpy_f32 launch
    fold = bool(l2_lambda) and isinstance(optimizer, Adam)
    fused_sq = fold and ({id(p) for g in optimizer.param_groups for p in g["params"]} == {id(p) for p in params}
                         and len({p.device for p in params}) == 1)
    l2 = l2_sqsum(params) if l2_lambda and not fused_sq else None
    if backward:
        (scaler.scale(loss) if scaled else loss).backward()
    if l2_lambda and not fold:
        add_l2_grad(params, l2_lambda, scale=scaler._scale if scaled else None)  # device-side scale: no sync
    else:  # the reference's (0 *) l2 term gives every parameter a gradient, so it is stepped
        for p in params:
            if p.grad is None and ops.deferred_grad(p) is None:
                p.grad = torch.zeros_like(p)
    if fold:
        optimizer._l2_extra = 2.0 * l2_lambda
        optimizer._want_sqsum = fused_sq
        optimizer._last_sqsum = None
    try:
        if scaled:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
    finally:
        if fold:
            optimizer._l2_extra = 0.0
            optimizer._want_sqsum = False
    if fused_sq:
        l2 = optimizer._last_sqsum
        if l2 is None:  # the step did not run the kernel (e.g. GradScaler skipped it on the host): measure it
            l2 = l2_sqsum(params)
    total = loss.detach()
    return total + l2_lambda * l2 if l2 is not None else total


def hyper_snapshot(optimizer) -> tuple:
    """The host-side hyper-parameters a captured optimizer launch bakes in (every group's scalar settings)."""
    return tuple(tuple(sorted((k, v) for k, v in g.items() if k != "params" and isinstance(v, (int, float, tuple))))
                 for g in optimizer.param_groups)


def replay_ready(optimizer, snapshot: tuple) -> bool:
    """Before replaying a captured step: True when the graph still applies the optimizer's current settings.
    train.Adam reads lr / weight_decay from device scalars, which this refreshes (outside the graph); any other
    optimizer's captured launches carry the capture-time values, so a changed lr (or other setting) means the
    step must be captured again (False)."""
    if isinstance(optimizer, Adam):
        optimizer.refresh_hyper()
        snap = hyper_snapshot(optimizer)
        strip = lambda sn: tuple(tuple(kv for kv in g if kv[0] not in ("lr", "weight_decay")) for g in sn)
        return strip(snap) == strip(snapshot)
    return hyper_snapshot(optimizer) == snapshot


class GraphedTrainStep:
    """train_step(model, data, y, optimizer, l2_lambda, scaler) replayed from a HIP graph: `WARM` eager steps (the
    caches the step builds on first use: the COO -> CSR conversion and tile plans, Adam's state and descriptor lists,
    the allocator's pools), then the whole step -- forward, loss, backward, the L2 term and the optimizer launch -- is
    captured once (torch.cuda.CUDAGraph) and every later call is one graph launch. At config 3 the eager step leaves
    the GPU idle between the backward's launches (host-side autograd work); the replay does not. Dropout draws fresh
    masks per replay (the capture registers the default generator's Philox offset). The inputs are static: `data.x`
    and `y` are read where they were at capture (copy new values into them). Returns the loss as the graph's static
    device scalar, overwritten by the next call.

    Learning-rate schedules: with train.Adam the replay reads lr / weight_decay from the optimizer's device scalars,
    refreshed before every replay, so ReduceLROnPlateau (fit(), trainer :84, :102) acts on the next step exactly as
    in eager steps; any other optimizer is captured again when one of its settings changes.

    Safety: before the first replay every descriptor table written after the capture is read back and every address
    it holds is checked against the allocator's live blocks (check_deferred; CHECK = False skips it). A step that
    cannot be captured raises (RuntimeError); with eager_fallback=True it runs eagerly instead and the reason is
    kept in `failed`."""
    WARM = 3
    CHECK = True  # check_deferred before the first replay of every capture

    def __init__(self, model, data, y: torch.Tensor, optimizer, l2_lambda: float = 0.0, scaler=None,
                 weight: float = 1.0, eager_fallback: bool = False):
        self.args = (model, data, y, optimizer)
        self.kw = dict(l2_lambda=l2_lambda, scaler=scaler, weight=weight)
        self._graph, self._loss, self._keep, self._eager = None, None, None, 0
        self._snap = None
        self.eager_fallback = bool(eager_fallback)
        self.failed = None
        self.captures = 0

    def __call__(self) -> torch.Tensor:
        if self._graph is not None:
            if replay_ready(self.args[3], self._snap):
                model, data = self.args[0], self.args[1]
                x = getattr(data, "x", None)
                if getattr(model, "_xb", None) is not None and x is not None:
                    model.bf16_input(x)  # the bf16 mode's cached input, refreshed outside the graph if x changed
                self._graph.replay()
                return self._loss
            self.close(keep_warm=True)  # a setting the graph baked in changed: capture this step again
            return self._capture()
        if self.failed is not None or self._eager < self.WARM:
            self._eager += 1
            return train_step(*self.args, **self.kw)
        return self._capture()

    def _capture(self) -> torch.Tensor:
        import sys
        opt = self.args[3]
        if isinstance(opt, Adam):
            opt.refresh_hyper()
        prepare_capture(self.args[2].device)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                loss = train_step(*self.args, **self.kw)
        except Exception as e:  # noqa: BLE001 -- re-raised unless the caller asked for the eager fallback
            _DEFERRED.clear()
            _CAPTURED_LISTS.clear()
            _ARENA.clear()
            self.failed = repr(e)[:300]
            if not self.eager_fallback:
                raise RuntimeError(f"GraphedTrainStep: HIP graph capture failed: {self.failed}") from e
            print(f"[GraphedTrainStep] HIP graph capture failed ({self.failed}); running eager steps", file=sys.stderr)
            torch.cuda.synchronize()
            return train_step(*self.args, **self.kw)
        # the descriptor lists the captured launches read by address (and their pinned staging copies, which the
        # captured uploads re-read) live as long as the graph
        self._keep = list(getattr(opt, "_tl_cache", {}).values()) + list(_LISTS.values()) + flush_deferred()
        if self.CHECK:
            check_deferred(self._keep)
        self._graph, self._loss, self._snap = g, loss, hyper_snapshot(opt)
        self.captures += 1
        g.replay()  # the step the capture recorded
        return loss

    def close(self, keep_warm: bool = False):
        """Drop the graph (later calls capture again, after WARM eager steps unless keep_warm)."""
        torch.cuda.synchronize()
        self._graph, self._loss, self._keep = None, None, None
        if not keep_warm:
            self._eager = 0


class EarlyStopper:
    """The reference trainer's early stopper (protgram_directgcn_trainer.py:48-65): stop once the loss has not
    improved on the best by more than min_delta for `patience` consecutive checks."""

    def __init__(self, patience: int = 1, min_delta: float = 0):
        self.patience = patience
        self.min_delta = min_delta
        self.counter = 0
        self.best_loss = float("inf")

    def early_stop(self, validation_loss: float) -> bool:
        if validation_loss < self.best_loss - self.min_delta:
            self.best_loss = validation_loss
            self.counter = 0
            return False
        self.counter += 1
        return self.counter >= self.patience


def fit(step, optimizer, epochs: int, *, use_lr_scheduler: bool = True, lr_patience: int = 10,
        lr_factor: float = 0.5, use_early_stopping: bool = True, es_patience: int = 25, es_min_delta: float = 1e-5,
        scheduler=None, on_epoch=None) -> List[dict]:
    """The reference's full-batch epoch loop (protgram_directgcn_trainer.py:76-108) around any step callable that
    returns the step's total loss as a device scalar: ``train_step`` (eager), a ``GraphedTrainStep``, or a bound
    ``shard.MiddleTrainer.step`` / ``ShardedTrainer.step`` (all ranks see the same all-reduced loss, so they take
    the same scheduler and stopping decisions). Per epoch: step -> ``scheduler.step(loss)`` (ReduceLROnPlateau
    'min', the trainer's patience / factor, config.py:77-79) -> early stop on ``loss.item()`` (EarlyStopper, config.py
    :81-83). The defaults are the reference configuration's. `scheduler` replaces the default ReduceLROnPlateau (any
    object with step(metric)). Returns one record per epoch: loss (float) and the learning rates the step used."""
    if scheduler is None and use_lr_scheduler:
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min", patience=lr_patience,
                                                               factor=lr_factor)
    stopper = EarlyStopper(patience=es_patience, min_delta=es_min_delta) if use_early_stopping else None
    history = []
    for epoch in range(1, epochs + 1):
        lrs = [float(g["lr"]) for g in optimizer.param_groups]
        loss = step()
        value = float(loss)  # the reference's one host sync per epoch (scheduler.step(loss), loss.item())
        history.append(dict(epoch=epoch, loss=value, lr=lrs))
        if scheduler is not None:
            scheduler.step(value)
        if on_epoch is not None:
            on_epoch(history[-1])
        if stopper is not None and stopper.early_stop(value):
            history[-1]["stopped"] = True
            break
    return history
