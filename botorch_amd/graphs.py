"""HIP-graph capture of an acquisition evaluation (hard
part 6: launch-bound inner loops).

A fused qEI / qLogEI forward (and, with ``with_grad``, its backward) issues a
fixed sequence of launches for a fixed X shape: prepare_rows, the K*x^T build,
the posterior kernel (+ its split reduction), the finalisation, and the
ladder-status reduction.  At small shapes (C2: 64 t-batches, n = 1024) the
host-side dispatch of that sequence costs as much as the kernels.
``GraphedAcquisition`` captures it once with ``torch.cuda.graph`` on the
caller's device and replays it: a call copies X into the captured input
buffer, replays the graph and returns the captured outputs.

The reference has no counterpart (it evaluates eagerly through gpytorch); the
values are the eager path's, bit for bit (tests/test_gpu_graphs.py).  The
jitter-ladder status never stalls a replay: the graph folds every replay's
[max info, max jitter] into a sticky device maximum and copies it to pinned
host memory as its last node; an event follows each replay.  With
``check_each_call`` a call acts on the status as soon as a finished replay has
published it (an event query, no wait: the host keeps issuing while the GPU
runs); ``check_status()`` waits for the last replay and acts (the device
optimiser's status reads).  NotPSDError / the jitter warning are raised as
[G] psd_safe_cholesky's are, a call or two late instead of one.

Constraints of capture: the model's caches, the Sobol base samples and the
split plans must exist before capture (two eager warm-up calls build them),
and the model must not change between replays (a changed model raises).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import kernels


class GraphedAcquisition:
    """Callable wrapper: ``GraphedAcquisition(acqf, X_example)(X)`` equals
    ``acqf(X)`` for X of X_example's shape; with ``with_grad`` it returns
    ``(acq, dacq_sum/dX)`` (the gradient ``gen_candidates_*`` needs)."""

    def __init__(self, acqf, X_example: torch.Tensor, with_grad: bool = False, warmup: int = 2,
                 check_each_call: bool = True, share_input: bool = False):
        """``share_input``: capture reading X_example's own storage (no copy);
        a call with that same tensor then replays without copying X in (the
        device optimiser's trial points; the caller owns the buffer)."""
        if not X_example.is_cuda:
            raise RuntimeError("GraphedAcquisition captures ROCm device work")
        self.acqf = acqf
        self.with_grad = with_grad
        self.check_each_call = check_each_call
        self.dev = X_example.device
        self.X = X_example.detach() if share_input else X_example.detach().clone()
        self._model_key = self._key()
        side = torch.cuda.Stream(self.dev)
        side.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream(self.dev).wait_stream(side)
        kernels.check_ladder_status(self.dev)
        self.graph = torch.cuda.CUDAGraph()
        self._sticky = torch.zeros(2, dtype=torch.float64, device=self.dev)
        self._what = None
        from . import _lib
        # forward-only: the fused forward's finalisation folds the status into
        # these coherent pinned words itself (sticky max), so the graph holds
        # just the forward's own kernels; otherwise (gradients, generic routes)
        # a status reduction, a device max and a pinned copy are captured too
        self._host = _lib.torch_ops().pinned_status() if not with_grad else \
            torch.zeros(2, dtype=torch.float64).pin_memory()
        # a device-side status of another route beside the native one (a body
        # mixing both) lands in a pinned pair of its own (kernels.
        # record_capture_status), never over the native route's words
        self._host2 = torch.zeros(2, dtype=torch.float64).pin_memory()
        counter = torch.zeros(1, dtype=torch.int32, device=self.dev)
        with kernels.capturing(self.dev) as cap:
            if not with_grad:
                kernels._CAPTURE_STATUS[cap.idx] = (self._host, counter)
            try:
                self.out = _capture(self.graph, self.dev, self._captured_body, cap.idx)
            finally:
                kernels._CAPTURE_STATUS.pop(cap.idx, None)
        self._counter = counter
        taken = kernels.take_captured_status(self.dev)
        self._what = taken[1] if taken is not None else None
        kernels.drop_keepalive()  # captured: no launch still needs the argument refs
        self._event = torch.cuda.Event()
        self._pending = False

    def _captured_body(self, idx):
        out = self._body()
        st = kernels._CAPTURE.get(idx)
        if st is not None and st[0] != "native":
            # the replay's status: sticky max, then to the host
            mixed = st[0] == "native+"
            torch.maximum(self._sticky, st[2] if mixed else st[0], out=self._sticky)
            (self._host2 if mixed else self._host).copy_(self._sticky, non_blocking=True)
        return out

    def _key(self):
        m = getattr(self.acqf, "model", None)
        return m._key() if m is not None and hasattr(m, "_key") else None

    def _body(self):
        if self.with_grad:
            # a fresh leaf per call over the captured buffer's storage: a leaf
            # reused across the side-stream warm-up and the capture would keep
            # its first AccumulateGrad node (bound to the warm-up stream)
            Xg = self.X.detach().requires_grad_(True)
            v = self.acqf(Xg)
            (g,) = torch.autograd.grad(v.sum(), Xg)
            return v.detach(), g
        with torch.no_grad():
            return self.acqf(self.X)

    def _act(self) -> None:
        """The replays' status published to the host so far (sticky max):
        raise / warn, and re-arm the device maximum after a warning."""
        info_max = max(float(self._host[0]), float(self._host2[0]))
        jitter_max = max(float(self._host[1]), float(self._host2[1]))
        if info_max > 0 or jitter_max > 0:
            # re-armed before acting: a warning is given once per jittered
            # stretch, and a NotPSDError reports only the replays up to now
            # (psd_safe_cholesky raises for the failing evaluation alone; a
            # later replay that factors cleanly must not raise again)
            self._sticky.zero_()
            self._host.zero_()
            self._host2.zero_()
            kernels._ladder_outcome(info_max, jitter_max, self._what)

    def check_status(self) -> None:
        """Wait for the last replay, then raise NotPSDError / warn for the
        jitter ladders of the replays so far."""
        if self._pending and self._what is not None:
            self._event.synchronize()
            self._pending = False
            self._act()

    def _poll(self) -> None:
        """The same without waiting: acts only once the last replay finished."""
        if self._pending and self._what is not None and self._event.query():
            self._pending = False
            self._act()

    def __call__(self, X: torch.Tensor):
        if X.shape != self.X.shape:
            raise ValueError(f"captured for X of shape {tuple(self.X.shape)}, got {tuple(X.shape)}")
        if self._key() != self._model_key:
            raise RuntimeError("the model changed since capture; build a new GraphedAcquisition")
        if self.check_each_call:
            self._poll()  # a finished replay's ladder status, without stalling this call
        if X.data_ptr() != self.X.data_ptr():  # (a caller that writes the captured buffer itself)
            self.X.copy_(X.detach())
        self.graph.replay()
        self._event.record(torch.cuda.current_stream(self.dev))
        self._pending = True
        return self.out


_CAPTURE_STREAMS = {}


def _capture(graph, dev, body, idx):
    """``with torch.cuda.graph(graph): body(idx)`` without that context's
    entry ``empty_cache()``: it hands every cached block back to the driver, so
    the capture's own allocations and the eager calls after it pay hipMalloc
    again (C3 at b = 2: a capture 3.0 -> 1.7 ms, tools/capture_cost.py).  The
    same device synchronisation, side stream, private memory pool and
    "global" capture mode as torch.cuda.graph."""
    torch.cuda.synchronize(dev)
    key = kernels._dev_index(dev)
    if key not in _CAPTURE_STREAMS:
        _CAPTURE_STREAMS[key] = torch.cuda.Stream(dev)
    stream = _CAPTURE_STREAMS[key]
    stream.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(stream):
        graph.capture_begin(capture_error_mode="global")
        try:
            out = body(idx)
        finally:
            graph.capture_end()
    torch.cuda.current_stream(dev).wait_stream(stream)
    return out


def graphed(acqf, X_example: torch.Tensor, with_grad: bool = False) -> Optional[GraphedAcquisition]:
    """GraphedAcquisition(acqf, X_example, with_grad)."""
    return GraphedAcquisition(acqf, X_example, with_grad=with_grad)
