"""Data-parallel training of the HIP matchers: the reference's ``train.py:307-309``
(``torch.nn.SyncBatchNorm.convert_sync_batchnorm`` + ``DistributedDataParallel``) for
``lightglue_amd.LightGlue`` and ``lightglue_amd.SuperGlue`` in training mode.

One process per GPU over ``torch.distributed`` (RCCL on MI355X; gloo works too, with device
tensors staged through the host).  Wrapping a model::

    model = LightGlue(conf).cuda().train()
    ddp = DataParallel(model)            # every rank, after init_process_group
    loss = torch.mean(model.loss(model(data), data)[0]["total"])
    loss.backward()                      # gradients arrive averaged over the ranks

What it does, and where it differs from torch's DDP:

* **Gradient averaging with overlap.**  The trunks' backward is one library call
  (``lg_train_backward`` / ``sg_train_backward``), so torch's per-parameter autograd hooks would see
  every trunk gradient only at its very end.  Instead the library reports each layer as soon as
  its gradients are final (``lg_set_grad_ready_hook`` / ``sg_set_grad_ready_hook``) and the layer's
  slice of one flat gradient buffer goes into an asynchronous all-reduce right there, under the
  remaining layers' backward kernels; the backward function waits for the buckets and divides by
  the world size before handing the gradients to autograd.  Parameters outside those calls
  (LightGlue's assignment heads and token confidences, whose backward runs first) are
  all-reduced from ``post_accumulate_grad`` hooks and finished by a callback queued on the
  autograd engine, as DDP finishes its buckets.
* **SyncBatchNorm** (SuperGlue): the library's BatchNorm kernels call back into
  ``sg_set_collective`` for every statistic, so each image set is normalised with its global
  batch's mean and variance and the backward uses the global per-channel sums -- what
  ``SyncBatchNorm`` does (``torch/nn/modules/_functions.py``).  Running statistics take the
  global unbiased variance.
* The loss stays the per-rank mean (``train.py:436``); with equal per-rank batches the averaged
  gradient equals the single-process gradient of the concatenated batch (``tests/test_ddp.py``:
  the semantics on the float64 oracle over gloo; ``tools/ddp_check.py``: this module on the GPU,
  two ranks against one process, run by ``tests/test_gpu_ddp.py``).
* **A rank failure is fatal to the job**, as under torch's DDP.  A failing rank (a library call
  that errors mid-backward, a failed collective in a callback) issues fewer collectives than its
  peers, which would then block forever in their next all-reduce.  ``DataParallel.abort`` waits
  for the collectives this rank already issued, destroys the process group -- the peers' pending
  collectives then fail instead of hanging -- and re-raises; the wrapper is unusable afterwards.
"""
import ctypes
import re

import torch
import torch.distributed as dist

from . import _lib

_TRUNK_LAYER = re.compile(r"^(?:transformers|gnn\.layers)\.(\d+)\.")


def _layer_of(name, n_layers, sg):
    """The library's gradient-ready id of parameter ``name``: its layer, or the id of the call's
    remaining group (LightGlue: -1 = input_proj / posenc; SuperGlue: L = final_proj / bin_score
    (ready first), -1 = the keypoint encoder)."""
    m = _TRUNK_LAYER.match(name)
    if m:
        return int(m.group(1))
    if sg and (name.startswith("final_proj.") or name == "bin_score"):
        return n_layers
    return -1


class _Buckets:
    """One backward call's flat gradient buffer: per-layer contiguous slices, an async all-reduce
    per slice as the library reports it, then wait + average."""

    def __init__(self, ddp, names, params, wanted, n_layers, sg, device):
        self.ddp = ddp
        order = sorted(range(len(names)), key=lambda i: (-_layer_of(names[i], n_layers, sg), i))
        numel = [params[i].numel() if wanted[i] else 0 for i in range(len(names))]
        self.flat = torch.empty(max(sum(numel), 1), dtype=torch.float32, device=device)
        self.grads = [None] * len(names)
        self.ranges = {}
        o = 0
        for i in order:
            if not numel[i]:
                continue
            lid = _layer_of(names[i], n_layers, sg)
            a, _ = self.ranges.get(lid, (o, o))
            self.grads[i] = self.flat[o:o + numel[i]].view_as(params[i])
            o += numel[i]
            self.ranges[lid] = (a, o)
        self.works = []
        self.error = None
        self.cb = None

    def callback(self, ctype):
        def ready(_ctx, layer, _stream):
            try:
                r = self.ranges.get(int(layer))
                if r is not None and r[1] > r[0]:
                    self.works.append(dist.all_reduce(self.flat[r[0]:r[1]], group=self.ddp.group, async_op=True))
            except Exception as e:  # noqa: BLE001 -- re-raised after the library call returns
                self.error = e
        self.cb = ctype(ready)
        return self.cb

    def finish(self):
        if self.error is not None:
            self.ddp.abort(self.error)
        try:
            for w in self.works:
                w.wait()
        except Exception as e:  # noqa: BLE001 -- a peer failed or the group is gone
            self.ddp.abort(e)
        self.works = []
        self.ddp._active = None
        self.flat.div_(self.ddp.world)
        return self.grads


class DataParallel:
    """DistributedDataParallel + SyncBatchNorm for a lightglue_amd matcher (module docstring)."""

    def __init__(self, model, process_group=None, sync_batchnorm=True):
        if not dist.is_available() or not dist.is_initialized():
            raise RuntimeError("DataParallel needs torch.distributed.init_process_group first")
        self.model = model
        self.group = process_group
        self.world = dist.get_world_size(process_group)
        self.sync_batchnorm = bool(sync_batchnorm)
        self._pending = []
        self._queued = False
        self._coll_buf = None
        self._coll_cb = None
        self._coll_error = None
        self._active = None  # the _Buckets of the backward call in progress
        self.broken = None
        model._ddp = self
        # same initial parameters everywhere (DDP broadcasts rank 0's at construction)
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t, src=dist.get_global_rank(process_group, 0) if process_group else 0, group=process_group)
        # parameters whose gradients come from outside the trunk calls (LightGlue's heads)
        self._hooks = []
        for name, p in model.named_parameters():
            if self._outside_trunk(name) and p.requires_grad:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._param_ready))

    # ------------------------------------------------------------------ parameters outside the trunk calls
    def _outside_trunk(self, name):
        return name.startswith(("log_assignment.", "token_confidence."))

    def _param_ready(self, p):
        self._check_usable()
        try:
            self._pending.append((p, dist.all_reduce(p.grad, group=self.group, async_op=True)))
        except Exception as e:  # noqa: BLE001
            self.abort(e)
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish_pending)

    def _finish_pending(self):
        try:
            for _, w in self._pending:
                w.wait()
        except Exception as e:  # noqa: BLE001
            self.abort(e)
        for p, _ in self._pending:
            p.grad.div_(self.world)
        self._pending = []
        self._queued = False

    # ------------------------------------------------------------------ failure: fatal to the job
    def _check_usable(self):
        if self.broken is not None:
            raise RuntimeError("DataParallel: an earlier rank failure destroyed the process group") from self.broken

    def abort(self, exc):
        """Fail this rank without stranding its peers: wait for every collective this rank issued
        (the peers issued them too), destroy the process group so that the peers' next collective
        raises instead of waiting for this rank forever, then re-raise ``exc``."""
        if self.broken is None:
            self.broken = exc
            works = [w for _, w in self._pending]
            if self._active is not None:
                works += self._active.works
                self._active.works = []
            self._pending, self._active, self._queued = [], None, False
            for w in works:
                try:
                    w.wait()
                except Exception:  # noqa: BLE001,S110 -- the group may already be broken
                    pass
            try:
                if dist.is_initialized():
                    dist.destroy_process_group(self.group)
            except Exception:  # noqa: BLE001,S110
                pass
        raise exc

    # ------------------------------------------------------------------ trunk calls (library hooks)
    def buckets(self, names, params, wanted, n_layers, sg, device):
        self._check_usable()
        self._active = _Buckets(self, names, params, wanted, n_layers, sg, device)
        return self._active

    # ------------------------------------------------------------------ SyncBatchNorm (SuperGlue)
    def attach_collective(self, lib, handle, device):
        """Register the SyncBatchNorm collective on a SuperGlue handle (idempotent)."""
        self._check_usable()
        if not self.sync_batchnorm:
            _lib.check(lib.sg_set_collective(handle, None, None, None, 0), "sg_set_collective")
            return
        n = int(lib.sg_collective_floats())
        if self._coll_buf is None or self._coll_buf.device != device:
            self._coll_buf = torch.zeros(n, dtype=torch.float32, device=device)

            def coll(_ctx, count, _stream):
                try:
                    dist.all_reduce(self._coll_buf[:int(count)], group=self.group)
                    return 0
                except Exception as e:  # noqa: BLE001 -- re-raised by check_collective
                    self._coll_error = e
                    return 1
            self._coll_cb = _lib.SG_COLLECTIVE_FN(coll)
        _lib.check(lib.sg_set_collective(handle, _lib.fnptr(self._coll_cb), None, ctypes.c_void_p(self._coll_buf.data_ptr()),
                                         n),
                   "sg_set_collective")

    def check_collective(self):
        """After a library call that ran SyncBatchNorm collectives: a failed one is fatal (abort)."""
        if self._coll_error is not None:
            e, self._coll_error = self._coll_error, None
            self.abort(e)
