"""Batched prediction export: the loop that feeds the matcher during
``gluefactory.eval.hpatches`` / ``megadepth1500`` and stores its outputs per pair
(``gluefactory/utils/export_predictions.py:17-85``).

Differences from the reference, all deliberate:

* **Every pair of a batch is written.**  The reference keeps ``v[0]`` only (``:68``), so a batch
  size > 1 silently drops pairs; here batch element ``b`` goes to group ``data["name"][b]``.
* **Keypoint renormalisation per pair.**  The reference multiplies by ``scales[None]`` (``:47-53``),
  which broadcasts correctly only for batch size 1; here each pair uses its own ``scales[b]``.
* **Copies overlap compute.**  On a HIP device the next batch is copied host -> device on a side
  stream while the current one is matched, and the results of batch i are copied device -> host
  and written while batch i+1 runs (the reference serialises copy, forward, ``.cpu()``, write).
* **The storage is an interface.**  :class:`H5Writer` writes the reference's ``predictions.h5``
  layout (one group per pair, one dataset per key) through ``h5py``; ``h5py`` is not installed in
  the build image, so that writer is parity-unpinned here.  :class:`NpzWriter` (one ``.npz`` per
  pair) and :class:`MemoryWriter` (a dict) implement the same interface.
"""
from pathlib import Path

import warnings

import numpy as np
import torch


def map_tensor(x, func):
    """utils/tensor.py:13-24."""
    if isinstance(x, (str, bytes)) or x is None:
        return x
    if isinstance(x, dict):
        return {k: map_tensor(v, func) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [map_tensor(v, func) for v in x]
    return func(x)


def batch_to_device(batch, device, non_blocking=True):
    """utils/tensor.py:31-35."""
    return map_tensor(batch, lambda t: t.to(device=device, non_blocking=non_blocking) if torch.is_tensor(t) else t)


class MemoryWriter:
    def __init__(self):
        self.groups = {}

    def write(self, name, arrays):
        if name in self.groups:
            raise RuntimeError(f"group {name} exists")  # h5py raises on a duplicate group name
        self.groups[name] = dict(arrays)

    def close(self):
        pass


class NpzWriter:
    """One ``<root>/<name>.npz`` per pair (names may contain '/', like HPatches' 'seq/1_2')."""

    def __init__(self, root):
        self.root = Path(root)

    def write(self, name, arrays):
        path = self.root / f"{name}.npz"
        if path.exists():
            raise RuntimeError(f"group {name} exists")
        path.parent.mkdir(parents=True, exist_ok=True)
        np.savez(path, **arrays)

    def close(self):
        pass


class H5Writer:
    """The reference's h5 layout (export_predictions.py:26,73-79): group per pair, dataset per key.
    Parity-unpinned in this image (no h5py)."""

    def __init__(self, path):
        import h5py  # noqa: deliberately lazy: absent in the build image

        Path(path).parent.mkdir(exist_ok=True, parents=True)
        self.f = h5py.File(str(path), "w")

    def write(self, name, arrays):
        grp = self.f.create_group(name)  # RuntimeError/ValueError on duplicates, as the reference
        for k, v in arrays.items():
            grp.create_dataset(k, data=v)

    def close(self):
        self.f.close()


def _renormalize(pred, data):
    """export_predictions.py:45-65, per pair: keypoints / lines were predicted on the resized
    image; divide by the view's resize scales."""
    out = dict(pred)
    for k, v in pred.items():
        prefix = next((p for p in ("keypoints", "lines", "orig_lines") if k.startswith(p)), None)
        if prefix is None or not torch.is_tensor(v):
            continue
        idx = k[len(prefix):]
        scales = 1.0 / (data["scales"] if len(idx) == 0 else data[f"view{idx}"]["scales"])
        # [B,2] -> [B,1,..,2]: each pair its own scale (the reference's scales[None] is B == 1 only)
        out[k] = v * scales.reshape(scales.shape[0], *([1] * (v.dim() - scales.dim())), scales.shape[-1])
    return out


@torch.no_grad()
def export_predictions(loader, model, output_file=None, as_half=False, keys="*", callback_fn=None,
                       optional_keys=(), writer=None, device=None):
    """export_predictions.py:17-85 for any batch size.  ``writer`` defaults to
    :class:`H5Writer` (``output_file``).  Returns ``output_file`` (or the writer).

    Tensor-valued predictions are written per pair (``v[b]``).  Per-pair LISTS of tensors (length B,
    what the matcher returns for ``log_assignment`` / ``ref_descriptors*`` of a pruned B > 1 batch:
    each pair's kept block) are written per pair too (``v[b]``).  Any other value (scalars, nested
    dicts, lists of another length) has no per-pair form; such keys are skipped with one warning
    naming them (the reference exports tensors only, ``export_predictions.py:66-68``)."""
    assert keys == "*" or isinstance(keys, (tuple, list))
    if writer is None:
        writer = H5Writer(output_file)
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    model = model.to(device).eval()
    on_gpu = device.type == "cuda"
    copy_stream = torch.cuda.Stream(device) if on_gpu else None

    def upload(batch):
        if not on_gpu:
            return batch_to_device(batch, device)
        with torch.cuda.stream(copy_stream):
            return batch_to_device(batch, device, non_blocking=True)

    warned = set()

    def finish(item):  # host side of one batch: wait for its D2H copies, write every pair
        host, host_lists, names, event = item
        if event is not None:
            event.synchronize()
        host = {k: v.numpy() for k, v in host.items()}
        host_lists = {k: [x.numpy() for x in v] for k, v in host_lists.items()}
        for b, name in enumerate(names):
            arrays = {k: v[b] for k, v in host.items()}
            arrays.update({k: v[b] for k, v in host_lists.items()})
            if as_half:
                arrays = {k: (v.astype(np.float16) if v.dtype == np.float32 else v) for k, v in arrays.items()}
            try:
                writer.write(name, arrays)
            except (RuntimeError, ValueError):
                continue  # duplicate group: skipped, as the reference (:80-81)

    it = iter(loader)
    nxt = next(it, None)
    staged = upload(nxt) if nxt is not None else None
    pending = None
    while nxt is not None:
        data_host, data = nxt, staged
        if on_gpu:
            torch.cuda.current_stream(device).wait_stream(copy_stream)
            map_tensor(data, lambda t: t.record_stream(torch.cuda.current_stream(device)) if torch.is_tensor(t) else t)
        pred = model(data)
        nxt = next(it, None)
        staged = upload(nxt) if nxt is not None else None  # overlaps this batch's forward
        if callback_fn is not None:
            pred = {**callback_fn(pred, data), **pred}
        if keys != "*":
            missing = set(keys) - set(pred.keys())
            if missing:
                raise ValueError(f"Missing key {missing}")
            pred = {k: v for k, v in pred.items() if k in list(keys) + list(optional_keys)}
        assert len(pred) > 0
        names = list(data_host["name"])
        pred = _renormalize(pred, data)
        lists = {k: v for k, v in pred.items() if isinstance(v, (list, tuple)) and len(v) == len(names)
                 and all(torch.is_tensor(x) for x in v)}
        tensors = {k: v for k, v in pred.items() if torch.is_tensor(v)}
        skipped = sorted(set(pred) - set(tensors) - set(lists) - warned)
        if skipped:
            warnings.warn(f"export_predictions: keys without a per-pair tensor form are not written: {skipped}")
            warned.update(skipped)
        if on_gpu:
            host = {k: v.to("cpu", non_blocking=True) for k, v in tensors.items()}
            host_lists = {k: [x.to("cpu", non_blocking=True) for x in v] for k, v in lists.items()}
            event = torch.cuda.Event()
            event.record(torch.cuda.current_stream(device))
        else:
            host, event = {k: v.cpu() for k, v in tensors.items()}, None
            host_lists = {k: [x.cpu() for x in v] for k, v in lists.items()}
        if pending is not None:
            finish(pending)  # batch i-1 is written while batch i runs
        pending = (host, host_lists, names, event)
    if pending is not None:
        finish(pending)
    writer.close()
    return output_file if output_file is not None else writer
