"""HBM-resident batches: PyTorch is used only as the device allocator
(plumbing); the work is done by libdcr.so kernels on the context stream."""
from __future__ import annotations

import numpy as np

from .batch import BATCH_FIELDS, OUT_COLS, OUT_SCALARS, OutArrays, PackedBatch


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("no GPU visible to torch (HIP)")
    return torch


class DeviceBatch:
    """A PackedBatch copied to HBM plus device output buffers."""

    def __init__(self, packed: PackedBatch, device="cuda:0"):
        torch = _torch()
        self.packed = packed
        self.device = device
        self.t = {}
        for k in BATCH_FIELDS:
            a = getattr(packed, k)
            self.t[k] = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(device)
        self.out = {}
        for kind, n_rec, n_cols in (("ss", 4 * packed.n_fam, packed.ss_cols),
                                    ("ds", 2 * packed.n_fam, packed.ds_cols)):
            d = {}
            for k, dt in OUT_SCALARS.items():
                d[k] = torch.zeros(max(n_rec, 1) * np.dtype(dt).itemsize, dtype=torch.uint8, device=device)
            for k, dt in OUT_COLS.items():
                d[k] = torch.zeros(max(n_cols, 1) * np.dtype(dt).itemsize, dtype=torch.uint8, device=device)
            self.out[kind] = d
        self.batch_struct = packed.as_struct({k: v.data_ptr() for k, v in self.t.items()})
        self.ss_struct = OutArrays.__new__(OutArrays)
        from .batch import DcrOut
        self.ss_struct = DcrOut(**{k: v.data_ptr() for k, v in self.out["ss"].items()})
        self.ds_struct = DcrOut(**{k: v.data_ptr() for k, v in self.out["ds"].items()})

    def input_bytes(self):
        return sum(v.numel() for v in self.t.values())

    def download(self):
        """Copy device outputs into host OutArrays (after a sync)."""
        res = []
        for kind, n_rec, n_cols in (("ss", 4 * self.packed.n_fam, self.packed.ss_cols),
                                    ("ds", 2 * self.packed.n_fam, self.packed.ds_cols)):
            oa = OutArrays(n_rec, n_cols)
            for k, dt in list(OUT_SCALARS.items()) + list(OUT_COLS.items()):
                host = self.out[kind][k].cpu().numpy().view(dt)
                dst = getattr(oa, k)
                dst[:] = host[:len(dst)]
            res.append(oa)
        return res
