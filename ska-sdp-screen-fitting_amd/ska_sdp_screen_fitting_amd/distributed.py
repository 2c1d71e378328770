"""Antenna sharding of the KL path over one process per GPU.

Every (antenna, time, freq) slot is independent in both the fit and the
evaluation, so the antenna axis is split into contiguous
shards, one per rank, with no data-path collective.  The only exchanges are
one-shot setup collectives over RCCL (backend "nccl") or gloo (CPU tests):

* broadcast from rank 0 of the shared geometry: the reference-station index
  and position, the piercepoints (the KL basis is rebuilt from them on every
  GPU), the midpoint and the grid coordinates;
* all-reduce(MAX) of the station distances to the reference station (the
  order scaling normalises by the maximum over ALL stations,
  stationscreen.py:1011-1012);
* broadcast of the reference station's phases [T, F, D] so every shard can
  reference its phases (stationscreen.py:994-997) without holding station
  ``ref_ant``.
"""

import os

import numpy as np

from . import geometry


def shard_range(n_ant_total, world, rank):
    """Contiguous antenna block [a0, a1) of ``rank``."""
    base, extra = divmod(n_ant_total, world)
    a0 = rank * base + min(rank, extra)
    return a0, a0 + base + (1 if rank < extra else 0)


def setup_shard(local, ant_offset, n_ant_total, rad, dec, width_deg,
                cellsize_deg, order=None, min_order=5, max_ref=10, group=None,
                device="cpu"):
    """Collective setup of one antenna shard.

    ``local`` is a SolutionSet-like object holding this rank's stations
    (val/weight [T, F, A_local, D], ant_pos [A_local, 3], dir_radec [D, 2]).
    Returns a dict with the global reference station, the local initial
    orders, the piercepoints/midpoint, the grid coordinates and the
    reference phases.  Rank 0 must hold the first ``max_ref`` stations (the
    reference station is drawn from them, processing_utils.py:538-574).
    """
    import torch
    import torch.distributed as dist

    # collectives run whenever a process group exists (at world size 1 too,
    # so a one-GPU job can exercise the RCCL path)
    coll = dist.is_initialized()
    rank = dist.get_rank(group) if coll else 0
    T, F, A, D = local.val.shape
    if order is None:
        order = min(20, D - 1)

    # --- rank 0: reference station + geometry --------------------------------
    n_grid = geometry.grid_size(width_deg, cellsize_deg)
    hdr = torch.zeros(8 + 3 * D + 2 * n_grid, dtype=torch.float64)
    if rank == 0:
        if ant_offset != 0 or A < min(max_ref, n_ant_total):
            raise ValueError("rank 0 must hold the first stations")
        w = np.sum(local.weight[:, :, :min(max_ref, A), :], axis=(0, 1, 3),
                   dtype=np.float64)
        ref = int(np.nonzero(w == w.max())[0][0])
        pp, mid_ra, mid_dec = geometry.piercepoints(local.dir_radec)
        x, y = geometry.grid_coords(rad, dec, width_deg, cellsize_deg, mid_ra,
                                    mid_dec)
        refpos = np.asarray(local.ant_pos[ref], np.float32).astype(np.float64)
        hdr[0] = ref
        hdr[1:4] = torch.from_numpy(refpos)
        hdr[4], hdr[5] = mid_ra, mid_dec
        hdr[8:8 + 3 * D] = torch.from_numpy(pp.ravel())
        hdr[8 + 3 * D:8 + 3 * D + n_grid] = torch.from_numpy(x)
        hdr[8 + 3 * D + n_grid:] = torch.from_numpy(y)
    hdr = hdr.to(device)
    if coll:
        dist.broadcast(hdr, 0, group=group)
    hdr = hdr.cpu().numpy()
    ref = int(hdr[0])
    refpos = hdr[1:4].astype(np.float32)
    pp = hdr[8:8 + 3 * D].reshape(D, 3)
    x = hdr[8 + 3 * D:8 + 3 * D + n_grid]
    y = hdr[8 + 3 * D + n_grid:]

    # --- orders: distances in float32, max over all stations ----------------
    pos = np.asarray(local.ant_pos, np.float32)
    dd = pos - refpos
    dloc = np.sqrt(dd[:, 0] ** 2 + dd[:, 1] ** 2 + dd[:, 2] ** 2)
    dmax = torch.tensor([float(dloc.max())], dtype=torch.float64, device=device)
    if coll:
        dist.all_reduce(dmax, op=dist.ReduceOp.MAX, group=group)
    scale = np.float32(dmax.item())
    root = np.sqrt((dloc / scale).astype(np.float32))
    st_order = [max(min_order, min(order, int(float(order) * float(r)))) for r in root]

    # --- reference phases ----------------------------------------------------
    refph = torch.zeros((T, F, D), dtype=torch.float64)
    if rank == 0:
        refph = torch.from_numpy(np.ascontiguousarray(local.val[:, :, ref, :]))
    refph = refph.to(device)
    if coll:
        dist.broadcast(refph, 0, group=group)
    return dict(ref_ant=ref, st_order=st_order, piercepoints=pp,
                mid_ra=float(hdr[4]), mid_dec=float(hdr[5]), x=x, y=y,
                ref_phase=refph, ant_offset=ant_offset)


def device_identity(torch, device):
    """Which physical GPU a rank runs on: its torch index, PCI address and
    UUID (what ``rocm-smi`` / the kernel name the card by)."""
    p = torch.cuda.get_device_properties(device)
    return {"index": int(device.index if device.index is not None else 0),
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(getattr(p, "uuid", "")), "name": p.name,
            "visible": os.environ.get("HIP_VISIBLE_DEVICES",
                                      os.environ.get("CUDA_VISIBLE_DEVICES"))}


def gather_records(record, group=None):
    """Every rank's ``record`` (a JSON-able dict), in rank order, on every
    rank (all_gather_object; one call, outside any timed region)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return [record]
    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, record, group=group)
    return out


def check_distinct_devices(idents, backend):
    """Refuse a one-process-per-GPU job whose ranks share a card: under
    nccl (RCCL) every rank must resolve to its own PCI device.  gloo
    rehearsals may share one (their rates then mean nothing).  Raises
    RuntimeError naming the ranks that collide."""
    if backend != "nccl":
        return
    seen = {}
    for r, d in enumerate(idents):
        key = d.get("uuid") or d.get("pci")
        if key in seen:
            raise RuntimeError(f"ranks {seen[key]} and {r} resolve to the same GPU "
                               f"({d.get('pci')}, uuid {d.get('uuid')})")
        seen[key] = r
