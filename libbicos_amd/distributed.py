"""Row-band data parallelism for one BICOS match across the GPUs of a node.

Every stage of the reference is row-local (transform per pixel; the search scans
only the same row, bicos.hpp:91-94; agree/subpixel read row `row` only,
agree.hpp:83,154-156), so a frame splits into G contiguous row bands with no
halo. Each rank (one process per GPU, torch.distributed over RCCL) matches its
band independently; the only exchange is ONE gather of the disparity and
correlation bands to the root rank (RCCL send/recv under dist.gather, over xGMI).
The result is byte-identical to the single-GPU match.

`compute_band` is injectable so the orchestration (partition, padding, gather,
reassembly) is testable on CPU with the gloo backend; the production path
passes libbicos_amd.device.Engine.match.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def band_rows(H: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous band [begin, end) of rank `rank`; bands differ by at most one row
    (the first H % world ranks get one extra row)."""
    base, extra = divmod(H, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def band_height(H: int, world: int) -> int:
    """Padded band height used for the gather (max band)."""
    return -(-H // world)


def gather_bands(band: torch.Tensor, H: int, group=None, dst: int = 0) -> Optional[torch.Tensor]:
    """Gather equally padded row bands [h_b, W] to `dst`; returns the [H, W] frame on
    `dst` and None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    hb = band_height(H, world)
    b, e = band_rows(H, world, rank)
    if band.shape[0] != e - b:
        raise ValueError("band has %d rows, expected %d" % (band.shape[0], e - b))
    if band.shape[0] != hb:
        pad = torch.zeros((hb,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
        pad[: band.shape[0]] = band
        band = pad
    else:
        band = band.contiguous()
    # collectives do not all take int16 (neither gloo nor RCCL): move raw bytes
    dtype = band.dtype
    raw = band.reshape(hb, -1).view(torch.uint8)
    parts: Optional[List[torch.Tensor]] = None
    if rank == dst:
        parts = [torch.empty_like(raw) for _ in range(world)]
    dist.gather(raw, parts, dst=dst, group=group)
    if rank != dst:
        return None
    rows = []
    for r in range(world):
        rb, re = band_rows(H, world, r)
        rows.append(parts[r][: re - rb].view(dtype).reshape((re - rb,) + tuple(band.shape[1:])))
    return torch.cat(rows, dim=0)


def match_sharded(stack0_band: torch.Tensor, stack1_band: torch.Tensor, H: int,
                  compute_band: Callable, cfg=None, group=None, dst: int = 0,
                  gather_corrmap: bool = True):
    """Match this rank's row band and gather the full maps to `dst`.

    compute_band(stack0_band, stack1_band, cfg) -> (disparity_band, corrmap_band|None)
    Returns (disparity, corrmap) on `dst`, (None, None) elsewhere."""
    disp, corr = compute_band(stack0_band, stack1_band, cfg)
    full_d = gather_bands(disp, H, group, dst)
    full_c = gather_bands(corr, H, group, dst) if (gather_corrmap and corr is not None) else None
    return full_d, full_c
