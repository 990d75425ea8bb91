"""Row-band data parallelism (libbicos_amd/distributed.py) on CPU with gloo.

Each rank matches its band (the CPU oracle stands in for the GPU engine here; the
orchestration under test is identical), the bands are gathered to rank 0, and the
result must be byte-identical to a single whole-frame match.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from libbicos_amd.distributed import band_height, band_rows, gather_bands, match_sharded


def test_band_partition():
    for H in (1, 7, 96, 1536, 2160):
        for world in (1, 2, 3, 4, 8):
            bands = [band_rows(H, world, r) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == H
            for (b0, e0), (b1, e1) in zip(bands, bands[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in bands]
            assert max(sizes) - min(sizes) <= 1
            assert max(sizes) == band_height(H, world)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, H, W, n, cfg, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from libbicos_amd.synthetic import stereo_stack
        from oracle import oracle as O
        b, e = band_rows(H, world, rank)
        L, R = stereo_stack(n, H, W, row_begin=b, row_end=e, dmin=2, drange=12)

        def compute_band(s0, s1, c):
            d, corr = O.match(s0.numpy(), s1.numpy(), O.OracleConfig(**c), nthreads=1)
            return torch.from_numpy(d), (torch.from_numpy(corr) if corr is not None else None)

        d, c = match_sharded(torch.from_numpy(L), torch.from_numpy(R), H, compute_band, cfg)
        if rank == 0:
            q.put((d.numpy(), None if c is None else c.numpy()))
        else:
            assert d is None and c is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cfg", [
    (2, dict(nxcorr_threshold=0.5, subpixel_step=0.1)),
    (3, dict(nxcorr_threshold=None, variant=1, max_lr_diff=1)),
])
def test_sharded_match_equals_whole_frame(world, cfg):
    from libbicos_amd.synthetic import stereo_stack
    from oracle import oracle as O
    O.build()
    H, W, n = 23, 96, 12
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, H, W, n, cfg, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    d, c = q.get(timeout=10)
    L, R = stereo_stack(n, H, W, dmin=2, drange=12)
    rd, rc = O.match(L, R, O.OracleConfig(**cfg))
    assert d.dtype == rd.dtype and np.array_equal(d.view(np.uint8), rd.view(np.uint8))
    if rc is not None:
        assert np.array_equal(c.view(np.uint8), rc.view(np.uint8))


def _gather_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        H, W = 10, 5
        b, e = band_rows(H, world, rank)
        band = torch.arange(b * W, e * W, dtype=torch.float32).reshape(e - b, W)
        full = gather_bands(band, H)
        if rank == 0:
            q.put(full.numpy())
    finally:
        dist.destroy_process_group()


def test_gather_ragged_bands():
    world = 4  # 10 rows over 4 ranks: bands of 3, 3, 2, 2 rows (padded to 3 for the gather)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    full = q.get(timeout=10)
    assert np.array_equal(full, np.arange(50, dtype=np.float32).reshape(10, 5))
