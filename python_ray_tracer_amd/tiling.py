"""Interleaved row tiling of a frame across ranks (the multi-GPU split of SURVEY.md §8e).

Rows are cut in blocks of ``row_block``; block b belongs to part ``b % n_parts``. A rank may render
a run of consecutive parts (a larger or smaller share of the frame, ``runs``): part_run *
row_block consecutive rows of every cycle. Interleaving
balances the load: sky rows (no hit, ~15 flops/pixel) and ground rows (thousands) alternate
across ranks instead of landing on one rank as contiguous strips would. Local row ``lr`` of part
``p`` is global row ``((lr // rb) * P + p) * rb + lr % rb`` — the mapping the kernel uses
(``global_row`` in rtx_kernels.hip).

Gather layout: every part travels as one flat buffer of ``part_len`` elements (the same length on
every rank, as a collective needs), holding that part's tile exactly as ``render_tile`` returns
it — colour ``[3, rows_p*W]`` or uint8 ``[rows_p, W, 3]`` — at its start. ``assemble`` is the
host-side un-permute of such buffers (CPU tensors / NumPy); on the GPU the same layout is
un-permuted by ``rtx_assemble_rows``.
"""

from __future__ import annotations

import numpy as np


def n_local_rows(height: int, row_block: int, n_parts: int, part: int, run: int = 1) -> int:
    """Rows of the run of ``run`` consecutive parts from ``part``: run * row_block rows of every
    cycle of n_parts * row_block rows (the last cycle's prefix)."""
    if row_block <= 0 or n_parts <= 0 or run <= 0 or not 0 <= part <= n_parts - run:
        raise ValueError(f"bad tiling: row_block={row_block} n_parts={n_parts} part={part} run={run}")
    cycle, own = row_block * n_parts, row_block * run
    q, rem = divmod(int(height), cycle)
    return q * own + min(max(rem - part * row_block, 0), own)


def tile_rows(height: int, row_block: int, n_parts: int, part: int, run: int = 1) -> np.ndarray:
    """Global row index of each local row of the run of ``run`` parts from ``part`` (ascending)."""
    n = n_local_rows(height, row_block, n_parts, part, run)
    lr = np.arange(n)
    own = row_block * run
    return (lr // own) * (n_parts * row_block) + part * row_block + lr % own


def runs(world: int, root_run: int = 1, run: int = 1):
    """(n_parts, [(first part, run) per rank]) of the shares: rank 0 renders parts [0, root_run),
    rank i >= 1 parts [root_run + (i - 1) run, root_run + i run)."""
    n_parts = root_run + (world - 1) * run
    return n_parts, [(0, root_run)] + [(root_run + (i - 1) * run, run) for i in range(1, world)]


def max_local_rows(height: int, row_block: int, n_parts: int) -> int:
    return n_local_rows(height, row_block, n_parts, 0)  # part 0 has the most rows


def tile_shape(height: int, width: int, row_block: int, n_parts: int, part: int, out: str | None = None,
               run: int = 1):
    """Shape ``render_tile`` returns for this part (or run of parts): (3, rows*W) colour or
    (rows, W, 3) uint8."""
    rows = n_local_rows(height, row_block, n_parts, part, run)
    return (rows, int(width), 3) if out == "u8" else (3, rows * int(width))


def part_len(height: int, width: int, row_block: int, n_parts: int, itemsize: int, out: str | None = None,
             root_run: int = 1, run: int = 1) -> int:
    """Elements of one gather buffer: the largest rank's tile (``n_parts`` ranks, shares as in
    ``runs``), rounded up to 16 bytes (so every tile of a [ranks, part_len] buffer starts 16-byte
    aligned for the device copy)."""
    np_, shares = runs(n_parts, root_run, run)
    n = 3 * max(n_local_rows(height, row_block, np_, f, k) for f, k in shares) * int(width)
    per16 = max(1, 16 // itemsize)
    return (n + per16 - 1) // per16 * per16


def assemble(tiles, height: int, width: int, row_block: int, out: str | None = None, root_run: int = 1,
             run: int = 1):
    """Un-permute gathered rank buffers ``tiles[r]`` (each ``part_len`` long, layout above; shares
    as in ``runs``) into one frame: [3, H*W] colour or [H, W, 3] uint8 (``out="u8"``). Torch tensors
    or NumPy arrays."""
    import torch

    n_parts, shares = runs(len(tiles), root_run, run)
    first = tiles[0]
    is_torch = isinstance(first, torch.Tensor)
    shape = (height, width, 3) if out == "u8" else (3, height, width)
    full = (torch.empty(shape, dtype=first.dtype, device=first.device) if is_torch
            else np.empty(shape, dtype=first.dtype))
    for p, (f, k_run) in enumerate(shares):
        rows = tile_rows(height, row_block, n_parts, f, k_run)
        k = len(rows)
        if k == 0:
            continue
        idx = torch.as_tensor(rows, device=first.device) if is_torch else rows
        src = tiles[p][:3 * k * width]
        if out == "u8":
            full[idx] = src.reshape(k, width, 3)
        else:
            full[:, idx] = src.reshape(3, k, width)
    return full if out == "u8" else full.reshape(3, height * width)
