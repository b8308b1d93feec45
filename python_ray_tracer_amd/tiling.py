"""Interleaved row tiling of a frame across ranks (the multi-GPU split of SURVEY.md §8e).

Rows are cut in blocks of ``row_block``; block b belongs to part ``b % n_parts``. Interleaving
balances the load: sky rows (no hit, ~15 flops/pixel) and ground rows (thousands) alternate
across ranks instead of landing on one rank as contiguous strips would. Local row ``lr`` of part
``p`` is global row ``((lr // rb) * P + p) * rb + lr % rb`` — the mapping the kernel uses
(``global_row`` in rtx_kernels.hip).
"""

from __future__ import annotations

import numpy as np


def n_local_rows(height: int, row_block: int, n_parts: int, part: int) -> int:
    if row_block <= 0 or n_parts <= 0 or not 0 <= part < n_parts:
        raise ValueError(f"bad tiling: row_block={row_block} n_parts={n_parts} part={part}")
    cycle = row_block * n_parts
    q, rem = divmod(int(height), cycle)
    return q * row_block + min(max(rem - part * row_block, 0), row_block)


def tile_rows(height: int, row_block: int, n_parts: int, part: int) -> np.ndarray:
    """Global row index of each local row of ``part`` (ascending)."""
    n = n_local_rows(height, row_block, n_parts, part)
    lr = np.arange(n)
    return ((lr // row_block) * n_parts + part) * row_block + lr % row_block


def max_local_rows(height: int, row_block: int, n_parts: int) -> int:
    return max(n_local_rows(height, row_block, n_parts, p) for p in range(n_parts))


def assemble(tiles, height: int, width: int, row_block: int, layout: str = "soa"):
    """Un-permute gathered tiles into one frame.

    ``tiles[p]`` is part p's tile padded to the same row count: ``[C, rows_max*W]`` (layout "soa",
    colour planes) or ``[rows_max, W, 3]`` (layout "hwc", uint8 pixels). Works on torch tensors
    (device-side index copy) and on NumPy arrays."""
    import torch

    n_parts = len(tiles)
    first = tiles[0]
    is_torch = isinstance(first, torch.Tensor)
    if layout == "soa":
        C = first.shape[0]
        full = (torch.empty((C, height, width), dtype=first.dtype, device=first.device) if is_torch
                else np.empty((C, height, width), dtype=first.dtype))
    else:
        full = (torch.empty((height, width, 3), dtype=first.dtype, device=first.device) if is_torch
                else np.empty((height, width, 3), dtype=first.dtype))
    for p, t in enumerate(tiles):
        rows = tile_rows(height, row_block, n_parts, p)
        k = len(rows)
        if k == 0:
            continue
        idx = torch.as_tensor(rows, device=first.device) if is_torch else rows
        if layout == "soa":
            src = t.reshape(t.shape[0], -1, width)[:, :k]
            full[:, idx] = src
        else:
            full[idx] = t[:k]
    if layout == "soa":
        return full.reshape(full.shape[0], height * width)
    return full
